# PMC of the class-list build on C2 and C5 (tile groups, class-pure shade):
# "shade" = class_list + shade_classq launches (profiles/pmc_summary.py).
set -e
P="python3 $PWD/tools/run_rounds.py"
bash tools/r04/gpu_pmc.sh r05_pmc3/c2 $P --config 2 --settle 34 --rounds 32
bash tools/r04/gpu_pmc.sh r05_pmc3/c5 $P --config 5 --settle 34 --rounds 32
find gpurun_out/r05_pmc3 -name "*.csv" -delete
find gpurun_out/r05_pmc3 -name "*.db" -delete
