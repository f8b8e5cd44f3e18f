# PMC passes over unsplit C3 rounds with the extend cap off and at 32.
set -e
P="python3 $PWD/tools/run_rounds.py"
bash tools/r04/gpu_pmc.sh r06_pmc_cap/off $P --config 3 --settle 34 --rounds 8 --split 1 --extend-cap 1
bash tools/r04/gpu_pmc.sh r06_pmc_cap/s32 $P --config 3 --settle 34 --rounds 8 --split 1 --extend-cap 32
find gpurun_out/r06_pmc_cap -name "*.csv" -delete
find gpurun_out/r06_pmc_cap -name "*.db" -delete
