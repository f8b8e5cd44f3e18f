# Round 6 final PMC passes (tools/r04/gpu_pmc.sh: one --pmc pass per counter
# group) over settled rounds of the final build with the bench's automatic
# schedule: C3 / C2 / C5 (three tile groups; class lists on C2 / C5), C1
# (fused round batches of 16), C4 whole frame and C4 rank 0 of 8 with two
# path streams.  Summaries carry each kernel's serialised dispatch time.
set -e
P="python3 $PWD/tools/run_rounds.py"
bash tools/r04/gpu_pmc.sh r06_pmc/c3 $P --config 3 --settle 34 --rounds 32
bash tools/r04/gpu_pmc.sh r06_pmc/c2 $P --config 2 --settle 34 --rounds 32
bash tools/r04/gpu_pmc.sh r06_pmc/c5 $P --config 5 --settle 34 --rounds 32
bash tools/r04/gpu_pmc.sh r06_pmc/c1 $P --config 1 --fused 1 --batch 16 --settle 8 --rounds 64
bash tools/r04/gpu_pmc.sh r06_pmc/c4 $P --config 4 --settle 16 --rounds 16
bash tools/r04/gpu_pmc.sh r06_pmc/c4_bands8x2 $P --config 4 --rank 0 --nranks 8 --streams 2 --settle 34 --rounds 32
find gpurun_out/r06_pmc -name "*.csv" -delete
find gpurun_out/r06_pmc -name "*.db" -delete
