# PMC passes (tools/r04/gpu_pmc.sh) over steady-state rounds of every config:
# C1 (fused rounds + 16-round batches), C2, C3, C5 (extend + shade), C4 whole
# frame on one GPU, and C4's rank 0 of 8 with two path streams.
set -e
P="python3 $PWD/tools/run_rounds.py"
bash tools/r04/gpu_pmc.sh r04_pmc/c1 $P --config 1 --fused 1 --batch 16 --settle 8 --rounds 64
bash tools/r04/gpu_pmc.sh r04_pmc/c2 $P --config 2 --settle 34 --rounds 32
bash tools/r04/gpu_pmc.sh r04_pmc/c3 $P --config 3 --settle 34 --rounds 32
bash tools/r04/gpu_pmc.sh r04_pmc/c5 $P --config 5 --settle 34 --rounds 32
bash tools/r04/gpu_pmc.sh r04_pmc/c4 $P --config 4 --settle 16 --rounds 16
bash tools/r04/gpu_pmc.sh r04_pmc/c4_bands8x2 $P --config 4 --rank 0 --nranks 8 --streams 2 --settle 34 --rounds 32
