# PMC passes (tools/r04/gpu_pmc.sh) over steady-state rounds of the round-5
# build: C1 (batches), C2, C5, C4 whole frame on one GPU, C4 rank 0 of 8 with
# two path streams (C3: profiles/r05_pmc/c3).
set -e
P="python3 $PWD/tools/run_rounds.py"
bash tools/r04/gpu_pmc.sh r05_pmc/c1 $P --config 1 --fused 1 --batch 16 --settle 8 --rounds 64
bash tools/r04/gpu_pmc.sh r05_pmc/c2 $P --config 2 --settle 34 --rounds 32
bash tools/r04/gpu_pmc.sh r05_pmc/c5 $P --config 5 --settle 34 --rounds 32
bash tools/r04/gpu_pmc.sh r05_pmc/c4 $P --config 4 --settle 16 --rounds 16
bash tools/r04/gpu_pmc.sh r05_pmc/c4_bands8x2 $P --config 4 --rank 0 --nranks 8 --streams 2 --settle 34 --rounds 32
