# Round 4's closing measurement of the final build (after the lean texel wrap and the constant untextured sky
# ): smoke, the driver's bench command with the CPU baseline and under
# rocprofv3 --kernel-trace --stats, C2 / C5 (8192 spp) / C4 / C1 lines and
# the steady-state PMC passes of C3 (its shade changed).
set -e
bash tools/gpu.sh r04_fin3 smoke benchcpu trace cfg=2 args=--steps,5,--warmup,1 bench \
  cfg=5 args=--steps,3,--warmup,1 bench cfg=4 args=--steps,2,--warmup,1 bench cfg=1 args= bench
bash tools/r04/gpu_pmc.sh r04_fin3/pmc_c3 python3 $PWD/tools/run_rounds.py --config 3 --settle 34 --rounds 32
