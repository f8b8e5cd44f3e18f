# Round 4's last build (after the sky pdf skip): smoke, the driver's bench
# command with the CPU baseline and under rocprofv3 --kernel-trace --stats,
# and C5 / C2 lines.
set -e
bash tools/gpu.sh r04_fin4 smoke benchcpu trace cfg=5 args=--steps,3,--warmup,1 bench cfg=2 args=--steps,5,--warmup,1 bench
