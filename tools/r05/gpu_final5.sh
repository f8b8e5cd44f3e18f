# Round-5 last build (tile groups, pinned CPU baseline, apportioned roofline, guarded frame end, class lists in tile groups): the whole GPU suite, smoke, the driver's
# bench command with the CPU baseline and under rocprofv3 --kernel-trace
# --stats, then every other config's line.
set -e
bash tools/gpu.sh r05_final5 tests smoke benchcpu trace cfg=5 args=--steps,3,--warmup,1 bench cfg=2 args=--steps,5,--warmup,1 bench cfg=1 args= bench cfg=4 args=--steps,1,--warmup,0,--no-steady bench
find gpurun_out/r05_final5 -name "*kernel_trace.csv" -delete
