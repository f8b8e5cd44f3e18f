# Round 6 final measurement, part 2: the driver's bench command with the CPU
# baseline (pinned before the oracle's first touch) and the CPU scaling table
# on the same box, the bench command under rocprofv3 --kernel-trace --stats,
# then every other config's line.
set -e
bash tools/gpu.sh r06_final2 benchcpu
O=gpurun_out/r06_final2
timeout -k 10 600 python3 tools/cpu_scaling.py $O/cpu_scaling.json > $O/cpu_scaling.log 2>&1
tail -c 300 $O/cpu_scaling.log
bash tools/gpu.sh r06_final2 trace cfg=5 args=--steps,3,--warmup,1 bench cfg=2 args=--steps,5,--warmup,1 bench cfg=1 args= bench cfg=4 args=--steps,1,--warmup,0,--no-steady bench
find $O -name "*kernel_trace.csv" -exec gzip -f {} \;
