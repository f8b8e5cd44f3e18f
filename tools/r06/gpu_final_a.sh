# Round 6 final measurement, part 1: the whole GPU suite, smoke, the driver's
# bench command with the CPU baseline, then the CPU thread-scaling table on
# the same box (one shared timing path with the bench's CPU leg).
set -e
bash tools/gpu.sh r06_final tests smoke benchcpu
O=gpurun_out/r06_final
timeout -k 10 600 python3 tools/cpu_scaling.py $O/cpu_scaling.json > $O/cpu_scaling.log 2>&1
tail -c 600 $O/cpu_scaling.log
