# Round 6 final measurement, part 3 (after the frame-schedule changes): the
# whole GPU suite, smoke, the driver's bench command with the CPU baseline,
# the C1 / C2 / C5 lines.
set -e
bash tools/gpu.sh r06_final3 tests smoke benchcpu cfg=1 args= bench cfg=2 args=--steps,5,--warmup,1 bench cfg=5 args=--steps,3,--warmup,1 bench
