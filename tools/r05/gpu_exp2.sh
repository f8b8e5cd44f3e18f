# Class-list builds on one box: in-tree (lists in tile groups only), exp2
# (the same source with -DPT_EXP_CLASSQ=1: lists on single-stream rounds
# too) and classq1s (the experiment build the product path came from).
set -e
STEPS=3 bash tools/r04/gpu_ab.sh r05_exp2_c2 2 2 base exp2 classq1s
STEPS=2 bash tools/r04/gpu_ab.sh r05_exp2_c5 5 1 base exp2 classq1s
