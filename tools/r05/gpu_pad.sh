# Kernel-argument layout: dslots padded as in the class-list experiment build
# (build/variants/pad.so) against the in-tree build, C2 / C5 / C3.
set -e
STEPS=3 bash tools/r04/gpu_ab.sh r05_pad_c2 2 2 base pad classq1s
STEPS=2 bash tools/r04/gpu_ab.sh r05_pad_c5 5 2 base pad classq1s
bash tools/r04/gpu_ab.sh r05_pad_c3 3 1 base pad
