# Under tile groups (three concurrent streams): shade occupancy floors and
# the tile-order re-sort period, against the in-tree build (5 waves, period 16).
set -e
bash tools/r04/gpu_ab.sh r05_splittune_c3 3 2 base dminw4 dminw6 period8 period32
STEPS=3 bash tools/r04/gpu_ab.sh r05_splittune_c2 2 1 base ominw4 ominw6 period8 period32
STEPS=2 bash tools/r04/gpu_ab.sh r05_splittune_c5 5 1 base ominw4 ominw6 period8 period32
