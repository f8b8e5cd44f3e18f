# Tile groups started a launch apart at each batch (-DPT_SPLIT_STAGGER=1)
# against the in-tree build (all groups start together).
set -e
bash tools/r04/gpu_ab.sh r05_stagger_c3 3 2 base stagger
STEPS=3 bash tools/r04/gpu_ab.sh r05_stagger_c2 2 1 base stagger
STEPS=2 bash tools/r04/gpu_ab.sh r05_stagger_c5 5 1 base stagger
