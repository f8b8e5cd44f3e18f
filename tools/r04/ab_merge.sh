# A/B of the shade branch merges (build/variants: merge = both, mergeL = sky /
# cosine lobe only, mergeS = shape transforms only) against the in-tree library.
set -e
bash tools/r04/gpu_ab.sh r04_merge2_c3 3 3 base merge mergeL mergeS
bash tools/r04/gpu_ab.sh r04_merge2_c2 2 1 base merge mergeL mergeS
