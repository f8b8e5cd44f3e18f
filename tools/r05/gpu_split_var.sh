# Tile-group variants (build/variants): contiguous tile runs per group
# (-DPT_SPLIT_CONTIG=1) and group streams at the lowest / highest priority
# (-DPT_SPLIT_PRIO=1/2), against the in-tree build (interleaved tiles, default
# priority).
set -e
bash tools/r04/gpu_ab.sh r05_splitvar_c3 3 2 base contig prio_low prio_high
STEPS=3 bash tools/r04/gpu_ab.sh r05_splitvar_c2 2 1 base contig prio_low prio_high
STEPS=2 bash tools/r04/gpu_ab.sh r05_splitvar_c5 5 1 base contig prio_low prio_high
