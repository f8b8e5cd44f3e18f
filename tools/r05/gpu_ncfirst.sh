# Node cache read order: LDS first for every lane, global only for uncached
# lanes (build/variants/ncfirst.so) vs the in-tree build (two branches, the
# LDS reads waiting on the global loads).
set -e
bash tools/r04/gpu_ab.sh r05_ncfirst_c3 3 3 base ncfirst head
