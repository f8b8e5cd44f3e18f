# LDS node cache size under tile groups (three concurrent streams): 96 / 256
# / 384 child pairs against the in-tree 160 (C3, interleaved, two rounds).
set -e
bash tools/r04/gpu_ab.sh r05_ncsplit_c3 3 2 base nc96 nc256 nc384
