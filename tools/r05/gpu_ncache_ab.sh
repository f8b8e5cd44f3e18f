# LDS node cache (extend): C3 / C5 / C2 A/B against the grey-record build
# without it (build/variants/grey.so) and round 4 (head.so).
set -e
bash tools/r04/gpu_ab.sh r05_ncache_c3 3 3 grey base head
STEPS=2 bash tools/r04/gpu_ab.sh r05_ncache_c5 5 2 grey base
STEPS=3 bash tools/r04/gpu_ab.sh r05_ncache_c2 2 2 grey base
