# Occupancy floor of the non-diffuse shade instantiations: 5 (in-tree) vs 4 / 6.
set -e
STEPS=1 ARGS="--spp 1024" bash tools/r04/gpu_ab.sh r04_minw_c5 5 2 base minw4 minw6
bash tools/r04/gpu_ab.sh r04_minw_c2 2 2 base minw4 minw6
