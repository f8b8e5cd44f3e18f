# Occupancy floor of the diffuse shade instantiations (C3's lean one): 5 (in-tree) vs 6 / 4.
set -e
bash tools/r04/gpu_ab.sh r04_dminw_c3 3 3 base dminw6 dminw4
