# Octant re-sort of the new rays after each class-pure shade
# (-DPT_LIST_REORDER=1): C2 / C5 split tests on the variant (bit-exact), then
# C2 / C5 A/B against the in-tree build (no re-sort).
set -e
O=gpurun_out/r05_reorder; mkdir -p $O
PT_HIP_LIB=$PWD/build/variants/reorder.so timeout -k 10 500 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_frame.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
STEPS=3 bash tools/r04/gpu_ab.sh r05_reorder_c2 2 2 base reorder
STEPS=2 bash tools/r04/gpu_ab.sh r05_reorder_c5 5 2 base reorder
