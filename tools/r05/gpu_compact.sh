# In-block ray compaction for extend (build/variants/compact*.so): the GPU
# tests on the compact build, then C3 A/B against the in-tree build (node cache).
set -e
O=gpurun_out/r05_compact; mkdir -p $O
PT_HIP_LIB=$PWD/build/variants/compact.so timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/r04/gpu_ab.sh r05_compact_c3 3 3 base compact compact7 compact8k
STEPS=2 bash tools/r04/gpu_ab.sh r05_compact_c5 5 1 base compact
STEPS=3 bash tools/r04/gpu_ab.sh r05_compact_c2 2 1 base compact
