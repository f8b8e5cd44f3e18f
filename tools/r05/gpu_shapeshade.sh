# Per-shape lean-shade records (one load level for the material and its
# texture record): GPU tests, then C3 A/B against the previous build (prev.so).
set -e
O=gpurun_out/r05_shapeshade; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/r04/gpu_ab.sh r05_shapeshade_c3 3 3 prev base
