# Two-select texel wrap in every instantiation but the general TEXWRAP one
# (in-tree "base") against the lean-only form (build/variants/head.so).
set -e
bash tools/r04/gpu_ab.sh r04_wrapall_c2 2 2 head base
STEPS=1 ARGS="--spp 1024" bash tools/r04/gpu_ab.sh r04_wrapall_c5 5 2 head base
bash tools/r04/gpu_ab.sh r04_wrapall_c3 3 2 head base
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_wrapall_tests.log 2>&1 || { tail -30 gpurun_out/r04_wrapall_tests.log; exit 1; }
tail -2 gpurun_out/r04_wrapall_tests.log
