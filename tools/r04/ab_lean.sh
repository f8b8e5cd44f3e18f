# The lean diffuse-mesh shade instantiation + merged sky / cosine lobe and
# shape transforms (in-tree "base") against the previous commit's library
# (build/variants/head.so), then the GPU test suite.
set -e
bash tools/r04/gpu_ab.sh r04_lean_c3 3 3 head base
bash tools/r04/gpu_ab.sh r04_lean_c2 2 2 head base
STEPS=1 ARGS="--spp 1024" bash tools/r04/gpu_ab.sh r04_lean_c5 5 1 head base
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_lean_tests.log 2>&1 || { tail -30 gpurun_out/r04_lean_tests.log; exit 1; }
tail -3 gpurun_out/r04_lean_tests.log
