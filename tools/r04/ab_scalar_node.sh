# Scalar child-pair loads for wave-uniform internal steps (in-tree "base")
# against vector loads only (build/variants/nosn.so), then the GPU tests.
set -e
bash tools/r04/gpu_ab.sh r04_sn_c3 3 3 nosn base
STEPS=1 ARGS="--spp 1024" bash tools/r04/gpu_ab.sh r04_sn_c5 5 1 nosn base
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_sn_tests.log 2>&1 || { tail -30 gpurun_out/r04_sn_tests.log; exit 1; }
tail -2 gpurun_out/r04_sn_tests.log
