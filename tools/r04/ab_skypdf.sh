# Sky pdf term dropped where the host proves it an exact +0 (in-tree "base")
# against the full expression (build/variants/head.so): C3 / C5, then the tests.
set -e
bash tools/r04/gpu_ab.sh r04_skypdf_c3 3 3 head base
STEPS=1 ARGS="--spp 1024" bash tools/r04/gpu_ab.sh r04_skypdf_c5 5 1 head base
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_skypdf_tests.log 2>&1 || { tail -30 gpurun_out/r04_skypdf_tests.log; exit 1; }
tail -2 gpurun_out/r04_skypdf_tests.log
