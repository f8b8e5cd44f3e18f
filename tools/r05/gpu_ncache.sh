# LDS node cache (extend): the GPU tests, then C3 A/B against the grey-record
# build without it (build/variants/grey.so) and round 4 (head.so).
set -e
O=gpurun_out/r05_ncache; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/r04/gpu_ab.sh r05_ncache_c3 3 3 grey base head
STEPS=2 bash tools/r04/gpu_ab.sh r05_ncache_c5 5 1 grey base
STEPS=3 bash tools/r04/gpu_ab.sh r05_ncache_c2 2 1 grey base
