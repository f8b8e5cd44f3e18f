# All GPU tests + one C3 bench line (no CPU baseline).
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 64 --warmup 4 --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1; rc=$?; echo "bench rc=$rc"
tail -1 gpurun_out/bench_quick.log
