# In-block refill extend variants (PT_EXTEND_POOL) on C3: parity + one bench line each.
mkdir -p gpurun_out
for v in ${POOLS:-0 1 2 3 4 5 6}; do
  PT_EXTEND_POOL=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pool_tests_$v.log 2>&1; rc=$?; echo "tests pool=$v rc=$rc: $(tail -1 gpurun_out/pool_tests_$v.log)"
  [ $rc -eq 0 ] || exit $rc
  PT_EXTEND_POOL=$v timeout -k 10 300 python bench.py --steps 64 --warmup 4 --no-cpu-baseline > gpurun_out/pool_bench_$v.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "bench pool=$v rc=$rc"; exit $rc; }
  python -c "import json;d=json.loads(open('gpurun_out/pool_bench_$v.log').read().strip().splitlines()[-1]);print('pool=$v',d['value'],d['roofline']['launch_avg_ms'])"
done
