# Extend-kernel occupancy sweep on C3: parity tests once, then one bench per variant.
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -le 1 ] || exit $rc
for v in ${VARIANTS:-0 1 2 3}; do
  PT_EXTEND_VARIANT=$v timeout -k 10 300 python bench.py --steps 32 --warmup 4 --no-cpu-baseline > gpurun_out/bench_v$v.log 2>&1; rc=$?; echo "v$v rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.loads(open('gpurun_out/bench_v$v.log').read().strip().splitlines()[-1]);print('v$v',d['value'],d['roofline']['launch_avg_ms'])"
done
