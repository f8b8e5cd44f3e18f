# Extend-kernel variant sweep on C3: GPU parity tests and one bench line per variant.
mkdir -p gpurun_out
for v in ${VARIANTS:-0 1 2 3 4}; do
  PT_EXTEND_VARIANT=$v timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/gpu_tests_v$v.log 2>&1; rc=$?; echo "tests v$v rc=$rc: $(tail -1 gpurun_out/gpu_tests_v$v.log)"
  [ $rc -eq 0 ] || exit $rc
  PT_EXTEND_VARIANT=$v timeout -k 10 300 python bench.py --steps 64 --warmup 4 --no-cpu-baseline > gpurun_out/bench_v$v.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "bench v$v rc=$rc"; exit $rc; }
  python -c "import json;d=json.loads(open('gpurun_out/bench_v$v.log').read().strip().splitlines()[-1]);print('v$v',d['value'],d['roofline']['launch_avg_ms'],'simd_eff',d['traversal']['simd_efficiency'])"
done
