# A/B of an environment knob on C3: VAR=<name> VALUES="0 1 2 ..." -> parity + bench per value.
mkdir -p gpurun_out
for v in ${VALUES}; do
  export $VAR=$v
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/env_tests_$v.log 2>&1; rc=$?; echo "tests $VAR=$v rc=$rc: $(tail -1 gpurun_out/env_tests_$v.log)"
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python bench.py --steps 64 --warmup 4 --no-cpu-baseline > gpurun_out/env_bench_$v.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "bench $v rc=$rc"; exit $rc; }
  python -c "import json;d=json.loads(open('gpurun_out/env_bench_$v.log').read().strip().splitlines()[-1]);print('$VAR=$v',d['value'],d['roofline']['launch_avg_ms'])"
done
