# A/B of an environment switch on C3: parity tests + bench with each setting.
# usage: AB_VAR=NAME AB_VALUES="a b" bash tools/gpu_ab_env.sh
mkdir -p gpurun_out
for v in $AB_VALUES; do
  env $AB_VAR=$v timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/ab_tests_$v.log 2>&1; rc=$?; echo "tests $AB_VAR=$v rc=$rc: $(tail -1 gpurun_out/ab_tests_$v.log)"
  [ $rc -eq 0 ] || exit $rc
  env $AB_VAR=$v timeout -k 10 300 python bench.py --steps 64 --warmup 4 --no-cpu-baseline > gpurun_out/ab_bench_$v.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "bench rc=$rc"; exit $rc; }
  python -c "import json;d=json.loads(open('gpurun_out/ab_bench_$v.log').read().strip().splitlines()[-1]);print('$AB_VAR=$v',d['value'],d['roofline']['launch_avg_ms'])"
done
