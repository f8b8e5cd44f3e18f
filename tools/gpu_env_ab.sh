# A/B of an environment switch: parity tests with the candidate value, then
# bench on each config for each value, interleaved, twice.
# usage: VAR=NAME VALUES="0 1" TEST_VALUE=1 CONFIGS="3 5" bash tools/gpu_env_ab.sh
set -u
O=gpurun_out/env_ab_${VAR}; mkdir -p $O
env $VAR=${TEST_VALUE} timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_coverage.py -q -m gpu -x --timeout 120 --timeout-method thread -k "not two_process" > $O/tests.log 2>&1; rc=$?
echo "tests ($VAR=${TEST_VALUE}) rc=$rc: $(tail -1 $O/tests.log)"; [ $rc -eq 0 ] || { tail -30 $O/tests.log; exit $rc; }
for rep in 1 2; do for cfg in ${CONFIGS:-3 5}; do for v in $VALUES; do
  env $VAR=$v timeout -k 10 120 python bench.py --config $cfg --steps 64 --warmup 8 --no-cpu-baseline > $O/b_${cfg}_${v}_$rep.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -5 $O/b_${cfg}_${v}_$rep.log; exit $rc; }
  python -c "import json;d=json.loads(open('$O/b_${cfg}_${v}_$rep.log').read().strip().splitlines()[-1]);print('C$cfg $VAR=$v rep=$rep',d['value'],d['roofline']['launch_avg_ms'])"
done; done; done
