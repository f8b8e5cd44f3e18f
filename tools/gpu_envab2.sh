# A/B of environment settings on C3: SETTINGS="A=1:B=2 A=0 ..." (':' joins the
# variables of one arm; "base" = no extra variables) -> parity + bench per arm.
# Optional CONFIGS="3 5 2" benches every arm on each config.
mkdir -p gpurun_out
CONFIGS=${CONFIGS:-3}
for set in ${SETTINGS}; do
  vars=""
  [ "$set" = "base" ] || vars=$(echo "$set" | tr ':' ' ')
  tag=$(echo "$set" | tr ':=/' '_-_' | tail -c 60)
  timeout -k 10 300 env $vars python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/ab_tests_$tag.log 2>&1; rc=$?
  echo "tests [$set] rc=$rc: $(tail -1 gpurun_out/ab_tests_$tag.log)"
  [ $rc -eq 0 ] || exit $rc
  for c in $CONFIGS; do
    timeout -k 10 300 env $vars python bench.py --steps 64 --warmup 4 --no-cpu-baseline --config $c > gpurun_out/ab_bench_${tag}_c$c.log 2>&1; rc=$?
    [ $rc -eq 0 ] || { echo "bench [$set] c$c rc=$rc"; tail -5 gpurun_out/ab_bench_${tag}_c$c.log; exit $rc; }
    python -c "import json;d=json.loads(open('gpurun_out/ab_bench_${tag}_c$c.log').read().strip().splitlines()[-1]);print('[$set] c$c',d['value'],d['roofline']['launch_avg_ms'])"
  done
done
