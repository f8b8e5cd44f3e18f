# Round 6: class-pure shade block order -- parity tests, then bench A/B of
# orders 0 / 1 / 2 on C2 and C5, interleaved.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06_classorder}
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_bench_path.py -v -m gpu -x --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
for cfg in 2 5; do
  for ord in 0 1 2 0 1 2; do
    timeout -k 10 300 python3 bench.py --config $cfg --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-steady --class-order $ord > "$O/b_c${cfg}_o$ord.log" 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 "$O/b_c${cfg}_o$ord.log"; exit $rc; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c', sys.argv[2], 'order', sys.argv[3], d['value'], d['ms_per_step'], d['roofline']['launch_avg_ms'])" "$O/b_c${cfg}_o$ord.log" $cfg $ord | tee -a "$O/ab.txt"
  done
done
