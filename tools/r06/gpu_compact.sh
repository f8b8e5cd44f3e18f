# Round 6: compaction across launches -- parity tests, then bench A/B of the
# extend cap (1 = off, 0 = automatic 32, others) on C3 and C2.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06_compact}
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_bench_path.py -v -m gpu -x --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
for cfg in 3 2; do
  for cap in 1 0 24 40 1 0; do
    timeout -k 10 200 python3 bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline --no-steady --extend-cap $cap > "$O/b_c${cfg}_cap$cap.log" 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 "$O/b_c${cfg}_cap$cap.log"; exit $rc; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c', sys.argv[2], 'cap', sys.argv[3], d['value'], d['ms_per_step'], d['roofline']['launch_avg_ms'], d['config']['extend_cap'])" "$O/b_c${cfg}_cap$cap.log" $cfg $cap | tee -a "$O/ab.txt"
  done
done
