# Round 6: guarded rounds without the guard kernel -- frame tests, then C1 /
# C2 / C3 bench lines.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06_guard}
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 700 python -u -m pytest tests/test_gpu_frame.py tests/test_gpu_bench_path.py tests/test_gpu_coverage.py -v -m gpu -x --timeout 400 --timeout-method thread > "$O/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
for cfg in 1 1 2 3; do
  timeout -k 10 300 python3 bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline --no-steady > "$O/b_c$cfg.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 "$O/b_c$cfg.log"; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c', sys.argv[2], d['value'], d['ms_per_step'], d['frame']['rounds_per_frame_rank0'][:2], d['roofline']['launch_avg_ms'])" "$O/b_c$cfg.log" $cfg | tee -a "$O/ab.txt"
done
