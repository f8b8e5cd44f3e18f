# Round 6: class-list renderers in slot order -- parity tests (in-tree
# build), then bench A/B against the octant-order variant build on C2 / C5.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06_slotorder}
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_bench_path.py tests/test_gpu_resume.py -v -m gpu -x --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
for cfg in 2 5; do
  for v in base octant base octant; do
    L="$R/path-tracer_amd/libpathtracer.so"; [ $v != base ] && L="$R/build/variants/$v.so"
    PT_HIP_LIB=$L timeout -k 10 300 python3 bench.py --config $cfg --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-steady > "$O/b_c${cfg}_$v.log" 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 "$O/b_c${cfg}_$v.log"; exit $rc; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c', sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], d['roofline']['launch_avg_ms'])" "$O/b_c${cfg}_$v.log" $cfg $v | tee -a "$O/ab.txt"
  done
done
