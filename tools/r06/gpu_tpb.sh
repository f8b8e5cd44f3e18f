# Round 6: multi-tile extend blocks with a proportionally larger LDS node
# cache (PT_EXTEND_TPB variant builds) -- parity of each variant, then a C3
# bench A/B against the in-tree build.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06_tpb}
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
for v in tpb2 tpb4; do
  PT_HIP_LIB=$R/build/variants/$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_path.py tests/test_gpu_parity.py -v -m gpu -x --timeout 300 --timeout-method thread -k "full_size or trace_rays or stack_formats or split_rounds or render_frame" > "$O/tests_$v.log" 2>&1
  rc=$?; echo "tests $v rc=$rc"; tail -2 "$O/tests_$v.log"; [ $rc -eq 0 ] || exit $rc
done
for v in base tpb2 tpb4 base tpb2 tpb4; do
  L="$R/path-tracer_amd/libpathtracer.so"; [ $v != base ] && L="$R/build/variants/$v.so"
  PT_HIP_LIB=$L timeout -k 10 300 python3 bench.py --config 3 --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-steady > "$O/b_$v.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 "$O/b_$v.log"; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['launch_avg_ms'])" "$O/b_$v.log" $v | tee -a "$O/ab.txt"
done
