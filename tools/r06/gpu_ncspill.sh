# Round 6: LDS node cache also for spilled u16 stacks (C5), and smaller LDS
# stacks traded for a bigger node cache (PT_EXTEND_CAP / PT_NODE_CACHE_PAIRS
# variants, spilling beyond the LDS rows) -- parity on every build, then a
# same-box A/B (prev = the tree before the change).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06_ncspill}
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_bench_path.py tests/test_gpu_gates.py -v -m gpu -x --timeout 400 --timeout-method thread > "$O/tests_base.log" 2>&1
rc=$?; echo "tests base rc=$rc"; tail -2 "$O/tests_base.log"; [ $rc -eq 0 ] || exit $rc
for v in cap12nc224 cap16nc192; do
  PT_HIP_LIB=$R/build/variants/$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_bench_path.py -v -m gpu -x --timeout 400 --timeout-method thread > "$O/tests_$v.log" 2>&1
  rc=$?; echo "tests $v rc=$rc"; tail -2 "$O/tests_$v.log"; [ $rc -eq 0 ] || exit $rc
done
bash tools/r06/gpu_ab_lib.sh ${1:-r06_ncspill} "5 3" base prev cap12nc224 cap16nc192
