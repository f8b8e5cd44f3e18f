# Round 6: two more compiler-flag variants of the whole library (-O2; no
# post-RA machine scheduler) -- parity subset on each, then same-box A/B.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06_flags}
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
for v in o2 nopostsched; do
  PT_HIP_LIB=$R/build/variants/$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_path.py -v -m gpu -x --timeout 300 --timeout-method thread > "$O/tests_$v.log" 2>&1
  rc=$?; echo "tests $v rc=$rc"; tail -1 "$O/tests_$v.log"; [ $rc -eq 0 ] || exit $rc
done
bash tools/r06/gpu_ab_lib.sh ${1:-r06_flags} "3 5" base o2 nopostsched
