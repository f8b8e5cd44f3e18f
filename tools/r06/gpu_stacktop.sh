# Round 6: BLAS stack top in a register (-DPT_STACK_TOP=1) -- parity tests on
# the variant, then same-box A/B against the in-tree build.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06_stacktop}
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
PT_HIP_LIB=$R/build/variants/stacktop.so timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_gates.py tests/test_gpu_bench_path.py tests/test_gpu_fuzz.py -v -m gpu -x --timeout 400 --timeout-method thread > "$O/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
bash tools/r06/gpu_ab_lib.sh ${1:-r06_stacktop} "3 5 2" base stacktop
