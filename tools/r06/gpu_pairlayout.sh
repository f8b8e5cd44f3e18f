# Round 6: 64-byte-aligned depth-first BLAS pair layout -- parity tests with
# the in-tree build, then A/B against the previous layout.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06_pairlayout}
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_gates.py tests/test_gpu_bench_path.py -v -m gpu -x --timeout 400 --timeout-method thread > "$O/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
bash tools/r06/gpu_ab_lib.sh ${1:-r06_pairlayout} "3 5" base oldlayout
