# Round 6: Run(R) as one round batch on fused renderers -- the tests that
# cover fused Run(2) against the oracle, then a C1 A/B.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06_runbatch}
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frame.py tests/test_gpu_resume.py tests/test_gpu_coverage.py -v -m gpu -x --timeout 400 --timeout-method thread > "$O/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
bash tools/r06/gpu_ab_lib.sh ${1:-r06_runbatch} "1" base head
