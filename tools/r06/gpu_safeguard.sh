# Round 6: the guarded end starts with a batch of the rounds that cannot
# overshoot -- frame tests, then same-box A/B against the previous build.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06_safeguard}
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 700 python -u -m pytest tests/test_gpu_frame.py -v -m gpu -x --timeout 400 --timeout-method thread > "$O/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
bash tools/r06/gpu_ab_lib.sh ${1:-r06_safeguard} "1 3 2" base head
