# Round 6, first GPU call: new bench-path and gate tests, frame-end read-back cost.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06_first}
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
#timeout -k 10 700 python -u -m pytest tests/test_gpu_bench_path.py tests/test_gpu_gates.py -v -m gpu -x --timeout 400 --timeout-method thread > "$O/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/exp_frame_end.py 3 2 > "$O/frame_end_c3.json" 2> "$O/frame_end_c3.err"
rc=$?; echo "frame_end rc=$rc"; cat "$O/frame_end_c3.json"; [ $rc -eq 0 ] || { tail -5 "$O/frame_end_c3.err"; exit $rc; }
