# Round 6: full -m gpu suite, frame-end cost with the exact loop, step-count
# dumps for the compaction model.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06_validate}
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 400 --timeout-method thread > "$O/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/exp_frame_end.py 3 2 > "$O/frame_end_c3.json" 2> "$O/frame_end_c3.err"
rc=$?; echo "frame_end rc=$rc"; cat "$O/frame_end_c3.json"; [ $rc -eq 0 ] || { tail -5 "$O/frame_end_c3.err"; exit $rc; }
for c in 3 5 2; do
  timeout -k 10 120 python -u tools/exp_compact2.py dump "$O/steps_c$c.npz" $c 3 > "$O/dump_c$c.log" 2>&1
  rc=$?; echo "dump c$c rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$O/dump_c$c.log"; exit $rc; }
done
