# Ray-reordering experiment (tools/exp_reorder.py) under rocprofv3 --kernel-trace.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/reorder
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d "$O/trace" -o run -- python3 $R/tools/exp_reorder.py ${ROUNDS:-30} > "$O/run.log" 2>&1
rc=$?; echo "run rc=$rc"; tail -5 "$O/run.log"; [ $rc -eq 0 ] || exit $rc
cd "$R" && python3 tools/exp_reorder_report.py "$O/trace" | tee "$O/report.txt"
