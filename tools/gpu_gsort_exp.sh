# Global-sort key / stale-LPT experiment (tools/exp_gsort.py) under rocprofv3 --kernel-trace.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/gsort_exp
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d "$O/trace" -o run -- python3 $R/tools/exp_gsort.py > "$O/run.log" 2>&1
rc=$?; echo "run rc=$rc"; tail -3 "$O/run.log"; [ $rc -eq 0 ] || exit $rc
cd "$R" && python3 tools/exp_reorder_report.py "$O/trace" > "$O/report.txt"; cat "$O/report.txt"
