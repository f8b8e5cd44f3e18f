# Ray-order experiments (tools/exp_gsort.py, tools/exp_bincost.py) under rocprofv3 --kernel-trace.
# usage: bash tools/gpu_gsort_exp.sh [SCRIPT_NAME]   (default exp_gsort)
set -u
R=$GRAFT_REPO_ROOT
E=${1:-exp_gsort}
O=$R/gpurun_out/$E
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d "$O/trace" -o run -- python3 $R/tools/$E.py > "$O/run.log" 2>&1
rc=$?; echo "run rc=$rc"; tail -3 "$O/run.log"; [ $rc -eq 0 ] || exit $rc
cd "$R" && python3 tools/exp_reorder_report.py "$O/trace" > "$O/report.txt"; cat "$O/report.txt"
