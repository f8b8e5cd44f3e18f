# Kernel trace of tools/gs_timing.py (40 rounds of C3) for env variants.
# usage: bash tools/gs_trace.sh TAG [VAR=VALUE ...]
set -u
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/gs_$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
env "$@" timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/tr" -o run -- python3 "$R/tools/gs_timing.py" > "$O/run.log" 2>&1
rc=$?; echo "$TAG rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$O/run.log"; exit $rc; }
tail -3 "$O/run.log" | cut -c1-120
cut -d, -f1-4 "$(find "$O/tr" -name '*kernel_stats.csv' | head -1)" | head -12
