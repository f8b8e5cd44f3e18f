# Kernel trace of a short C3 bench with the extend cap off / on (A/B of
# the per-kernel durations).  usage: gpu_trace_ab.sh TAG CFG CAP...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; CFG=$2; shift 2
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
for cap in "$@"; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$O/trace_cap$cap" -o run -- python3 "$R/bench.py" --config $CFG --steps 2 --warmup 1 --no-cpu-baseline --no-steady --extend-cap $cap ${TRACE_ARGS:-} > "$O/trace_cap$cap.log" 2>&1)
  rc=$?; echo "trace cap $cap rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$O/trace_cap$cap.log"; exit $rc; }
  f=$(find "$O/trace_cap$cap" -name '*kernel_stats.csv' | head -1)
  cp "$f" "$O/kernel_stats_cap$cap.csv"
  cut -d, -f1-8 "$O/kernel_stats_cap$cap.csv" | head -8
  find "$O/trace_cap$cap" -name '*kernel_trace.csv' -exec gzip {} \;
done
