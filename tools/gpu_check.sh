# GPU check of the current tree: all -m gpu tests, the driver's exact bench
# command three times, and a rocprofv3 kernel trace of that same command.
# usage: bash tools/gpu_check.sh TAG [pytest-args...]
set -u
TAG=${1:-check}; shift || true
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 1000 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread "$@" > "$O/gpu_tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$O/gpu_tests.log"
[ $rc -le 1 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$O/bench_$i.log" 2>&1
  rc=$?; echo "bench $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  tail -1 "$O/bench_$i.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['launch_avg_ms'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$O/trace" -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$O/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
cp $(find "$O/trace" -name "*kernel_stats.csv") "$O/kernel_stats.csv"
cat "$O/kernel_stats.csv" | cut -d, -f1-8 | head -12
