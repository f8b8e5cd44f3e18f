# One parameterised GPU-box script (replaces the round-2 per-experiment
# gpu_*.sh copies).  Runs the named steps in order, each under its own time
# limit, stopping at the first failure; output under gpurun_out/TAG/.
#
# usage: bash tools/gpu.sh TAG STEP [STEP ...]
#   tests[=PYTEST_K]   all -m gpu tests (or those matching -k PYTEST_K)
#   bench[=N]          the driver's bench command N times (default 1), no CPU baseline
#   benchcpu           the driver's bench command once, with the CPU baseline
#   trace              rocprofv3 --kernel-trace --stats of the driver's bench command
#   pmc                separate --pmc passes over a short bench (HBM bytes, VALU issue)
#   cfg=K              later bench / trace / pmc steps use --config K
#   args=A,B,..        extra bench.py arguments for later steps (commas -> spaces)
#   env=NAME=V[,..]    environment for later steps (A/B variants)
#   ab=NAME=V1/V2[/..] the bench step once per value of NAME (env A/B on one box)
#   smoke              __graft_entry__.smoke()
#   flow               bench.py --gpus 2 --one-gpu-flow-check (self-launched ranks on one GPU; RCCL refuses
#                      two ranks on one device, so the exchange takes the gloo fallback), both shards
set -u
TAG=${1:?tag}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
CFG=3
EXTRA=""
export TMPDIR=/tmp
BENCH_ARGS() { echo "--gpus 1 --steps 20 --warmup 5 --config $CFG $EXTRA"; }
fail() { echo "step $1 rc=$2"; exit "$2"; }
for S in "$@"; do
  case "$S" in
    cfg=*) CFG=${S#cfg=} ;;
    args=*) EXTRA=$(echo "${S#args=}" | tr ',' ' ') ;;
    env=*) for kv in $(echo "${S#env=}" | tr ',' ' '); do export "$kv"; echo "env $kv"; done ;;
    tests|tests=*)
      K=""; [ "$S" != tests ] && K="-k ${S#tests=}"
      (cd "$R" && timeout -k 10 1100 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread $K > "$O/gpu_tests.log" 2>&1)
      rc=$?; echo "tests rc=$rc"; tail -3 "$O/gpu_tests.log"; [ $rc -le 1 ] || fail tests $rc; [ $rc -eq 0 ] || exit $rc ;;
    bench|bench=*)
      N=1; [ "$S" != bench ] && N=${S#bench=}
      for i in $(seq 1 "$N"); do
        (cd "$R" && timeout -k 10 400 python3 bench.py $(BENCH_ARGS) --no-cpu-baseline > "$O/bench_c${CFG}_$i.log" 2>&1)
        rc=$?; [ $rc -eq 0 ] || { tail -5 "$O/bench_c${CFG}_$i.log"; fail bench $rc; }
        tail -1 "$O/bench_c${CFG}_$i.log" > "$O/bench_c${CFG}_$i.json"
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', d['value'], d['ms_per_step'], d['roofline']['launch_avg_ms'], (d.get('steady_state') or {}).get('mrays_per_s_per_gpu'))" "$O/bench_c${CFG}_$i.json"
      done ;;
    ab=*)
      spec=${S#ab=}; NAME=${spec%%=*}; VALS=${spec#*=}
      for v in $(echo "$VALS" | tr '/' ' '); do
        (cd "$R" && env "$NAME=$v" timeout -k 10 400 python3 bench.py $(BENCH_ARGS) --no-cpu-baseline > "$O/ab_${NAME}_$v.log" 2>&1)
        rc=$?; [ $rc -eq 0 ] || { tail -5 "$O/ab_${NAME}_$v.log"; fail "ab $NAME=$v" $rc; }
        tail -1 "$O/ab_${NAME}_$v.log" > "$O/ab_${NAME}_$v.json"
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['launch_avg_ms'], (d.get('steady_state') or {}).get('mrays_per_s_per_gpu'))" "$O/ab_${NAME}_$v.json" "$NAME=$v"
      done ;;
    benchcpu)
      (cd "$R" && timeout -k 10 400 python3 bench.py $(BENCH_ARGS) > "$O/benchcpu_c$CFG.log" 2>&1)
      rc=$?; [ $rc -eq 0 ] || { tail -5 "$O/benchcpu_c$CFG.log"; fail benchcpu $rc; }
      tail -1 "$O/benchcpu_c$CFG.log" > "$O/benchcpu_c$CFG.json"; echo "benchcpu ok" ;;
    trace)
      (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$O/trace_c$CFG" -o run -- python3 "$R/bench.py" $(BENCH_ARGS) --no-cpu-baseline > "$O/trace_c$CFG.log" 2>&1)
      rc=$?; [ $rc -eq 0 ] || fail trace $rc
      cp "$(find "$O/trace_c$CFG" -name '*kernel_stats.csv' | head -1)" "$O/kernel_stats_c$CFG.csv"
      grep "^{\"metric\"" "$O/trace_c$CFG.log" | tail -1 > "$O/trace_bench_c$CFG.json"
      python3 "$R/profiles/timed_region.py" "$(find "$O/trace_c$CFG" -name '*kernel_trace.csv' | head -1)" "$O/trace_bench_c$CFG.json" "$O/timed_region_c$CFG.json" || true
      cut -d, -f1-8 "$O/kernel_stats_c$CFG.csv" | head -8 ;;
    pmc)
      i=0
      while read -r P; do
        [ -z "$P" ] && continue
        i=$((i+1))
        (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$O/pmc_c${CFG}_$i" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 --spp 256 --config $CFG $EXTRA --no-cpu-baseline --no-steady > "$O/pmc_c${CFG}_$i.log" 2>&1)
        rc=$?; echo "pmc pass $i ($P) rc=$rc"; [ $rc -eq 0 ] || fail pmc $rc
      done <<'PASSES'
FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
TCC_HIT_sum TCC_MISS_sum
SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE
TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE
TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE
PASSES
      python3 "$R/profiles/pmc_summary.py" "$O/pmc_summary_c$CFG.json" $(find "$O" -path "*pmc_c${CFG}_*" -name "*counter_collection.csv") > "$O/pmc_summary_c$CFG.txt"
      grep -E "^(extend|shade|round)" "$O/pmc_summary_c$CFG.txt" | cut -c1-300 ;;
    flow)
      for sh in samples bands; do
        (cd "$R" && timeout -k 10 400 python3 bench.py --gpus 2 --one-gpu-flow-check --steps 2 --warmup 1 --spp 64 --config $CFG --shard $sh --no-cpu-baseline --no-steady > "$O/flow_$sh.log" 2>&1)
        rc=$?; [ $rc -eq 0 ] || { tail -20 "$O/flow_$sh.log"; fail "flow $sh" $rc; }
        grep '^{"metric"' "$O/flow_$sh.log" | tail -1 > "$O/flow_$sh.json"
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('flow', sys.argv[2], d['n_gpus'], d['value'], d['config']['exchange'], d['config']['comm_ranks'], d['frame']['rounds_per_frame_rank0'])" "$O/flow_$sh.json" $sh
      done ;;
    smoke)
      (cd "$R" && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1)
      rc=$?; tail -2 "$O/smoke.log"; [ $rc -eq 0 ] || fail smoke $rc ;;
    *) echo "unknown step $S"; exit 2 ;;
  esac
done
echo "all steps ok"
