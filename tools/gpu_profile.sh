# Profiles bench.py (C3, N=1) on the GPU box:
#   1. rocprofv3 --kernel-trace --stats  -> kernel_stats.csv
#   2. separate --pmc passes (FETCH_SIZE | WRITE_SIZE | SQ | TCC hit/miss)
#   3. pmc_summary.json (HBM bytes per launch, corrected per MI355X_MICROARCH.md)
#   4. the default bench line (with cpu_baseline) -> bench.json
# usage: bash tools/gpu_profile.sh TAG
set -u
TAG=${1:-current}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
# the driver's exact bench command (BENCH_rNN.json "cmd")
B="$R/bench.py --gpus 1 --steps 20 --warmup 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$O/trace" -o run -- python3 $B > "$O/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE" "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 5 180 rocprofv3 --pmc $P --output-format csv -d "$O/pmc$i" -o run -- python3 $R/bench.py --steps 4 --warmup 1 --no-cpu-baseline > "$O/pmc$i.log" 2>&1
  rc=$?; echo "pmc$i ($P) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 $R/profiles/pmc_summary.py "$O/pmc_summary.json" $(find "$O" -name "*counter_collection.csv") > "$O/pmc_summary.txt"
cp $(find "$O/trace" -name "*kernel_stats.csv") "$O/kernel_stats.csv"
cd "$R"
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench.json.log" 2>&1; rc=$?; echo "bench rc=$rc"
tail -1 "$O/bench.json.log" > "$O/bench.json"
cat "$O/pmc_summary.txt"; cat "$O/bench.json"
python3 $R/profiles/timed_region.py $(find "$O/trace" -name "*kernel_trace.csv") 20 "$O/timed_region.json"
