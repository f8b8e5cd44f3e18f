# PMC passes (one rocprofv3 --pmc run per counter group; <= 2 TA / TCP counters
# per pass) over a short C3 bench; summary per kernel -> gpurun_out/pmc_$TAG/.
# usage: bash tools/gpu_pmc.sh TAG
set -u
TAG=${1:-current}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
i=0
while read -r P; do
  [ -z "$P" ] && continue
  i=$((i+1))
  timeout -k 5 180 rocprofv3 --pmc $P --output-format csv -d "$O/p$i" -o run -- python3 $R/bench.py --steps 4 --warmup 1 --no-cpu-baseline > "$O/p$i.log" 2>&1
  rc=$?; echo "pass $i ($P) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done <<'PASSES'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY
SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum
TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum
PASSES
python3 $R/profiles/pmc_summary.py "$O/pmc_summary.json" $(find "$O" -name "*counter_collection.csv") > "$O/pmc_summary.txt"
grep -E "^(extend|shade)" "$O/pmc_summary.txt"
