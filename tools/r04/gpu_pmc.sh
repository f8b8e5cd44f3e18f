# Separate rocprofv3 --pmc passes (MI355X_MICROARCH.md: one block's slots per
# pass) over one command, then the per-kernel summary (profiles/pmc_summary.py).
# usage: bash tools/r04/gpu_pmc.sh TAG python3 SCRIPT ARGS...
O=$PWD/gpurun_out/$1; shift; mkdir -p $O; export TMPDIR=/tmp
i=0
while read -r P; do
  [ -z "$P" ] && continue
  i=$((i+1))
  (cd /tmp && timeout -s KILL 180 rocprofv3 --pmc $P --output-format csv -d $O/pmc_$i -o run -- "$@" > $O/pmc_$i.log 2>&1)
  rc=$?; echo "pmc pass $i ($P) rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/pmc_$i.log; exit $rc; }
done <<'PASSES'
FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
TCC_HIT_sum TCC_MISS_sum
SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE
TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE
PASSES
python3 $GRAFT_REPO_ROOT/profiles/pmc_summary.py $O/pmc_summary.json $(find $O -name "*counter_collection.csv") > $O/pmc_summary.txt
grep -E "^(extend|shade|round|rounds) " $O/pmc_summary.txt | cut -c1-400
