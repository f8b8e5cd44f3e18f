# HBM bytes (FETCH_SIZE / WRITE_SIZE passes) of settled C2 / C5 rounds with
# class lists in slot order (in-tree) and octant order (variant build).
set -e
O=$PWD/gpurun_out/r06_pmc_slotorder; mkdir -p $O/c2_base $O/c2_octant $O/c5_base $O/c5_octant; export TMPDIR=/tmp
for cfg in 2 5; do
  for v in base octant; do
    L="$PWD/path-tracer_amd/libpathtracer.so"; [ $v != base ] && L="$PWD/build/variants/$v.so"
    i=0
    for P in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum"; do
      i=$((i+1))
      (cd /tmp && timeout -s KILL 180 rocprofv3 --pmc $P --output-format csv -d $O/c${cfg}_$v/pmc_$i -o run -- python3 $GRAFT_REPO_ROOT/tools/run_rounds.py --lib $L --config $cfg --settle 34 --rounds 16 > $O/c${cfg}_$v/pmc_$i.log 2>&1) || { echo "pass $i failed"; tail -5 $O/c${cfg}_$v/pmc_$i.log; exit 1; }
    done
    python3 $GRAFT_REPO_ROOT/profiles/pmc_summary.py $O/c${cfg}_$v/pmc_summary.json $(find $O/c${cfg}_$v -name "*counter_collection.csv") > $O/c${cfg}_$v/pmc_summary.txt
    echo "c$cfg $v"; grep -E "^(shade|extend|class_list|shade_classq) " $O/c${cfg}_$v/pmc_summary.txt | cut -c1-300
  done
done
find $O -name "*.csv" -delete; find $O -name "*.db" -delete
