# Shade traffic attribution: per variant of tools/exp_shade_traffic.py, one
# --pmc pass each for FETCH_SIZE, WRITE_SIZE and the L2->fabric read request
# sizes, then pmc_summary.py per variant.
# usage: bash tools/gpu_shade_attr.sh [VARIANTS...]
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/shade_attr
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
VARS=${*:-base notex noaccum notex_noaccum}
for v in $VARS; do
  i=0; mkdir -p "$O/$v"
  for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$O/$v/pmc$i" -o run -- python3 $R/tools/exp_shade_traffic.py $v --steps 4 > "$O/$v/pmc$i.log" 2>&1
    rc=$?; echo "$v pmc$i ($P) rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python3 $R/profiles/pmc_summary.py "$O/$v/pmc_summary.json" $(find "$O/$v" -name "*counter_collection.csv") > "$O/$v/pmc_summary.txt"
  grep shade "$O/$v/pmc_summary.txt"
done
