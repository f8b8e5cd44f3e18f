# Same-box A/B of the in-tree library against variant builds: bench lines
# interleaved.  usage: gpu_ab_lib.sh TAG "CFGS" VARIANT... (base = in-tree)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; CFGS=$2; shift 2
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
for rep in 1 2; do
  for cfg in $CFGS; do
    for v in "$@"; do
      L="$R/path-tracer_amd/libpathtracer.so"; [ $v != base ] && L="$R/build/variants/$v.so"
      PT_HIP_LIB=$L timeout -k 10 300 python3 bench.py --config $cfg --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-steady > "$O/b_c${cfg}_$v.log" 2>&1
      rc=$?; [ $rc -eq 0 ] || { tail -5 "$O/b_c${cfg}_$v.log"; exit $rc; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c', sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], d['roofline']['launch_avg_ms'])" "$O/b_c${cfg}_$v.log" $cfg $v | tee -a "$O/ab.txt"
    done
  done
done
