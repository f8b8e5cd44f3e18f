# A/B of alternative libpathtracer.so builds (build/variants/NAME.so; "base" =
# the in-tree library) on one box: bench.py --config $CFG, interleaved $REP times.
# usage: bash tools/r04/gpu_ab.sh TAG CFG REP NAME...
O=gpurun_out/$1; CFG=$2; REP=$3; shift 3; mkdir -p $O
for i in $(seq 1 $REP); do
  for v in "$@"; do
    if [ "$v" = base ]; then L=path-tracer_amd/libpathtracer.so; else L=build/variants/$v.so; fi
    PT_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --config $CFG --steps ${STEPS:-3} --warmup 1 ${ARGS:-} --no-cpu-baseline --no-steady > $O/ab_${v}_$i.log 2>&1 || { tail -5 $O/ab_${v}_$i.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['launch_avg_ms'])" $O/ab_${v}_$i.log $v
  done
done
