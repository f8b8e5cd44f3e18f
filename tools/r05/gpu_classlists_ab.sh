# Same box: the product class-list path (in-tree, automatic), the experiment
# build it came from (build/variants/classq1s.so) and the lists off.
set -e
O=gpurun_out/r05_classlists_ab; mkdir -p $O
for c in 2 5; do
  for i in 1 2; do
    for v in auto exp off; do
      L=$PWD/path-tracer_amd/libpathtracer.so; A=""
      [ $v = exp ] && L=$PWD/build/variants/classq1s.so
      [ $v = off ] && A="--class-lists 1"
      PT_HIP_LIB=$L timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 $A --no-cpu-baseline --no-steady > $O/ab_c${c}_${v}_$i.log 2>&1 || { tail -5 $O/ab_c${c}_${v}_$i.log; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['launch_avg_ms'])" $O/ab_c${c}_${v}_$i.log "C$c $v"
    done
  done
done
