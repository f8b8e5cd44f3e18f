# Tile groups: bench.py A/B over K = 1..4 (interleaved) on C3 (x2), C2, C5
# and C4 (--spp 256), to pick the automatic K.
set -e
O=gpurun_out/r05_splitk; mkdir -p $O
run() {  # config reps extra-args
  for i in $(seq 1 $2); do
    for k in 1 2 3 4; do
      timeout -k 10 300 python bench.py --config $1 --steps ${STEPS:-3} --warmup 1 --split $k --no-cpu-baseline --no-steady $3 > $O/ab_c$1_k${k}_$i.log 2>&1 || { tail -5 $O/ab_c$1_k${k}_$i.log; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['launch_avg_ms'])" $O/ab_c$1_k${k}_$i.log "C$1 K=$k"
    done
  done
}
run 3 2 ""
run 2 1 ""
run 5 1 ""
STEPS=1 run 4 1 "--spp 256"
