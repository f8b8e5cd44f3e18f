# Tile-group count with class lists (C2, C5): --split 2 / 3 / 4 interleaved.
set -e
O=gpurun_out/r05_lists_k; mkdir -p $O
for c in 2 5; do
  for i in 1 2; do
    for k in 2 3 4; do
      timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --split $k --no-cpu-baseline --no-steady > $O/ab_c${c}_k${k}_$i.log 2>&1 || { tail -5 $O/ab_c${c}_k${k}_$i.log; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['config']['class_lists'], d['roofline']['launch_avg_ms'])" $O/ab_c${c}_k${k}_$i.log "C$c K=$k"
    done
  done
done
