# Tile groups on concurrent streams (ptSetBasicRendererSplit): the split
# tests, the whole GPU suite, then bench.py A/B with the automatic split
# (K = 2 on full frames) against --split 1, interleaved, C3 / C2 / C5.
set -e
O=gpurun_out/r05_split; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/split_tests.log 2>&1 || { tail -40 $O/split_tests.log; exit 1; }
tail -3 $O/split_tests.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for c in 3 2 5; do
  for i in 1 2; do
    for k in 0 1; do
      timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --split $k --no-cpu-baseline --no-steady > $O/ab_c${c}_split${k}_$i.log 2>&1 || { tail -5 $O/ab_c${c}_split${k}_$i.log; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['config']['split'], d['roofline']['launch_avg_ms'])" $O/ab_c${c}_split${k}_$i.log "C$c split=$k"
    done
  done
done
