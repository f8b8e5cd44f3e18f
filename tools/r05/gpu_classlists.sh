# Class-pure shade for list-using renderers (tile groups and their single-stream rounds): the whole GPU suite,
# then bench A/B of --class-lists 0 (automatic: on for C2 / C5) against 1
# (off), interleaved, C2 and C5; C3 once (single material: unaffected).
set -e
O=gpurun_out/${TAG:-r05_classlists}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for c in 2 5; do
  for i in 1 2; do
    for m in 0 1; do
      timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --class-lists $m --no-cpu-baseline --no-steady > $O/ab_c${c}_cl${m}_$i.log 2>&1 || { tail -5 $O/ab_c${c}_cl${m}_$i.log; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['config']['class_lists'], d['roofline']['launch_avg_ms'])" $O/ab_c${c}_cl${m}_$i.log "C$c class_lists=$m"
    done
  done
done
