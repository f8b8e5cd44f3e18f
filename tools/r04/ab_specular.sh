# Merged metal / translucent sampling (in-tree "base") against the previous
# commit's library (build/variants/head.so) on C5 and C2, the GPU test suite,
# then the per-rank work of sample shards at N = 2 / 4 / 8 (C3 frames at
# 1024 / N spp on one GPU, no exchange).
set -e
STEPS=1 ARGS="--spp 1024" bash tools/r04/gpu_ab.sh r04_spec_c5 5 2 head base
bash tools/r04/gpu_ab.sh r04_spec_c2 2 2 head base
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_spec_tests.log 2>&1 || { tail -30 gpurun_out/r04_spec_tests.log; exit 1; }
tail -2 gpurun_out/r04_spec_tests.log
O=gpurun_out/r04_shards; mkdir -p $O
for spp in 1024 512 256 128; do
  timeout -k 10 300 python bench.py --config 3 --spp $spp --steps 20 --warmup 5 --no-cpu-baseline --no-steady > $O/c3_spp$spp.log 2>&1 || { tail -5 $O/c3_spp$spp.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('spp', sys.argv[2], d['value'], d['ms_per_step'], d['frame'] if 'frame' in d else '')" $O/c3_spp$spp.log $spp
done
