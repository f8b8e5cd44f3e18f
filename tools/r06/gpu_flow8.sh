# The 8-rank flow checks again on the round-6 build (exact frame end, resized class lists) (each rank's rounds in
# three tile groups on its own streams; every rank on device 0, so the
# exchange takes the gloo fallback).
set -e
O=gpurun_out/r06_flow8; mkdir -p $O
run() { name=$1; shift; timeout -k 10 400 python bench.py --gpus 8 --one-gpu-flow-check --no-cpu-baseline --no-steady "$@" > $O/$name.log 2>&1 || { tail -20 $O/$name.log; exit 1; }; grep '^{' $O/$name.log > $O/$name.json; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print(sys.argv[2], d['n_gpus'], d['value'], c['shard'], c['streams'], c['split'], c['exchange'], c['image_identity'], d['frame']['rounds_per_frame_rank0'])" $O/$name.json $name; }
run c4_bands --config 4 --spp 16 --steps 2 --warmup 1
run c3_bands --config 3 --shard bands --spp 32 --steps 2 --warmup 1
run c3_samples --config 3 --spp 64 --steps 2 --warmup 1
run c2_samples --config 2 --spp 32 --steps 2 --warmup 1
