# bench.py self-launching 4 ranks on a one-GPU box (--one-gpu-flow-check: every rank on
# device 0, the exchange over the gloo fallback since RCCL refuses ranks sharing a device),
# both shards.  Output under gpurun_out/r03_flow4/.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03_flow4
mkdir -p "$O"
for sh in samples bands; do
  timeout -k 10 500 python3 bench.py --gpus 4 --one-gpu-flow-check --steps 2 --warmup 1 --spp 64 --shard $sh \
      --no-cpu-baseline --no-steady > "$O/flow_$sh.log" 2>&1 || { tail -20 "$O/flow_$sh.log"; exit 1; }
  grep '^{"metric"' "$O/flow_$sh.log" | tail -1 > "$O/flow_$sh.json"
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('flow', sys.argv[2], d['n_gpus'], d['value'], d['config']['exchange'], d['frame']['rounds_per_frame_rank0'])" "$O/flow_$sh.json" $sh
done
