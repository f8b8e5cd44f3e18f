set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_coverage.py -x -v --timeout 200 --timeout-method thread -m gpu -k "sample_shard or sample_shards" -p no:cacheprovider > gpurun_out/shard_tests.log 2>&1 || { tail -30 gpurun_out/shard_tests.log; exit 1; }
tail -4 gpurun_out/shard_tests.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { tail -20 gpurun_out/bench1.err; exit 1; }
cut -c1-400 gpurun_out/bench1.json
for sh in samples bands; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --one-gpu-flow-check --no-cpu-baseline --shard $sh > gpurun_out/bench2_$sh.json 2> gpurun_out/bench2_$sh.err || { tail -30 gpurun_out/bench2_$sh.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/bench2_$sh.json').read().strip().splitlines()[-1]);print('$sh', d['value'], d['n_gpus'], d['scaling'], d['config']['exchange'], d['config']['parallelism'])"
done
