# Rehearses bench.py's multi-rank flow (torch.distributed.run, 2 ranks) on one
# GPU with PT_BENCH_REHEARSAL=1, then a normal N=1 line.
mkdir -p gpurun_out
PT_BENCH_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 8 --warmup 2 > gpurun_out/rehearse2.log 2>&1; rc=$?; echo "rehearsal N=2 rc=$rc"; tail -1 gpurun_out/rehearse2.log | cut -c1-600
[ $rc -eq 0 ] || exit $rc
