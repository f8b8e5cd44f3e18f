"""Rank program for tests/test_distributed.py, launched exactly like bench.py
(python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1).

Each rank renders its 16-row pixel bands with the CPU
oracle, then the float4 accumulators are summed to rank 0 with a gloo
reduce — the CPU stand-in for ptCommReduceSampleBuffer's ncclReduce — and
rank 0 writes the reduced frame plus the max-over-ranks wall time.
"""
from __future__ import annotations

import os
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
import conftest  # noqa: E402  (package loader + spectrum table path)
import oracle_lib  # noqa: E402


def main():
    out_path, cfg, W, H = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    pt = conftest.load_package()
    scene = pt.Scene.config(cfg)
    o = oracle_lib.OracleRenderer(scene.packs(), W, H, rank=rank, nranks=world, threads=2)
    o.RenderFlags = 3
    dist.barrier()
    t0 = time.perf_counter()
    o.reset()
    o.run(2)
    o.run(1)
    acc = torch.from_numpy(o.accum())
    dist.reduce(acc, dst=0, op=dist.ReduceOp.SUM)
    dist.barrier()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    owned = torch.tensor([int(pt.owned_pixels(W, H, rank, world).sum())], dtype=torch.int64)
    dist.all_reduce(owned, op=dist.ReduceOp.SUM)
    if rank == 0:
        np.savez(out_path, accum=acc.numpy(), seconds=dt.numpy(), owned=owned.numpy(), world=world)
    o.close()
    scene.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
