"""Rank program for the multi-process tests, launched exactly like bench.py
(python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1).

Each rank renders its 16-row pixel bands over two
progressive frames (Reset + Run(2) + Run(1), then one more Run(1)); after
each frame the float4 accumulators are summed to rank 0 with a gloo reduce,
the CPU stand-in for ptCommReduceSampleBuffer's ncclReduce: like it, each
rank contributes only its own bands.  Rank 0 writes both reduced frames and
the max-over-ranks wall time.

PT_DIST_RENDERER=gpu renders with the product (libpathtracer.so, every rank
on device 0, -m gpu tests); the default is the CPU oracle (the CPU suite).
PT_DIST_SHARD=samples: sample sharding instead (bench.py's default) -- every
rank renders the whole frame from FrameIndex rank << 24 and the whole
accumulators are summed (the stand-in for ptCommReduceSampleBufferInto).
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
    gpu = os.environ.get("PT_DIST_RENDERER") == "gpu"
    samples = os.environ.get("PT_DIST_SHARD") == "samples"
    prank, pn = (0, 1) if samples else (rank, world)
    if gpu:
        dev = pt.Device(0)
        ds = pt.DeviceScene(dev)
        ds.update(scene)
        sb = pt.SampleBuffer(dev, W, H)
        r = pt.BasicRenderer(dev, ds, sb, rank=prank, nranks=pn)
        accum = sb.read
    else:
        r = oracle_lib.OracleRenderer(scene.packs(), W, H, rank=prank, nranks=pn, threads=2)
        accum = r.accum
    r.RenderFlags = 3
    if samples:
        r.FrameIndex = rank << 24
    owned = pt.owned_pixels(W, H, prank, pn)
    frames = []
    dist.barrier()
    t0 = time.perf_counter()
    r.reset()
    r.run(2)
    r.run(1)
    for frame in range(2):
        if frame:
            r.run(1)
        a = accum()
        a[~owned] = 0.0
        acc = torch.from_numpy(a)
        dist.reduce(acc, dst=0, op=dist.ReduceOp.SUM)
        frames.append(acc.numpy().copy())
    dist.barrier()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    n_owned = torch.tensor([int(owned.sum())], dtype=torch.int64)
    dist.all_reduce(n_owned, op=dist.ReduceOp.SUM)
    if rank == 0:
        np.savez(out_path, accum=frames[0], accum2=frames[1], seconds=dt.numpy(), owned=n_owned.numpy(), world=world)
    r.close()
    if gpu:
        for x in (sb, ds, dev):
            x.close()
    scene.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
