"""Multi-rank path on CPU: world_size-2 gloo run of the band-partitioned
render + frame-end sum reduce over two progressive frames (the flow of
bench.py / ptCommReduceSampleBuffer, with the CPU oracle standing in for the
GPU renderer here; tests/test_gpu_coverage.py runs the same worker with the
product renderer on the GPU).  Both reduced frames must equal the
single-rank render bit for bit."""
from __future__ import annotations

import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np

import oracle_lib

HERE = Path(__file__).resolve().parent


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_band_render_reduces_to_full_frame(pt, tmp_path):
    cfg, W, H = 1, 48, 80          # 5 bands of 16 rows: rank 0 owns 3, rank 1 owns 2
    out = tmp_path / "reduced.npz"
    env = dict(os.environ, OMP_NUM_THREADS="2", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}",
           str(HERE / "dist_worker.py"), str(out), str(cfg), str(W), str(H)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    got = np.load(out)
    assert int(got["world"]) == 2
    assert int(got["owned"][0]) == W * H           # bands cover the frame exactly once
    s = pt.Scene.config(cfg)
    o = oracle_lib.OracleRenderer(s.packs(), W, H, threads=2)
    o.RenderFlags = 3
    o.reset()
    o.run(2)
    o.run(1)
    full = o.accum()
    o.run(1)
    full2 = o.accum()
    o.close()
    s.close()
    assert np.array_equal(got["accum"].view(np.uint32), full.view(np.uint32))
    assert np.array_equal(got["accum2"].view(np.uint32), full2.view(np.uint32))


def test_two_rank_sample_shards_reduce_to_sum(pt, tmp_path):
    """Sample sharding (bench.py's default): both ranks render the whole
    frame, rank r from FrameIndex r << 24; the reduced frames are the sum of
    the two single-process renders with those offsets."""
    cfg, W, H = 1, 40, 24
    out = tmp_path / "reduced.npz"
    env = dict(os.environ, OMP_NUM_THREADS="2", HSA_ENABLE_IPC_MODE_LEGACY="0", PT_DIST_SHARD="samples")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}",
           str(HERE / "dist_worker.py"), str(out), str(cfg), str(W), str(H)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    got = np.load(out)
    assert int(got["owned"][0]) == 2 * W * H       # every rank renders every pixel
    s = pt.Scene.config(cfg)
    want = [np.zeros((H, W, 4), np.float32), np.zeros((H, W, 4), np.float32)]
    for rank in range(2):
        o = oracle_lib.OracleRenderer(s.packs(), W, H, threads=2)
        o.RenderFlags = 3
        o.FrameIndex = rank << 24
        o.reset()
        o.run(2)
        o.run(1)
        want[0] = want[0] + o.accum()
        o.run(1)
        want[1] = want[1] + o.accum()
        o.close()
    s.close()
    assert np.array_equal(got["accum"].view(np.uint32), want[0].view(np.uint32))
    assert np.array_equal(got["accum2"].view(np.uint32), want[1].view(np.uint32))
    assert got["accum"][..., 3].sum() > 0


def test_band_ownership(pt):
    for H in (16, 80, 1080, 2160):
        for N in (1, 2, 3, 8):
            masks = [pt.owned_pixels(8, H, r, N) for r in range(N)]
            assert np.array_equal(sum(m.astype(int) for m in masks), np.ones((H, 8), int))
    rows = pt.band_rows(1080, 1, 8)
    assert rows[0] == 16 and rows[15] == 31 and rows[16] == 16 * 9
