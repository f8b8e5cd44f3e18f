"""Experiment: which global sort key, and how well does a one-round-stale
longest-first block order work with it?  (GPU; run under rocprofv3
--kernel-trace, durations matched by tools/exp_reorder_report.py.)

Renders C3, reads the rays of two consecutive rounds (A, then B).  For each
key scheme the rays of B are sorted by key (stable: slot order within a key)
and traced through ptTraceRays in three block orders:
  nolpt    key order;
  stale    256-ray blocks sorted by the max step count of the block with the
           same index in A's sorted order (what the renderer can know: the
           previous round's block times);
  perfect  blocks sorted by their own max step count (unattainable bound).
Hits are identical in every order (checked).
"""
import importlib.util
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tests"))
import kat  # noqa: E402


def load():
    spec = importlib.util.spec_from_file_location("path_tracer_amd", ROOT / "path-tracer_amd" / "__init__.py",
                                                  submodule_search_locations=[str(ROOT / "path-tracer_amd")])
    m = importlib.util.module_from_spec(spec)
    sys.modules["path_tracer_amd"] = m
    spec.loader.exec_module(m)
    return m


def spread(v, bits):
    out = np.zeros_like(v, dtype=np.uint64)
    for b in range(bits):
        out |= ((v.astype(np.uint64) >> np.uint64(b)) & np.uint64(1)) << np.uint64(3 * b)
    return out


def keys(O, V, lo, hi):
    """Key schemes: name -> uint64 key per ray."""
    rel = (O - lo) / np.maximum(hi - lo, 1e-9)
    oct_ = ((V[:, 0] < 0).astype(np.uint64) | ((V[:, 1] < 0).astype(np.uint64) << np.uint64(1))
            | ((V[:, 2] < 0).astype(np.uint64) << np.uint64(2)))
    a = np.abs(V)
    s = a.sum(1)
    du, dv = a[:, 0] / s, a[:, 1] / s

    def cell(bits):
        q = np.clip((rel * (1 << bits)).astype(np.int64), 0, (1 << bits) - 1)
        return spread(q[:, 0], bits) | (spread(q[:, 1], bits) << np.uint64(1)) | (spread(q[:, 2], bits) << np.uint64(2))

    def dirb(bits):
        n = 1 << bits
        qu = np.clip((du * n).astype(np.int64), 0, n - 1).astype(np.uint64)
        qv = np.clip((dv * n).astype(np.int64), 0, n - 1).astype(np.uint64)
        return (qu << np.uint64(bits)) | qv

    c2, c3, c4, c10 = cell(2), cell(3), cell(4), cell(10)
    d1, d2 = dirb(1), dirb(2)
    return {
        "oct_cell8": (oct_ << np.uint64(9)) | c3,
        "oct_cell16": (oct_ << np.uint64(12)) | c4,
        "oct_cell1024": (oct_ << np.uint64(30)) | c10,
        "oct_cell8_dir4": (oct_ << np.uint64(11)) | (c3 << np.uint64(2)) | d1,
        "oct_cell8_dir16": (oct_ << np.uint64(13)) | (c3 << np.uint64(4)) | d2,
        "oct_cell4_dir16": (oct_ << np.uint64(10)) | (c2 << np.uint64(4)) | d2,
        "oct_dir16_cell8": (oct_ << np.uint64(13)) | (d2 << np.uint64(9)) | c3,
        "oct_cell16_dir16": (oct_ << np.uint64(16)) | (c4 << np.uint64(4)) | d2,
    }


def main():
    pt = load()
    scene = pt.Scene.config(3)
    info = scene.info
    W, H = info.width, info.height
    dev = pt.Device(0)
    ds = pt.DeviceScene(dev)
    ds.update(scene)
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    r.RenderFlags = info.render_flags
    r.reset()
    r.run(2)
    for _ in range(30):
        r.run(1)
    dev.synchronize()
    y, x = np.divmod(np.arange(W * H), W)
    slot = ((y // 16) * (W // 16) + x // 16) * 256 + (y % 16) * 16 + x % 16
    base = np.argsort(slot, kind="stable")
    rays = []
    for _ in range(2):
        st = r.read_state().reshape(-1)
        O = st["origin"][base].astype(np.float32)
        PV = st["packed_velocity"][base].astype(np.uint32)
        rays.append((O, PV))
        r.run(1)
        dev.synchronize()
    n = len(rays[0][1])
    dur = np.full(n, 1048576.0, np.float32)
    lo = np.minimum(rays[0][0].min(0), rays[1][0].min(0))
    hi = np.maximum(rays[0][0].max(0), rays[1][0].max(0))
    steps = []
    K = []
    for O, PV in rays:
        steps.append(ds.trace_rays_stats(O, PV, dur)[1].astype(np.int64))
        K.append(keys(O, kat.unpack_unit_vector(PV), lo, hi))
    nb = (n + 255) // 256

    def block_cost(st):
        pad = np.zeros(nb * 256, np.int64)
        pad[:n] = st
        return pad.reshape(nb, 256).max(1)

    def by_blocks(p, cost):
        blocks = np.argsort(-cost, kind="stable")
        idx = (blocks[:, None] * 256 + np.arange(256)[None, :]).reshape(-1)
        return p[idx[idx < n]]

    orders = {}
    eff = {}
    for name in K[1]:
        pa = np.argsort(K[0][name], kind="stable")
        pb = np.argsort(K[1][name], kind="stable")
        orders[name + "|nolpt"] = pb
        orders[name + "|stale"] = by_blocks(pb, block_cost(steps[0][pa]))
        orders[name + "|perfect"] = by_blocks(pb, block_cost(steps[1][pb]))
        w = np.zeros(((n + 63) // 64) * 64, np.int64)
        w[:n] = steps[1][pb]
        wm = w.reshape(-1, 64).max(1)
        eff[name] = {"simd_eff": round(float(steps[1].sum() / (wm.sum() * 64)), 4),
                     "stale_cost_corr": round(float(np.corrcoef(block_cost(steps[0][pa]), block_cost(steps[1][pb]))[0, 1]), 3)}
    # Baseline: the production layout (TileOrder: octant sort inside each
    # 256-slot tile) with the stale longest-first order of the same tiles.
    octs = [K[i]["oct_cell8"] >> np.uint64(9) for i in range(2)]
    idx = np.arange(n)
    ta = np.lexsort((octs[0], idx // 256))
    tb = np.lexsort((octs[1], idx // 256))
    orders["tileorder|stale"] = by_blocks(tb, block_cost(steps[0][ta]))
    orders["tileorder|perfect"] = by_blocks(tb, block_cost(steps[1][tb]))
    # Sorts inside groups of G tiles (one LDS counting sort per group, no
    # global pass), with the stale order of the groups' blocks.
    for G in (16, 32, 64):
        for name in ("oct_cell8", "oct_cell8_dir4"):
            ga = np.lexsort((K[0][name], idx // (256 * G)))
            gb = np.lexsort((K[1][name], idx // (256 * G)))
            orders[f"group{G}_{name}|stale"] = by_blocks(gb, block_cost(steps[0][ga]))
            orders[f"group{G}_{name}|nolpt"] = gb
    orders["slot"] = np.arange(n)
    print(json.dumps(eff, indent=1), flush=True)
    O, PV = rays[1]
    ref = None
    log = []
    for name, p in orders.items():
        for k in range(3):
            h = ds.trace_rays(O[p], PV[p], dur)
            back = np.empty_like(h)
            back[p] = h
            if ref is None:
                ref = back
            same = bool(np.array_equal(back.view(np.uint8), ref.view(np.uint8)))
            log.append({"order": name, "rep": k, "identical": same})
            if not same:
                print("MISMATCH", name, flush=True)
    (ROOT / "gpurun_out").mkdir(exist_ok=True)
    (ROOT / "gpurun_out" / "exp_reorder_orders.json").write_text(json.dumps(log))
    (ROOT / "gpurun_out" / "exp_gsort_eff.json").write_text(json.dumps(eff, indent=1))
    for o in (r, sb, ds):
        o.close()
    dev.close()


if __name__ == "__main__":
    main()
