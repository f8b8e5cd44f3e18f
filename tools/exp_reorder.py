"""Experiment: does reordering extension rays speed up the extend kernel?

Renders C3 for a few rounds, reads back the slot rays, then traces the same
ray set through ptTraceRays (the production extend kernel over caller arrays)
in several orders.  Run under `rocprofv3 --kernel-trace`; the per-dispatch
extend durations are matched to the orders by `tools/exp_reorder_report.py`.
Hits must be identical per ray in every order (checked here).
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


def morton3(q):
    """Interleave three 10-bit integers (n,3) into 30-bit codes."""
    def spread(v):
        v = v.astype(np.uint64) & 0x3FF
        v = (v | (v << 16)) & 0x030000FF
        v = (v | (v << 8)) & 0x0300F00F
        v = (v | (v << 4)) & 0x030C30C3
        v = (v | (v << 2)) & 0x09249249
        return v
    return spread(q[:, 0]) | (spread(q[:, 1]) << 1) | (spread(q[:, 2]) << 2)


def main():
    pt = load()
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    scene = pt.Scene.config(3)
    info = scene.info
    W, H = info.width, info.height
    dev = pt.Device(0)
    ds = pt.DeviceScene(dev)
    ds.update(scene)
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    r.RenderFlags = info.render_flags
    r.PathTerminationProbability = info.termination_probability
    r.reset()
    r.run(2)
    for _ in range(rounds):
        r.run(1)
    dev.synchronize()
    st = r.read_state().reshape(-1)
    y, x = np.divmod(np.arange(W * H), W)
    slot = ((y // 16) * (W // 16) + x // 16) * 256 + (y % 16) * 16 + x % 16
    base = np.argsort(slot, kind="stable")          # pixel indices in slot order
    O = st["origin"][base].astype(np.float32)
    PV = st["packed_velocity"][base].astype(np.uint32)
    n = len(PV)
    V = kat.unpack_unit_vector(PV)
    lo, hi = O.min(0), O.max(0)
    q = np.clip(((O - lo) / np.maximum(hi - lo, 1e-9) * 1023).astype(np.int64), 0, 1023)
    oct_ = ((V[:, 0] < 0).astype(np.uint64) | ((V[:, 1] < 0).astype(np.uint64) << 1)
            | ((V[:, 2] < 0).astype(np.uint64) << 2))
    mo = morton3(q)
    qd = np.clip(((V + 1) * 0.5 * 1023).astype(np.int64), 0, 1023)
    md = morton3(qd)
    rng = np.random.default_rng(1)

    def blockwise(key, b):
        idx = np.arange(n)
        return np.lexsort((key, idx // b))

    def coarse(bits):
        return (oct_ << np.uint64(bits - 3)) | (mo >> np.uint64(30 - (bits - 3)))

    # Pixel (x, y) of every ray in slot order; wave footprints other than the
    # tile layout's 16x4 rows.
    px, py = x[base], y[base]
    tile = (py // 16) * (W // 16) + px // 16
    quad = ((py % 16) // 8) * 2 + (px % 16) // 8
    in8 = (py % 8) * 8 + px % 8
    orders = {
        "slot": np.arange(n),
        "wave8x8": np.lexsort((in8, quad, tile)),
        "wave8x8_z": np.lexsort((morton3(np.stack([px % 8, py % 8, np.zeros_like(px)], 1)), quad, tile)),
        "global_oct_morton": np.lexsort((mo, oct_)),
        "global_morton_origin": np.argsort(mo, kind="stable"),
        "global_bin9": np.argsort(coarse(9), kind="stable"),
        "global_bin12": np.argsort(coarse(12), kind="stable"),
        "global_bin15": np.argsort(coarse(15), kind="stable"),
        "global_bin18": np.argsort(coarse(18), kind="stable"),
        "global_morton12": np.argsort(mo >> np.uint64(18), kind="stable"),
        "block256_oct_dir": blockwise((oct_ << 30) | md, 256),
        "block256_oct": blockwise(oct_, 256),
        "block256_oct_dir6": blockwise((oct_ << 6) | (md >> 24), 256),
        "block256_dir": blockwise(md, 256),
        "block512_oct_dir": blockwise((oct_ << 30) | md, 512),
        "block256_oct_morton": blockwise((oct_ << 30) | mo, 256),
        "slot_again": np.arange(n),
    }
    dur = np.full(n, 1048576.0, np.float32)
    # Per-ray traversal steps (order-independent), for longest-first block
    # permutations of every order: a block lives as long as its slowest ray's
    # wave, so blocks sorted by their max step count, descending, emulate the
    # production extend's longest-first tile dispatch (with perfect costs).
    stats, steps = ds.trace_rays_stats(O, PV, dur)
    print("slot-order stats", json.dumps(stats), flush=True)

    def lpt(p):
        st = steps[p]
        nb = (n + 255) // 256
        pad = np.zeros(nb * 256, np.int64)
        pad[:n] = st
        cost = pad.reshape(nb, 256).max(1)
        blocks = np.argsort(-cost, kind="stable")
        idx = (blocks[:, None] * 256 + np.arange(256)[None, :]).reshape(-1)
        idx = idx[idx < n]
        return p[idx]

    def groupwise(key, g):
        idx = np.arange(n)
        return np.lexsort((key, idx // (256 * g)))

    orders["group4_oct_morton"] = groupwise((oct_ << np.uint64(30)) | mo, 4)
    orders["group16_oct_morton"] = groupwise((oct_ << np.uint64(30)) | mo, 16)
    orders["group64_oct_morton"] = groupwise((oct_ << np.uint64(30)) | mo, 64)
    for k in list(orders):
        if k != "slot_again":
            orders[k + "+lpt"] = lpt(orders[k])
    # per-order SIMD efficiency (wave max vs mean steps) and wave-step totals
    eff = {}
    for k, p in orders.items():
        st = steps[p].astype(np.int64)
        nw = (n + 63) // 64
        pad = np.zeros(nw * 64, np.int64)
        pad[:n] = st
        w = pad.reshape(nw, 64)
        eff[k] = {"wave_steps": int(w.max(1).sum()), "simd_eff": round(float(st.sum() / max(w.max(1).sum() * 64, 1)), 4)}
    (ROOT / "gpurun_out").mkdir(exist_ok=True)
    (ROOT / "gpurun_out" / "exp_reorder_eff.json").write_text(json.dumps(eff, indent=1))
    reps = 3
    ref = None
    log = []
    for name, p in orders.items():
        for k in range(reps):
            h = ds.trace_rays(O[p], PV[p], dur)
            back = np.empty_like(h)
            back[p] = h
            if ref is None:
                ref = back
            same = bool(np.array_equal(back.view(np.uint8), ref.view(np.uint8)))
            log.append({"order": name, "rep": k, "identical": same})
            print(name, k, "identical" if same else "MISMATCH", flush=True)
    (ROOT / "gpurun_out").mkdir(exist_ok=True)
    (ROOT / "gpurun_out" / "exp_reorder_orders.json").write_text(json.dumps(log))
    for o in (r, sb, ds):
        o.close()
    dev.close()


if __name__ == "__main__":
    main()
