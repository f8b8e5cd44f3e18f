"""Step-budget split of the extend kernel, simulated on real per-ray step
counts (ptExtendStepCounts): phase 1 traces every ray for at most K steps,
the rays still running are compacted (order kept) and finished in phase 2.
Prints the wave-step cost of each K relative to one pass (the SIMD lanes a
wave occupies until its longest ray ends)."""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))
from exp_reorder import load  # noqa: E402


def wave_cost(steps):
    n = len(steps) // 64 * 64
    w = steps[:n].reshape(-1, 64)
    tail = steps[n:]
    return int(w.max(axis=1).sum()) + (int(tail.max()) if len(tail) else 0)


pt = load()
dev = pt.Device(0)
for cid in [int(c) for c in (sys.argv[1:] or ["3", "5"])]:
    scene = pt.Scene.config(cid)
    info = scene.info
    ds = pt.DeviceScene(dev)
    ds.update(scene)
    sb = pt.SampleBuffer(dev, info.width, info.height)
    r = pt.BasicRenderer(dev, ds, sb)
    r.RenderFlags = info.render_flags
    r.PathTerminationProbability = info.termination_probability
    r.reset()
    r.run(10)
    s = r.extend_step_counts().astype(np.int64)
    base = wave_cost(s)
    out = {"rays": int((s > 0).sum()), "lane_steps": int(s.sum()), "one_pass_wave_steps": base,
           "simd_eff": round(s.sum() / (64 * base), 4),
           "pct": {int(p): int(np.percentile(s[s > 0], p)) for p in (50, 90, 99, 100)}}
    res = {}
    for K in (8, 12, 16, 20, 24, 32, 40, 48):
        p1 = wave_cost(np.minimum(s, K))
        rest = s[s > K] - K
        p2 = wave_cost(rest)
        res[K] = {"rel": round((p1 + p2) / base, 4), "stragglers": round(len(rest) / max(len(s), 1), 4)}
    out["split"] = res
    print(f"C{cid}", json.dumps(out), flush=True)
    for o in (r, sb, ds):
        o.close()
dev.close()
