"""Predictors for the longest-first tile order (see exp_lpt.py): block times
(max wave steps) of 12 consecutive rounds; the order for the next round from
the last round alone, or from an exponential moving average of the rounds."""
import heapq
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))
from exp_reorder import load  # noqa: E402


def makespan(durations, slots=2048):
    heap = [0.0] * slots
    for d in durations:
        heapq.heappush(heap, heapq.heappop(heap) + d)
    return max(heap)


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
    r.run(2)
    r.run(32)
    hist = []
    for k in range(13):
        s = r.extend_step_counts().astype(np.int64)
        hist.append(s.reshape(-1, 64).max(axis=1).reshape(-1, 4).max(axis=1).astype(float))
        r.run(1)
    target = hist[-1]
    bound = target.sum() / 2048
    out = {"natural": makespan(target) / bound, "oracle": makespan(np.sort(target)[::-1]) / bound}
    prev = hist[-2]
    out["prev"] = makespan(target[np.argsort(-prev, kind="stable")]) / bound
    for a in (0.5, 0.25, 0.125):
        ema = hist[0].copy()
        for h in hist[1:-1]:
            ema = (1 - a) * ema + a * h
        out[f"ema{a}"] = makespan(target[np.argsort(-ema, kind="stable")]) / bound
    mean = np.mean(hist[:-1], axis=0)
    out["mean12"] = makespan(target[np.argsort(-mean, kind="stable")]) / bound
    print(f"C{cid}", json.dumps({k: round(v, 4) for k, v in out.items()}), flush=True)
    for o in (r, sb, ds):
        o.close()
dev.close()
