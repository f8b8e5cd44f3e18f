"""Block-level tail of the extend kernel, simulated from real per-ray step
counts (ptExtendStepCounts): a block's duration ~ its longest wave (max steps
among the wave's 64 rays); 2048 block slots (256 CUs x 8) filled greedily in
dispatch order.  Prints the makespan of the natural tile order and of the
longest-first order against the perfect-packing bound sum / slots."""
import heapq
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))
from exp_reorder import load  # noqa: E402


def makespan(durations, slots):
    heap = [0.0] * slots
    for d in durations:
        t = heapq.heappop(heap)
        heapq.heappush(heap, t + d)
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
    s = r.extend_step_counts().astype(np.int64)
    waves = s.reshape(-1, 64).max(axis=1)
    blocks = waves.reshape(-1, 4).max(axis=1).astype(float)
    wave_sum = waves.reshape(-1, 4).sum(axis=1)
    bound = blocks.sum() / 2048
    out = {"blocks": len(blocks), "natural": round(makespan(blocks, 2048) / bound, 4),
           "longest_first": round(makespan(np.sort(blocks)[::-1], 2048) / bound, 4),
           "block_eff": round(float(wave_sum.sum() / (4 * blocks.sum())), 4)}
    s2 = None
    # previous-round predictor: next round's blocks in the order of this round's durations
    r.run(1)
    s2 = r.extend_step_counts().astype(np.int64)
    b2 = s2.reshape(-1, 64).max(axis=1).reshape(-1, 4).max(axis=1).astype(float)
    order = np.argsort(-blocks, kind="stable")
    out["next_round_natural"] = round(makespan(b2, 2048) / (b2.sum() / 2048), 4)
    rng = np.random.default_rng(1)
    perm = rng.permutation(len(b2))
    out["next_round_random"] = round(makespan(b2[perm], 2048) / (b2.sum() / 2048), 4)
    nb = len(b2)
    bits = int(np.ceil(np.log2(nb)))
    rev = np.array([int(format(i, f"0{bits}b")[::-1], 2) for i in range(1 << bits)])
    rev = rev[rev < nb]
    out["next_round_bitrev"] = round(makespan(b2[rev], 2048) / (b2.sum() / 2048), 4)
    # reversed natural order (bottom rows first)
    out["next_round_reversed"] = round(makespan(b2[::-1], 2048) / (b2.sum() / 2048), 4)
    out["next_round_prev_order"] = round(makespan(b2[order], 2048) / (b2.sum() / 2048), 4)
    print(f"C{cid}", json.dumps(out), flush=True)
    for o in (r, sb, ds):
        o.close()
dev.close()
