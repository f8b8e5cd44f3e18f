"""Active-ray compaction ACROSS launches, modelled on real step counts
(VERDICT r05 task 3).

Round 5 compacted rays inside a block, between barriers, and lost: the
block's waves then stepped in lock-step and the latency hiding between them
was gone ("Extend cost model").  The variant asked for here needs
no barrier: every extend launch stops each wave after S steps; the rays of a
wave still traversing save their traversal state (lane_state: the level ray,
the closest hit so far, the node words, the stack) to a queue, packed by
one ballot + mbcnt + one atomic per wave; a continuation launch traces the
queue densely, 64 survivors per wave, and so on.

This script answers the "measure first" part.

  dump   (GPU)  per-ray traversal step counts of several settled rounds of a
                config, per ray position (ptExtendStepCounts), to an .npz;
  model  (CPU)  wave-steps of the one-launch extend against S-capped launches
                with compacted continuations, and the bytes the saved states
                move (64 B of lane state + 2 B per stack entry, each way).

A wave step is the unit of issue time: a wave of 64 lanes costs as long as
its longest ray.  The model counts wave-steps only; it does not credit the
continuation's incoherent rays or charge their cache misses, so it is an
upper bound on what compaction can save.

usage: python tools/exp_compact2.py dump OUT.npz CONFIG [ROUNDS]
       python tools/exp_compact2.py model IN.npz [IN.npz ...] > OUT.json
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent


def dump(out, config, rounds=3):
    sys.path.insert(0, str(ROOT))
    import __graft_entry__ as ge
    pt = ge._load_package()
    s = pt.Scene.config(config)
    info = s.info
    dev = pt.Device(0)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    sb = pt.SampleBuffer(dev, info.width, info.height)
    r = pt.BasicRenderer(dev, ds, sb)
    r.RenderFlags = info.render_flags
    r.PathTerminationProbability = info.termination_probability
    r.reset()
    r.run(2)
    r.run_rounds(34)
    steps = []
    for _ in range(rounds):
        steps.append(np.minimum(r.extend_step_counts(), 65535).astype(np.uint16))
        r.run_rounds(1)
    dev.synchronize()
    np.savez_compressed(out, steps=np.stack(steps), config=config, width=info.width, height=info.height,
                        split=r.split()["groups"])
    for x in (r, sb, ds, dev):
        x.close()
    s.close()


def wave_max(a):
    """a: (..., 64*k) -> per 64-lane wave maximum."""
    return a.reshape(-1, 64).max(axis=1)


def schedule(steps, caps, order="source"):
    """Wave-steps of launches capped at caps[0], caps[1], ... (the last
    launch uncapped) with survivors compacted between launches.

    steps: per-ray step counts in ray-position order (waves = 64 consecutive).
    order: how the survivors of a launch are packed -- "source" keeps the
    positions' order (each wave's survivors land as one contiguous chunk,
    chunks in wave order); "shuffle" puts the chunks in random order (the
    atomics' arrival order).  Returns (wave_steps per launch, survivors
    saved per launch, survivor stack-depth proxy)."""
    rng = np.random.default_rng(1)
    cur = steps.astype(np.int64)
    ws, saved = [], []
    for i, cap in enumerate(list(caps) + [None]):
        n = cur.size
        pad = (-n) % 64
        w = np.concatenate([cur, np.zeros(pad, np.int64)]) if pad else cur
        m = wave_max(w)
        if cap is None:
            ws.append(int(m.sum()))
            saved.append(0)
            break
        ws.append(int(np.minimum(m, cap).sum()))
        alive = w > cap
        if order == "shuffle":
            idx = np.arange(w.size).reshape(-1, 64)
            perm = rng.permutation(idx.shape[0])
            wv = w.reshape(-1, 64)[perm].reshape(-1)
            av = alive.reshape(-1, 64)[perm].reshape(-1)
            nxt = wv[av] - cap
        else:
            nxt = w[alive] - cap
        saved.append(int(nxt.size))
        cur = nxt
        if cur.size == 0:
            break
    return ws, saved


def model(paths):
    out = {}
    for p in paths:
        d = np.load(p)
        steps = d["steps"].astype(np.int64)      # (rounds, positions)
        cfg = int(d["config"])
        base = sum(int(wave_max(np.concatenate([s, np.zeros((-s.size) % 64, np.int64)])).sum()) for s in steps)
        lane = int(steps.sum())
        res = {"rays_per_round": int(steps.shape[1]), "rounds": int(steps.shape[0]),
               "steps_per_ray": round(lane / steps.size, 2),
               "p50": int(np.percentile(steps, 50)), "p90": int(np.percentile(steps, 90)),
               "p99": int(np.percentile(steps, 99)), "max": int(steps.max()),
               "simd_efficiency": round(lane / (64 * base), 4), "schedules": {}}
        for caps in ([16], [24], [32], [40], [48], [64], [24, 48], [32, 64], [16, 32, 48], [32, 48, 64, 96]):
            for order in ("source", "shuffle"):
                tot, sv = 0, 0
                per = None
                for s in steps:
                    ws, saved = schedule(s, caps, order)
                    tot += sum(ws)
                    sv += sum(saved)
                    per = ws if per is None else [a + b for a, b in zip(per, ws)]
                key = "/".join(map(str, caps)) + ":" + order
                res["schedules"][key] = {
                    "wave_steps_vs_one_launch": round(tot / base, 4),
                    "saved_states_per_ray": round(sv / steps.size, 4),
                    # 64 B of lane state + a 16-entry u16 stack allowance, written and read back
                    "state_bytes_per_ray": round(sv / steps.size * 2 * (64 + 32), 2),
                    "launch_share": [round(x / tot, 3) for x in per],
                }
        out[f"C{cfg}"] = res
    return out


def main():
    if sys.argv[1] == "dump":
        dump(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]) if len(sys.argv) > 4 else 3)
    else:
        print(json.dumps(model(sys.argv[2:]), indent=1))


if __name__ == "__main__":
    main()
