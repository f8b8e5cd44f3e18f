"""Experiment (simulation on real step counts): compacting a tile's unfinished
rays into fewer waves at fixed step marks.

The extend kernel runs one 256-ray tile per block, four waves of 64 rays; a
wave lasts as long as its longest ray, so about half of its lane-steps are
idle (SIMD efficiency ~0.5).  If the block's four waves stopped at step K,
packed the still-traversing rays of the tile into the first ceil(R/64)
waves (order kept) and the emptied waves exited, the wave-steps of the tile
would drop.  This script reads every ray's traversal step count for several
settled rounds (ptExtendStepCounts, per ray position) and reports the
wave-steps of compaction schedules relative to none.
"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))
from exp_reorder import load  # noqa: E402


def wave_steps(steps, marks):
    """steps: (tiles, 256) per-position step counts.  marks: increasing step
    marks where the tile compacts.  Returns total wave-steps."""
    total = 0
    cur = steps.copy()            # remaining steps per ray, rays in current lane order
    alive = cur > 0
    done_before = 0
    for k in list(marks) + [None]:
        # rays still running, packed in order at the start of the block
        T = cur.shape[0]
        order = np.argsort(~alive, axis=1, kind="stable")
        packed = np.take_along_axis(np.where(alive, cur, 0), order, axis=1)
        waves = packed.reshape(T, 4, 64).max(axis=2)                      # remaining max per wave
        seg = waves if k is None else np.minimum(waves, k - done_before)
        total += int(seg.sum())
        if k is None:
            break
        cur = np.maximum(packed - (k - done_before), 0)
        alive = cur > 0
        done_before = k
    return total


def main():
    pt = load()
    dev = pt.Device(0)
    for cid in [int(c) for c in (sys.argv[1:] or ["3", "5", "2"])]:
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
        rows = []
        for _ in range(3):
            rows.append(r.extend_step_counts().astype(np.int64).reshape(-1, 256))
            r.run(1)
        steps = np.concatenate(rows)
        base = wave_steps(steps, [])
        lane = int(steps.sum())
        out = {"tiles": int(steps.shape[0]), "simd_eff": round(lane / (64 * base), 4)}
        for marks in ([16], [24], [32], [40], [16, 32], [24, 40], [16, 32, 48], [12, 24, 36, 48],
                      list(range(8, 160, 8)), list(range(16, 160, 16))):
            ws = wave_steps(steps, marks)
            out[",".join(map(str, marks[:4])) + ("..." if len(marks) > 4 else "")] = round(ws / base, 4)
        print(f"C{cid}", json.dumps(out), flush=True)
        for o in (r, sb, ds):
            o.close()
    dev.close()


if __name__ == "__main__":
    main()
