"""What a frame's read-backs cost (VERDICT r05 task 6).

ptRenderFrame reads the completed-path count back between batches of
rounds.  Making the frame end exact without any assumption on the completion
rate means batches no longer than the rounds that cannot overshoot
(ceil(remaining / pixels)), so more batches and more read-backs.  This
script times, on the C3 frame with the product's defaults:

  frame   ptRenderFrame(1024 spp) as built;
  one     Reset, Run(2), then the same rounds in ONE run_rounds call and one
          synchronize (no read-back at all: the floor);
  safe    Reset, Run(2), then batches of ceil(remaining / pixels) rounds with
          a stats() read-back after each, the last rounds one at a time
          (the schedule of an unconditionally exact host loop).

usage: python tools/exp_frame_end.py [CONFIG] [REPS]  -> one JSON line
"""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import __graft_entry__ as ge  # noqa: E402

SIZES = {1: (256, 256, 16), 2: (1024, 1024, 256), 3: (1920, 1080, 1024), 5: (2048, 1024, 8192)}


def main():
    config = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    pt = ge._load_package()
    W, H, spp = SIZES[config]
    if config == 5:
        spp = 1024
    target = spp * W * H
    s = pt.Scene.config(config)
    dev = pt.Device(0)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    r.RenderFlags = s.info.render_flags
    r.PathTerminationProbability = s.info.termination_probability
    px = W * H
    r.FrameIndex = 0
    rounds, samples = r.render_frame(target)   # warm-up, and the round count
    out = {"config": config, "W": W, "H": H, "spp": spp, "rounds": rounds, "split": r.split(), "frame": [],
           "one": [], "safe": [], "safe_batches": 0}

    def timed(fn):
        r.FrameIndex = 0   # every variant renders the same frame (Reset keeps FrameIndex)
        dev.synchronize()
        t = time.perf_counter()
        v = fn()
        dev.synchronize()
        return time.perf_counter() - t, v

    def one():
        r.reset()
        r.run(2)
        r.run_rounds(rounds - 2)
        return r.stats()[1]

    def safe():
        r.reset()
        r.run(2)
        n, batches = 2, 0
        done = 0
        while True:
            done = r.stats()[1]
            if done >= target:
                break
            k = max(1, -(-(target - done) // px))
            r.run_rounds(k)
            n += k
            batches += 1
        return n, batches, done

    for _ in range(reps):
        dt, v = timed(lambda: r.render_frame(target))
        assert v == (rounds, samples), v
        out["frame"].append(dt * 1e3)
        dt, v = timed(one)
        out["one"].append(dt * 1e3)
        dt, (n, b, done) = timed(safe)
        assert n == rounds and done == samples, (n, rounds, done, samples)
        out["safe"].append(dt * 1e3)
        out["safe_batches"] = b
    for k in ("frame", "one", "safe"):
        out[k + "_ms"] = min(out[k])
    print(json.dumps(out), flush=True)
    for x in (r, sb, ds, dev):
        x.close()
    s.close()


if __name__ == "__main__":
    main()
