"""Experiment: does running two halves of a frame on two HIP streams (two
pt_device objects on one GPU, so two hardware queues) overlap one half's
kernel tails with the other half's work?

Renders C3 rounds three ways, after settling each renderer for --settle
rounds:
  full   one renderer, the whole frame, one stream (the bench's layout);
  serial2 two band renderers (16-row bands, rank 0 / 1 of 2) on ONE device:
         the same work in two launches per kernel, one stream;
  streamsN N band renderers (rank k of N), each on its own device (stream).
Each is timed over --rounds Run(1) rounds per renderer (enqueued alternately,
one synchronize at the end); rays = rounds x slots.  Any partition gives the
same per-slot results (the band split is bit-exact per pixel), so this only
measures throughput.

usage: python tools/exp_two_streams.py [--config 3] [--settle 34] [--rounds 64] [--parts 2,3,4]
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--settle", type=int, default=34)
    ap.add_argument("--rounds", type=int, default=64)
    ap.add_argument("--parts", default="2,3,4", help="band partitions, one device (stream) each")
    a = ap.parse_args()
    a.parts = [int(x) for x in a.parts.split(",")]
    import bench
    pt = bench.load_package()
    scene = pt.Scene.config(a.config)
    info = scene.info
    W, H = info.width, info.height

    def make(dev, rank, nranks):
        ds = pt.DeviceScene(dev)
        ds.update(scene)
        sb = pt.SampleBuffer(dev, W, H)
        r = pt.BasicRenderer(dev, ds, sb, rank=rank, nranks=nranks)
        r.RenderFlags = info.render_flags
        r.PathTerminationProbability = info.termination_probability
        r.reset()
        r.run(2)
        for _ in range(a.settle):
            r.run(1)
        return r, (ds, sb)

    def timed(pairs):
        devs = {id(r.device): r.device for r, _ in pairs}
        for d in devs.values():
            d.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.rounds):
            for r, _ in pairs:
                r.run(1)
        for d in devs.values():
            d.synchronize()
        dt = time.perf_counter() - t0
        rays = sum(r.slot_count for r, _ in pairs) * a.rounds
        return {"seconds": round(dt, 4), "mrays_per_s": round(rays / dt / 1e6, 1),
                "ms_per_round": round(dt / a.rounds * 1e3, 4)}

    out = {"config": a.config, "settle": a.settle, "rounds": a.rounds}
    devs = [pt.Device(0) for _ in range(max(a.parts))]
    made = []
    full = make(devs[0], 0, 1)
    made.append(full)
    out["full"] = timed([full])
    s0, s1 = make(devs[0], 0, 2), make(devs[0], 1, 2)
    made += [s0, s1]
    out["serial2"] = timed([s0, s1])
    for n in a.parts:
        parts = [make(devs[k], k, n) for k in range(n)]
        made += parts
        out[f"streams{n}"] = timed(parts)
        out["full_again"] = timed([full])
    print(json.dumps(out))
    for r, keep in made:
        r.close()
        for k in keep:
            k.close()
    for d in devs:
        d.close()


if __name__ == "__main__":
    main()
