"""Render ROUNDS separate-kernel rounds of config K with a given build of
libpathtracer.so (for profilers: PC sampling, PMC passes on one kernel mix).

usage: python tools/run_rounds.py [--lib build/variants/NAME.so] [--config K] [--settle S] [--rounds R]
"""
import argparse
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--settle", type=int, default=34)
    ap.add_argument("--rounds", type=int, default=64)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--nranks", type=int, default=1)
    ap.add_argument("--streams", type=int, default=1)
    ap.add_argument("--fused", type=int, default=0, help="ptSetBasicRendererFusedRounds mode (0 never, 1 auto)")
    ap.add_argument("--batch", type=int, default=1, help="round batch for the timed rounds (1: one launch pair each)")
    ap.add_argument("--split", type=int, default=0, help="tile groups (ptSetBasicRendererSplit; 0 automatic, 1 off)")
    a = ap.parse_args()
    if a.lib:
        os.environ["PT_HIP_LIB"] = str((ROOT / a.lib) if not os.path.isabs(a.lib) else a.lib)
    sys.path.insert(0, str(ROOT))
    import bench
    pt = bench.load_package()
    scene = pt.Scene.config(a.config)
    info = scene.info
    dev = pt.Device(0)
    ds = pt.DeviceScene(dev)
    ds.update(scene)
    sb = pt.SampleBuffer(dev, info.width, info.height)
    r = pt.BasicRenderer(dev, ds, sb, rank=a.rank, nranks=a.nranks, streams=a.streams)
    r.set_fused_rounds(a.fused)
    r.set_round_batch(a.batch)
    r.set_split(a.split)
    r.RenderFlags = info.render_flags
    r.PathTerminationProbability = info.termination_probability
    r.reset()
    r.run(2)
    # Settle with the same launch schedule as the timed rounds (a profile
    # then averages launches of one kind: whole-frame or one tile group's).
    r.run_rounds(a.settle)
    dev.synchronize()
    t0 = time.perf_counter()
    r.run_rounds(a.rounds)
    dev.synchronize()
    dt = time.perf_counter() - t0
    print(f"C{a.config} rank {a.rank}/{a.nranks} x{a.streams} streams, batch {a.batch}, split {r.split()}: {a.rounds} rounds, "
          f"{dt / a.rounds * 1e3:.4f} ms per round, {r.slot_count} slots", flush=True)
    for x in (r, sb, ds, dev):
        x.close()


if __name__ == "__main__":
    main()
