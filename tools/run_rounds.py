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
    r = pt.BasicRenderer(dev, ds, sb)
    r.set_fused_rounds(0)
    r.RenderFlags = info.render_flags
    r.PathTerminationProbability = info.termination_probability
    r.reset()
    r.run(2)
    for _ in range(a.settle):
        r.run(1)
    dev.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.rounds):
        r.run(1)
    dev.synchronize()
    dt = time.perf_counter() - t0
    print(f"C{a.config} {a.rounds} rounds: {dt / a.rounds * 1e3:.4f} ms per round", flush=True)
    for x in (r, sb, ds, dev):
        x.close()


if __name__ == "__main__":
    main()
