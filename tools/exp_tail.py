"""Is a small partition's extend bound by its longest waves?  (GPU experiment)

For C3 (or --config) rank 0 of N: after the settle rounds, per ray position
the traversal steps of the current rays (ptExtendStepCounts), summarised per
wave (64 positions = one wave of the extend kernel), next to the extend
launch time of the same rounds.  If the launch time follows the slowest
wave's step count rather than the mean, the partition is tail-bound.
usage: python tools/exp_tail.py [--config 3] [--ns 1,2,4,8] [--samples 8]
"""
import argparse
import importlib.util
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]


def load_package():
    spec = importlib.util.spec_from_file_location("path_tracer_amd", ROOT / "path-tracer_amd" / "__init__.py",
                                                  submodule_search_locations=[str(ROOT / "path-tracer_amd")])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["path_tracer_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--samples", type=int, default=8)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    pt = load_package()
    dev = pt.Device(0)
    scene = pt.Scene.config(args.config)
    W, H = scene.info.width, scene.info.height
    ds = pt.DeviceScene(dev)
    ds.update(scene)
    rows = []
    for n in [int(x) for x in args.ns.split(",")]:
        sb = pt.SampleBuffer(dev, W, H)
        r = pt.BasicRenderer(dev, ds, sb, rank=0, nranks=n)
        r.RenderFlags = scene.info.render_flags
        r.reset()
        r.run(2)
        r.run(32)
        dev.synchronize()
        wave_max, ray_steps, ext_ms = [], [], []
        for _ in range(args.samples):
            s = r.extend_step_counts().astype(np.int64)
            ray_steps.append(s)
            wave_max.append(s.reshape(-1, 64).max(1))
            dev.set_profiling(True, period=1)
            dev.reset_kernel_stats()
            r.run(1)
            dev.synchronize()
            k, ms = dev.kernel_stats(1)
            ext_ms.append(ms / max(k, 1))
            dev.set_profiling(False)
        rs = np.concatenate(ray_steps)
        wm = np.concatenate(wave_max)
        per_round_max = [int(w.max()) for w in wave_max]
        row = {
            "config": args.config, "n": n, "slots": int(r.slot_count), "waves": int(len(wave_max[0])),
            "ray_steps_mean": round(float(rs.mean()), 2), "ray_steps_p99": int(np.percentile(rs, 99)),
            "ray_steps_max": int(rs.max()),
            "wave_max_mean": round(float(wm.mean()), 1), "wave_max_p50": int(np.percentile(wm, 50)),
            "wave_max_p99": int(np.percentile(wm, 99)), "wave_max_max_per_round": per_round_max,
            "extend_ms_per_round": [round(x, 4) for x in ext_ms],
            "us_per_step_of_longest_wave": round(1e3 * float(np.mean(ext_ms)) / float(np.mean(per_round_max)), 4),
        }
        print(json.dumps(row), flush=True)
        rows.append(row)
        r.close()
        sb.close()
    if args.out:
        Path(args.out).write_text(json.dumps(rows, indent=1))
    ds.close()
    scene.close()
    dev.close()


if __name__ == "__main__":
    main()
