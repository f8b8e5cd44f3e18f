"""One-GPU rehearsal of the N-GPU strong-scaling run (bench.py --gpus N).

For each config and N, renders the partition rank 0 of N gets (the 16-row
bands b with b % N == 0: the most bands of any rank, so the slowest rank)
on device 0 and times K rounds.  The predicted N-GPU throughput is the whole
frame's rays per round / rank 0's round time.  This is a PREDICTION: the
other ranks run on other GPUs in the real run, and the frame-end RCCL band
gather (ptCommGatherSampleBuffer) is not included.

usage: python tools/rehearse_scaling.py OUT.json [--steps K] [--configs 3,4] [--ns 1,2,4,8]
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import sys
import time
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
    ap.add_argument("out")
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--configs", default="3,4")
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--groups", default="", help="comma list of PT_RUN_GROUPS values to try (default: the runtime's choice)")
    ap.add_argument("--batches", default="0", help="comma list of round batches (ptSetBasicRendererRoundBatch) to try")
    args = ap.parse_args()
    pt = load_package()
    dev = pt.Device(0)
    rows = []
    for cfg in [int(c) for c in args.configs.split(",")]:
        scene = pt.Scene.config(cfg)
        W, H = scene.info.width, scene.info.height
        ds = pt.DeviceScene(dev)
        ds.update(scene)
        for n, groups, batch in [(int(x), g, int(b)) for x in args.ns.split(",")
                                 for g in (args.groups.split(",") if args.groups else [None])
                                 for b in args.batches.split(",")]:
            if groups is None:
                os.environ.pop("PT_RUN_GROUPS", None)
            else:
                os.environ["PT_RUN_GROUPS"] = groups
            sb = pt.SampleBuffer(dev, W, H)
            r = pt.BasicRenderer(dev, ds, sb, rank=0, nranks=n)
            r.RenderFlags = scene.info.render_flags
            r.set_round_batch(batch)
            r.reset()
            r.run(2)
            r.run(32)
            dev.synchronize()
            dev.set_profiling(True, period=4)
            dev.reset_kernel_stats()
            rays0, _ = r.stats()
            t0 = time.perf_counter()
            if batch != 1:                 # 0 = automatic round batches, R >= 2 = R per launch
                r.run_rounds(args.steps)
            else:
                for _ in range(args.steps):
                    r.run(1)
            dev.synchronize()
            dt = time.perf_counter() - t0
            rays1, _ = r.stats()
            ne, me = dev.kernel_stats(1)
            ns_, ms = dev.kernel_stats(2)
            nr, mr = dev.kernel_stats(5)
            dev.set_profiling(False)
            owned = int(np.sum(pt.owned_pixels(W, H, 0, n)))
            step_ms = dt / args.steps * 1e3
            row = {
                "config": cfg, "frame": f"{W}x{H}", "n_gpus": n, "rank0_pixels": owned,
                "rank0_tiles": r.slot_count // 256, "run_groups": r.run_groups, "round_batch": batch,
                "rank0_ms_per_step": round(step_ms, 4),
                "rank0_mrays_per_s": round((rays1 - rays0) / dt / 1e6, 1),
                "extend_ms": round(me / max(ne, 1), 4), "shade_ms": round(ms / max(ns_, 1), 4),
                "round_launch_ms": round(mr / max(nr, 1), 4),   # fused round / round batch launch
                "predicted_frame_mrays_per_s": round(W * H / (step_ms * 1e-3) / 1e6, 1),
            }
            rows.append(row)
            print(json.dumps(row), flush=True)
            r.close()
            sb.close()
        ds.close()
        scene.close()
    base = {}
    for r in rows:
        if r["n_gpus"] == 1:
            base[r["config"]] = max(base.get(r["config"], 0), r["predicted_frame_mrays_per_s"])
    for r in rows:
        b = base.get(r["config"])
        if b:
            r["predicted_efficiency"] = round(r["predicted_frame_mrays_per_s"] / (b * r["n_gpus"]), 3)
    out = {"kind": "prediction: rank 0 of N timed alone on one MI355X; exchange not included; unmeasured on N GPUs",
           "steps": args.steps, "rows": rows}
    Path(args.out).write_text(json.dumps(out, indent=1))
    dev.close()


if __name__ == "__main__":
    main()
