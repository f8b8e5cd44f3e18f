"""One-GPU rehearsal of the N-GPU strong-scaling run (bench.py --gpus N).

For each config and N, renders the partition rank 0 of N gets (the 16-row
bands b with b % N == 0: the most bands of any rank, so the slowest rank)
on device 0 and times K rounds.  The predicted N-GPU throughput is rank 0's
ray rate scaled to the whole frame (rank 0 owns the most bands).  Band
partitions carry path streams (bench.py's automatic count: about 2^21 slots
per launch) unless --streams says otherwise.  This is a PREDICTION: the
other ranks run on other GPUs in the real run, and the frame-end RCCL band
gather (ptCommGatherSampleBuffer) is not included.

usage: python tools/rehearse_scaling.py OUT.json [--steps K] [--configs 3,4] [--ns 1,2,4,8] [--streams auto|1,2,..]
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
FILL_SLOTS = 1 << 21      # as bench.py


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
    ap.add_argument("--streams", default="auto", help="comma list of path stream counts, or auto (bench.py's choice)")
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
        for n, st, batch in [(int(x), k, int(b)) for x in args.ns.split(",")
                             for k in args.streams.split(",") for b in args.batches.split(",")]:
            owned = int(np.sum(pt.owned_pixels(W, H, 0, n)))
            streams = max(1, round(FILL_SLOTS / owned)) if st == "auto" else int(st)
            sb = pt.SampleBuffer(dev, W, H)
            r = pt.BasicRenderer(dev, ds, sb, rank=0, nranks=n, streams=streams)
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
            per_round = {}
            for name, k in (("extend", 1), ("shade", 2), ("round", 5), ("rounds", 6)):
                nk, mk = dev.kernel_stats(k)
                if nk:
                    per_round[name] = round(mk / max(dev.kernel_rounds(k), 1), 4)
            dev.set_profiling(False)
            step_ms = dt / args.steps * 1e3
            rate = (rays1 - rays0) / dt / 1e6
            row = {
                "config": cfg, "frame": f"{W}x{H}", "n_gpus": n, "rank0_pixels": owned, "streams": streams,
                "rank0_slots": r.slot_count, "round_batch": batch,
                "rank0_ms_per_step": round(step_ms, 4),
                "rank0_mrays_per_s": round(rate, 1),
                "kernel_ms_per_round": per_round,
                "predicted_frame_mrays_per_s": round(rate * W * H / owned, 1),
            }
            rows.append(row)
            print(json.dumps(row), flush=True)
            r.close()
            sb.close()
        ds.close()
        scene.close()
    base = {}
    for r in rows:
        if r["n_gpus"] == 1 and r["streams"] == 1:
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
