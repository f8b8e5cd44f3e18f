"""Experiment: what would a step-budget split's second pass cost?

A budget of K traversal steps per ray in the extend kernel (experiment build
PT_EXP_STEP_CAP) cut C3 extend from 0.325 to 0.241 ms at K=40
(profiles/r02_stepcap).  The rays cut off ("stragglers") would have to finish
in a second, compacted pass before shade.  This script renders C3 to a
settled state, takes the rays whose traversal exceeds K steps, and traces
them -- compacted, in slot order, from the start (so the time is an upper
bound of a resumed pass) -- through ptTraceRays (the production extend
kernel over caller arrays).  Run it under `rocprofv3 --kernel-trace`;
tools/exp_reorder_report.py-style matching is done by exp_straggler_report
below (dispatches in call order).
"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))
from exp_predict import positions  # noqa: E402
from exp_reorder import load  # noqa: E402


def main():
    pt = load()
    dev = pt.Device(0)
    scene = pt.Scene.config(3)
    info = scene.info
    W, H = info.width, info.height
    ds = pt.DeviceScene(dev)
    ds.update(scene)
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    r.RenderFlags = info.render_flags
    r.reset()
    r.run(2)
    r.run(40)
    dev.synchronize()
    st = r.read_state()
    steps_pos = r.extend_step_counts().astype(np.int64)
    pix = positions(W, H, st)                      # per position: pixel (or -1)
    valid = pix >= 0
    steps = np.zeros(W * H, np.int64)
    steps[pix[valid]] = steps_pos[valid]
    # slot order of the pixels (tile-major), the layout the extend kernel sees
    y, x = np.divmod(np.arange(W * H), W)
    slot = ((y // 16) * (W // 16) + x // 16) * 256 + (y % 16) * 16 + x % 16
    order = np.argsort(slot, kind="stable")
    O = st["origin"].reshape(-1, 3)[order].astype(np.float32)
    PV = st["packed_velocity"].reshape(-1)[order].astype(np.uint32)
    S = steps[order]
    log = []
    cases = [("all", np.ones(len(S), bool))] + [(f"K{k}", S > k) for k in (24, 32, 40, 48, 63)]
    for name, m in cases:
        n = int(m.sum())
        o, v = O[m], PV[m]
        pad = (-n) % 256                                   # whole blocks: repeat the last ray
        if pad:
            o = np.concatenate([o, np.repeat(o[-1:], pad, 0)])
            v = np.concatenate([v, np.repeat(v[-1:], pad)])
        d = np.full(len(v), 1048576.0, np.float32)
        rem = int(np.maximum(S[m] - int(name[1:]) if name != "all" else S[m], 0).sum())
        for k in range(3):
            ds.trace_rays(o, v, d)
            log.append({"case": name, "rep": k, "rays": n, "max_steps": int(S[m].max()) if n else 0,
                        "remaining_lane_steps": rem})
        print(name, n, "rays; max steps", int(S[m].max()) if n else 0, "; remaining lane steps", rem, flush=True)
    (ROOT / "gpurun_out").mkdir(exist_ok=True)
    (ROOT / "gpurun_out" / "exp_straggler_cases.json").write_text(json.dumps(log))
    for o_ in (r, sb, ds):
        o_.close()
    dev.close()


def report(trace_dir):
    import csv
    import glob
    from collections import defaultdict
    cases = json.load(open(ROOT / "gpurun_out" / "exp_straggler_cases.json"))
    rows = []
    for f in glob.glob(f"{trace_dir}/**/*kernel_trace.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if "extend_kernel" in row["Kernel_Name"] and "ray_source_arrays" in row["Kernel_Name"]:
                rows.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
    rows.sort()
    rows = rows[-len(cases):]
    acc = defaultdict(list)
    meta = {}
    for c, (s, e) in zip(cases, rows):
        acc[c["case"]].append((e - s) / 1e6)
        meta[c["case"]] = c
    for k, v in acc.items():
        print(f"{k:5s} rays {meta[k]['rays']:8d} max_steps {meta[k]['max_steps']:4d} "
              f"remaining {meta[k]['remaining_lane_steps']:9d}  best {min(v):.4f} ms  mean {sum(v) / len(v):.4f} ms")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "report":
        report(sys.argv[2])
    else:
        main()
