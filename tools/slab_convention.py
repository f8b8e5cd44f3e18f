"""What the reciprocal slab-test convention changes against IEEE division.

The device and the oracle evaluate the slab test's (Min - O) / V
(common.glsl.inc:157-158) as correctly rounded IEEE division, the convention
SURVEY.md §7/§8(c) wrote down (the device reaches it through an
FMA-corrected reciprocal).  Round 2 had used the reciprocal form
RN((Min - O) * RN(1/V)); it is kept in the oracle only for this measurement
(oracle_set_slab_division(0)), which showed it is not a conforming
restatement.  This script runs the CPU oracle in both conventions on the same
inputs and reports, per scene:

* rays:  hit-record differences over 20 000 random rays (the parity tests'
  generator) and over the path rays of a rendered frame (each slot's next ray
  after rounds 1, 2, 4, 8, 16 of the rcp-convention render), each difference
  classed as an exact tie (same hit time bits, another primitive) or not
  (time differs: by how many ulps);
* state: pixels whose slot state differs after Reset / Run(2) / Run(1);
* image: relative L2 between the two accumulators after Reset / Run(2) /
  14 x Run(1) (16 rounds), and the count of differing pixels.

CPU only (test infrastructure: the oracle).  Usage:
  python tools/slab_convention.py [--out profiles/r03_slab/slab_convention.json] [--quick]
"""
from __future__ import annotations

import argparse
import concurrent.futures
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tests"))
import conftest  # noqa: E402,F401  (package import + spectrum table path)
import fuzz_scenes  # noqa: E402
import oracle_lib  # noqa: E402
from rays import random_rays  # noqa: E402

THREADS = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))


def trace(packs, o, v, d, mode):
    """oracle_trace_rays in `mode`, chunked over threads (ctypes drops the GIL)."""
    n = len(v)
    chunks = np.array_split(np.arange(n), max(1, min(THREADS, n // 4096 + 1)))
    with oracle_lib.slab_division(mode):
        with concurrent.futures.ThreadPoolExecutor(len(chunks)) as ex:
            parts = list(ex.map(lambda c: oracle_lib.trace_rays(packs, o[c], v[c], d[c]), chunks))
    return np.concatenate(parts)


def ulp_distance(a, b):
    """|a - b| in float32 ulps (same-sign finite values)."""
    ia = a.view(np.int32).astype(np.int64)
    ib = b.view(np.int32).astype(np.int64)
    ia = np.where(ia < 0, -(ia & 0x7FFFFFFF), ia)
    ib = np.where(ib < 0, -(ib & 0x7FFFFFFF), ib)
    return np.abs(ia - ib)


def compare_hit_sets(a, b):
    """Differences between two hit-record arrays: counts and classes."""
    sm = a["shape_material"] != b["shape_material"]
    both = (a["shape_material"] != 0xFFFFFFFF) & (b["shape_material"] != 0xFFFFFFFF)
    fields = np.zeros(len(a), bool)
    for f in ("time", "packed_normal", "packed_tangent", "u", "v"):
        fields |= both & (a[f].view(np.uint32) != b[f].view(np.uint32))
    differ = sm | fields
    idx = np.flatnonzero(differ)
    hit_miss = int(np.sum(sm & ~both))
    same_time = both & (a["time"].view(np.uint32) == b["time"].view(np.uint32))
    ties = int(np.sum(differ & same_time))
    nontie = differ & both & ~same_time
    ulps = ulp_distance(a["time"][nontie], b["time"][nontie]) if nontie.any() else np.zeros(0, np.int64)
    return {
        "rays": int(len(a)),
        "differ": int(idx.size),
        "differ_frac": float(idx.size / max(len(a), 1)),
        "exact_ties": ties,
        "hit_vs_miss": hit_miss,
        "time_differs": int(nontie.sum()),
        "time_ulps_max": int(ulps.max()) if ulps.size else 0,
        "time_ulps_hist": {str(k): int(c) for k, c in zip(*np.unique(np.minimum(ulps, 100), return_counts=True))},
        "first": idx[:4].tolist(),
    }


def state_diff(a, b):
    """Pixels whose slot state differs in any field (bitwise)."""
    return int(np.sum(np.any(a.view(np.uint8).reshape(a.size, -1) != b.view(np.uint8).reshape(b.size, -1), axis=1)))


def render(packs, W, H, schedule, mode, flags=3, termination=0.0, camera=0):
    with oracle_lib.slab_division(mode):
        o = oracle_lib.OracleRenderer(packs, W, H, threads=THREADS)
        o.RenderFlags = flags
        o.PathTerminationProbability = termination
        o.CameraIndex = camera
        o.reset()
        states = []
        for r in schedule:
            o.run(r)
            states.append(o.state())
        acc = o.accum()
        o.close()
    return states, acc


def measure_scene(packs, arrays, W, H, rounds, flags=3, termination=0.0, ray_seed=0, n_random=20000,
                  path_rounds=(1, 2, 4, 8, 16)):
    out = {"frame": [W, H], "rounds": rounds}
    o, v, d = random_rays(arrays, n_random, seed=ray_seed)
    out["random_rays"] = compare_hit_sets(trace(packs, o, v, d, "rcp"), trace(packs, o, v, d, "ieee"))

    schedule = [2] + [1] * (rounds - 2)
    st_r, acc_r = render(packs, W, H, schedule, "rcp", flags, termination)
    st_i, acc_i = render(packs, W, H, schedule, "ieee", flags, termination)
    out["state_after_reset_run2_run1"] = {"pixels": W * H, "differ": state_diff(st_r[1], st_i[1])}
    out["state_after_all_rounds"] = {"pixels": W * H, "differ": state_diff(st_r[-1], st_i[-1])}
    # per-round pixel divergence curve (round index = rounds completed)
    curve = {}
    done = 2
    for k, (a, b) in enumerate(zip(st_r, st_i)):
        curve[str(done)] = state_diff(a, b)
        done += 1
    out["state_differ_by_round"] = curve
    rel = float(np.linalg.norm(acc_r - acc_i) / max(np.linalg.norm(acc_r), 1e-30))
    out["image"] = {"rel_l2": rel, "pixels_differ": int(np.sum(np.any(acc_r != acc_i, axis=-1))),
                    "samples": float(acc_r[..., 3].sum())}

    # Path rays: every slot's next ray after the listed rounds of the rcp render.
    dur = np.full(W * H, 1048576.0, np.float32)
    agg = None
    per = {}
    done = 2
    for k, s in enumerate(st_r):
        if done in path_rounds:
            po = np.ascontiguousarray(s["origin"].reshape(-1, 3))
            pv = np.ascontiguousarray(s["packed_velocity"].reshape(-1))
            c = compare_hit_sets(trace(packs, po, pv, dur, "rcp"), trace(packs, po, pv, dur, "ieee"))
            per[str(done)] = c
            if agg is None:
                agg = {k2: c[k2] for k2 in ("rays", "differ", "exact_ties", "hit_vs_miss", "time_differs")}
                agg["time_ulps_max"] = c["time_ulps_max"]
            else:
                for k2 in ("rays", "differ", "exact_ties", "hit_vs_miss", "time_differs"):
                    agg[k2] += c[k2]
                agg["time_ulps_max"] = max(agg["time_ulps_max"], c["time_ulps_max"])
        done += 1
    if agg:
        agg["differ_frac"] = agg["differ"] / max(agg["rays"], 1)
    out["path_rays"] = {"total": agg, "by_round": per}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=str(ROOT / "profiles" / "r03_slab" / "slab_convention.json"))
    ap.add_argument("--quick", action="store_true", help="reduced frames (CPU test sizes)")
    ap.add_argument("--configs", default="1,2,3,5")
    ap.add_argument("--fuzz", type=int, default=24)
    args = ap.parse_args()
    pt = conftest.load_package()
    full = {1: (256, 256), 2: (1024, 1024), 3: (1920, 1080), 5: (2048, 1024)}
    quick = {1: (64, 64), 2: (96, 96), 3: (160, 90), 5: (128, 64)}
    sizes = quick if args.quick else full
    res = {"threads": THREADS, "scenes": {}}
    for c in [int(x) for x in args.configs.split(",") if x]:
        t0 = time.time()
        s = pt.Scene.config(c)
        W, H = sizes[c]
        res["scenes"][f"C{c}"] = measure_scene(s.packs(), s.arrays(), W, H, 16, ray_seed=c)
        res["scenes"][f"C{c}"]["seconds"] = round(time.time() - t0, 1)
        print(f"C{c}", json.dumps(res["scenes"][f"C{c}"]["image"]), res["scenes"][f"C{c}"]["random_rays"]["differ"],
              res["scenes"][f"C{c}"]["path_rays"]["total"]["differ"], flush=True)
        s.close()
    for seed in range(args.fuzz):
        s, st = fuzz_scenes.build(pt, seed)
        W, H = (72, 40) if seed % 3 else (33, 17)
        r = measure_scene(s.packs(), s.arrays(), W, H, 16, flags=st["flags"], termination=st["termination"],
                          ray_seed=seed, n_random=8192)
        res["scenes"][f"fuzz{seed}"] = r
        print(f"fuzz{seed}", json.dumps(r["image"]), r["random_rays"]["differ"], r["path_rays"]["total"]["differ"],
              flush=True)
        s.close()
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    Path(args.out).write_text(json.dumps(res, indent=1))
    print("wrote", args.out)


if __name__ == "__main__":
    main()
