"""Shade branch occupancy (VERDICT r03 "next" #1, step 1): how many lanes of a
wave are active in each branch of Scatter (basic_scatter.glsl:44-360).

Needs the experiment build:  python tools/build_variant.py shadestats -DPT_SHADE_STATS=1
usage (GPU box):  python tools/shade_stats.py OUT.json [CONFIG ...]

For each config: Reset, Run(2), SETTLE rounds, then the counters of ROUNDS
shade launches.  Per mark k (kernels.hip SM_*): waves = wave executions that
reached it, lanes = active lanes summed over them; lanes / waves = the mark's
mean SIMD occupancy (of 64), waves / waves(entry) = how often a wave runs it.
"""
import ctypes as C
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
VARIANT = Path(os.environ.get("PT_STATS_LIB", ROOT / "build" / "variants" / "shadestats.so"))
os.environ["PT_HIP_LIB"] = str(VARIANT)
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402  (package loader)

MARKS = ["entry", "hit", "escape", "medium_event", "surface", "real", "light", "light_below",
         "diffuse_cosine", "diffuse_eval", "metal_eval", "metal_sample", "trans_eval", "trans_sample",
         "trans_reflect", "trans_refract", "openpbr", "not_real", "roulette", "completed", "continue",
         "exterior_medium", "mesh_hit", "sphere_hit", "cube_hit", "plane_hit"]
SETTLE, ROUNDS = 32, 32


def main():
    out_path = sys.argv[1]
    configs = [int(c) for c in sys.argv[2:]] or [2, 3, 5]
    pt = bench.load_package()
    lib = pt._native.hip_lib()
    fn = lib.ptShadeStatsRead
    fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    fn.restype = C.c_int
    buf = (C.c_ulonglong * 64)()
    res = {}
    dev = pt.Device(0)
    for cfg in configs:
        scene = pt.Scene.config(cfg)
        info = scene.info
        ds = pt.DeviceScene(dev)
        ds.update(scene)
        sb = pt.SampleBuffer(dev, info.width, info.height)
        r = pt.BasicRenderer(dev, ds, sb)
        r.set_fused_rounds(0)
        r.RenderFlags = info.render_flags
        r.PathTerminationProbability = info.termination_probability
        r.reset()
        r.run(2)
        for _ in range(SETTLE):
            r.run(1)
        dev.synchronize()
        n = fn(None, 1)
        assert n == len(MARKS), (n, len(MARKS))
        for _ in range(ROUNDS):
            r.run(1)
        dev.synchronize()
        fn(buf, 1)
        entry_waves = max(buf[0], 1)
        rows = {}
        for k, name in enumerate(MARKS):
            w, l = int(buf[2 * k]), int(buf[2 * k + 1])
            rows[name] = {"waves": w, "lanes": l, "lanes_per_wave": round(l / w, 2) if w else None,
                          "wave_frac": round(w / entry_waves, 4)}
        res[f"C{cfg}"] = {"width": info.width, "height": info.height, "rounds": ROUNDS, "marks": rows}
        print(f"C{cfg} {info.width}x{info.height}, {ROUNDS} rounds after {SETTLE + 2}")
        print(f"  {'mark':16s} {'waves/entry':>11s} {'lanes/wave':>10s} {'lanes/entry-lanes':>17s}")
        el = max(rows["entry"]["lanes"], 1)
        for name, v in rows.items():
            if v["waves"]:
                print(f"  {name:16s} {v['wave_frac']:11.4f} {v['lanes_per_wave']:10.2f} {v['lanes'] / el:17.4f}")
        for x in (r, sb, ds):
            x.close()
    dev.close()
    Path(out_path).parent.mkdir(parents=True, exist_ok=True)
    Path(out_path).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
