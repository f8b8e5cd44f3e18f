"""Measurements of the SURVEY.md §8(f) rows built beside the hot path.

* resolve (RenderSampleBuffer, resolve.hip): XYZ accumulator -> tone-mapped
  sRGB, per pixel 16 B read + 16 B float4 colour + 4 B sRGB8 written = 36 B;
  GB/s against the 8 TB/s HBM roofline, every tone-mapping mode, at C3's
  1920x1080 and C4's 3840x2160.
* preview (RenderPreview, preview.hip): one primary ray per pixel through
  the device traversal plus the AOV / pick write-back; Mrays/s per render
  mode on C3 and C5 at 1920x1080.
* OpenPBR shading (opt-in, §6 row 4): Mrays/s of the layered OpenPBR scene
  of tests/test_openpbr.py at 1920x1080, shaded, against the same scene with
  OpenPBR hits ending the path (the reference's behaviour).
* host builds (§8(f) row 3): mesh BVH build of a 1.96 M-face mesh on 1 and
  on all of the job's threads, and the RGB -> spectrum table.

Kernel times are HIP events on the device stream (ptGetKernelStats).
Prints one JSON object.
"""
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))
sys.path.insert(0, str(ROOT / "tests"))
from exp_reorder import load  # noqa: E402

HBM_GBPS = 8000.0
K_RESOLVE, K_PREVIEW, K_EXTEND, K_SHADE, K_ROUND = 3, 4, 1, 2, 5


def timed(dev, kernel, fn, reps):
    dev.synchronize()
    dev.reset_kernel_stats()
    dev.set_profiling(True, period=1)
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    dev.synchronize()
    wall = time.perf_counter() - t0
    n, ms = dev.kernel_stats(kernel)
    dev.set_profiling(False)
    return ms / max(n, 1), wall / reps * 1e3


def resolve(pt, dev):
    out = {}
    scene = pt.Scene.config(3)
    ds = pt.DeviceScene(dev)
    ds.update(scene)
    for W, H in ((1920, 1080), (3840, 2160)):
        sb = pt.SampleBuffer(dev, W, H)
        r = pt.BasicRenderer(dev, ds, sb)
        r.RenderFlags = 3
        r.reset()
        r.run(4)
        for mode, name in ((pt.TONE_MAPPING_CLAMP, "clamp"), (pt.TONE_MAPPING_REINHARD, "reinhard"),
                           (pt.TONE_MAPPING_HABLE, "hable"), (pt.TONE_MAPPING_ACES, "aces")):
            sb.render(ToneMappingMode=mode)   # warm
            ms, _ = timed(dev, K_RESOLVE, lambda: sb.render(ToneMappingMode=mode, Brightness=1.3), 50)
            gbps = 36.0 * W * H / (ms * 1e-3) / 1e9
            out[f"{W}x{H}_{name}"] = {"ms": round(ms, 4), "gbps": round(gbps, 1), "frac": round(gbps / HBM_GBPS, 3)}
        r.close()
        sb.close()
    ds.close()
    return out


def preview(pt, dev):
    out = {}
    modes = {"base_color": pt.PREVIEW_RENDER_MODE_BASE_COLOR, "shaded": pt.PREVIEW_RENDER_MODE_BASE_COLOR_SHADED,
             "normal": pt.PREVIEW_RENDER_MODE_NORMAL, "mesh_complexity": pt.PREVIEW_RENDER_MODE_MESH_COMPLEXITY}
    for cid in (3, 5):
        s = pt.Scene.config(cid)
        ds = pt.DeviceScene(dev)
        ds.update(s)
        cam = s.arrays()["cameras"][0]["Transform"]["To"]
        ctx = pt.PreviewRenderContext(dev, ds)
        for name, mode in modes.items():
            p = pt.PreviewParameters(cam, RenderMode=mode, RenderSizeX=1920, RenderSizeY=1080, MouseX=960, MouseY=540)
            ctx.render(p)
            ms, _ = timed(dev, K_PREVIEW, lambda: ctx.render(p), 30)
            out[f"C{cid}_{name}"] = {"ms": round(ms, 4), "mrays_per_s": round(1920 * 1080 / (ms * 1e-3) / 1e6, 1)}
        ctx.close()
        ds.close()
        s.close()
    return out


def openpbr(pt, dev):
    import test_openpbr
    s = test_openpbr.openpbr_scene(pt)
    out = {}
    W, H = 1920, 1080
    for shaded in (True, False):
        ds = pt.DeviceScene(dev)
        ds.update(s)
        sb = pt.SampleBuffer(dev, W, H)
        r = pt.BasicRenderer(dev, ds, sb)
        r.RenderFlags = 3
        r.set_openpbr(shaded)
        r.reset()
        r.run(2)
        r.run(16)
        dev.synchronize()
        rays0, _ = r.stats()
        dev.reset_kernel_stats()
        dev.set_profiling(True, period=1)
        t0 = time.perf_counter()
        for _ in range(32):
            r.run(1)
        dev.synchronize()
        dt = time.perf_counter() - t0
        rays1, _ = r.stats()
        ke = {k: dev.kernel_stats(i) for k, i in (("extend", K_EXTEND), ("shade", K_SHADE), ("round", K_ROUND))}
        dev.set_profiling(False)
        out["openpbr_shaded" if shaded else "openpbr_ends_path"] = {
            "mrays_per_s": round((rays1 - rays0) / dt / 1e6, 1),
            "ms": {k: round(v[1] / v[0], 4) for k, v in ke.items() if v[0]}}
        for x in (r, sb, ds):
            x.close()
    s.close()
    return out


def host_builds(pt):
    import fuzz_scenes
    out = {}
    rng = np.random.default_rng(0)
    mesh = fuzz_scenes.blob_mesh(rng, 700, 1400, 0.05)
    threads = os.environ.get("OMP_NUM_THREADS") or str(os.cpu_count())
    for t in ("1", threads):
        os.environ["PT_BVH_THREADS"] = t
        s = pt.Scene.empty()
        t0 = time.perf_counter()
        s.create_mesh(*mesh)
        out[f"bvh_{len(mesh[1])}_faces_threads_{t}_s"] = round(time.perf_counter() - t0, 3)
        s.close()
    os.environ.pop("PT_BVH_THREADS", None)
    t0 = time.perf_counter()
    pt.build_spectrum_table(None, int(threads))
    out[f"spectrum_table_threads_{threads}_s"] = round(time.perf_counter() - t0, 2)
    return out


def main():
    pt = load()
    dev = pt.Device(0)
    res = {"resolve": resolve(pt, dev), "preview": preview(pt, dev), "openpbr": openpbr(pt, dev)}
    dev.close()
    res["host"] = host_builds(pt)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
