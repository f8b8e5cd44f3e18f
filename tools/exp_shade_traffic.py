"""Shade HBM-traffic attribution (GPU experiment, run under rocprofv3 --pmc).

Renders C3 like bench.py (Reset + Run(2) + settle rounds, then --steps
single rounds) in one of these variants, so that separate FETCH_SIZE /
WRITE_SIZE passes per variant split shade's bytes by source:
  base      the bench workload
  notex     every material's texture slot set to none (no atlas gathers;
            the packed material words are patched before upload)
  noaccum   RenderFlags = JITTER only (the accumulator is overwritten,
            not read-modify-written)
  notex_noaccum  both
usage: python tools/exp_shade_traffic.py VARIANT [--steps 8]
"""
import argparse
import ctypes as C
import importlib.util
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
    ap.add_argument("variant", choices=["base", "notex", "noaccum", "notex_noaccum"])
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--config", type=int, default=3)
    args = ap.parse_args()
    pt = load_package()
    from path_tracer_amd import _native as N
    scene = pt.Scene.config(args.config)
    W, H = scene.info.width, scene.info.height
    dev = pt.Device(0)
    ds = pt.DeviceScene(dev)
    packs = scene.packs()
    keep = None
    if "notex" in args.variant:
        words = np.ctypeslib.as_array(C.cast(packs.material_data, C.POINTER(C.c_uint32)),
                                      shape=(packs.material_word_count,)).copy().reshape(-1, 32)
        words[:, 1 + 3] = 0xFFFFFFFF        # PT_BASIC_DIFFUSE_BASE_SPECTRUM + 3: base texture index
        keep = np.ascontiguousarray(words.reshape(-1))
        packs.material_data = keep.ctypes.data
    ds.update(packs)
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    r.RenderFlags = pt.RENDER_FLAG_SAMPLE_JITTER if "noaccum" in args.variant else scene.info.render_flags
    r.reset()
    r.run(2)
    r.run(32)
    for _ in range(args.steps):
        r.run(1)
    dev.synchronize()
    rays, samples = r.stats()
    print(f"{args.variant}: {rays} rays, {samples} samples")
    for x in (r, sb, ds):
        x.close()
    dev.close()
    scene.close()


if __name__ == "__main__":
    main()
