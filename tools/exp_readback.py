"""Host hand-over cost of a frame (PCIe-inclusive rate, north_star / DESIGN §4).

The benchmark times frames whose output stays in HBM (the reference displays
its sample buffer through Vulkan and never reads it back).  A caller that
wants the frame on the host reads the accumulator (rgba32f, 16 B/px:
ptReadSampleBuffer) or resolves it and reads 8-bit sRGB (4 B/px:
ptRenderSampleBuffer + ptReadResolvedImageSRGB8).  This times both after
whole C3 frames and reports the frame rate with each hand-over included.

usage: python tools/exp_readback.py [CONFIG] [FRAMES] [OUT.json]
"""
import json
import math
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    import bench
    config = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    out = sys.argv[3] if len(sys.argv) > 3 else None
    pt = bench.load_package()
    scene = pt.Scene.config(config)
    info = scene.info
    W, H, spp = info.width, info.height, info.spp
    dev = pt.Device(0)
    ds = pt.DeviceScene(dev)
    ds.update(scene)
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    r.RenderFlags = info.render_flags
    r.PathTerminationProbability = info.termination_probability
    target = spp * W * H
    rec = {"config": config, "width": W, "height": H, "spp": spp, "frames": []}
    r.render_frame(target)          # warm-up frame (and first-touch of the host buffers below)
    sb.read()
    sb.render()
    sb.read_srgb8()
    dev.synchronize()
    for _ in range(frames):
        t0 = time.perf_counter()
        rounds, samples = r.render_frame(target)
        dev.synchronize()
        t1 = time.perf_counter()
        a = sb.read()
        t2 = time.perf_counter()
        sb.render()
        img = sb.read_srgb8()
        t3 = time.perf_counter()
        rays = rounds * W * H   # one slot per pixel (the bench counts owned pixels, not tile padding)
        rec["frames"].append({"rounds": rounds, "frame_s": t1 - t0, "read_rgba32f_s": t2 - t1,
                              "resolve_read_srgb8_s": t3 - t2, "rays": rays,
                              "accum_bytes": int(a.nbytes), "srgb8_bytes": int(img.nbytes)})
    f = rec["frames"]
    fs = sum(x["frame_s"] for x in f)
    rays = sum(x["rays"] for x in f)
    ra = sum(x["read_rgba32f_s"] for x in f)
    rs = sum(x["resolve_read_srgb8_s"] for x in f)
    rec["mrays_per_s_resident"] = round(rays / fs / 1e6, 1)
    rec["mrays_per_s_with_rgba32f_read"] = round(rays / (fs + ra) / 1e6, 1)
    rec["mrays_per_s_with_srgb8_read"] = round(rays / (fs + rs) / 1e6, 1)
    rec["rgba32f_read_gbps"] = round(f[0]["accum_bytes"] * len(f) / ra / 1e9, 2)
    rec["srgb8_read_ms"] = round(rs / len(f) * 1e3, 3)
    rec["rgba32f_read_ms"] = round(ra / len(f) * 1e3, 3)
    print(json.dumps(rec), flush=True)
    if out:
        Path(out).write_text(json.dumps(rec, indent=1))
    r.close(); sb.close(); ds.close(); dev.close()
    assert math.isfinite(rec["mrays_per_s_resident"])


if __name__ == "__main__":
    main()
