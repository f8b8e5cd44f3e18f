"""Writes the sort keys of C3's settled rays (3 consecutive rounds, slot
order, u16; 0xFFFF never occurs: every C3 slot is inside the image) to
gpurun_out/gsort_bench/keys.bin for gsort_bench (GPU; the renderer in its
default mode, keys recomputed from the slot rays with RayKey's formula over
the origins' bounding box)."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "tools"))
import kat  # noqa: E402
from exp_gsort import load  # noqa: E402

pt = load()
scene = pt.Scene.config(3)
W, H = scene.info.width, scene.info.height
dev = pt.Device(0)
ds = pt.DeviceScene(dev)
ds.update(scene)
sb = pt.SampleBuffer(dev, W, H)
r = pt.BasicRenderer(dev, ds, sb)
r.RenderFlags = scene.info.render_flags
r.reset()
r.run(2)
for _ in range(30):
    r.run(1)
dev.synchronize()
y, x = np.divmod(np.arange(W * H), W)
slot = ((y // 16) * (W // 16) + x // 16) * 256 + (y % 16) * 16 + x % 16
base = np.argsort(slot, kind="stable")
out = []
for _ in range(3):
    st = r.read_state().reshape(-1)
    O = st["origin"][base].astype(np.float32)
    V = kat.unpack_unit_vector(st["packed_velocity"][base].astype(np.uint32))
    lo, hi = O.min(0), O.max(0)
    c = np.clip(((O - lo) * (np.float32(8) / np.maximum(hi - lo, np.float32(1e-30)))).astype(np.int64), 0, 7)

    def spread(v):
        return (v & 1) | ((v & 2) << 2) | ((v & 4) << 4)

    oct_ = (V[:, 0] < 0).astype(np.int64) | ((V[:, 1] < 0).astype(np.int64) << 1) | ((V[:, 2] < 0).astype(np.int64) << 2)
    k = (oct_ << 9) | spread(c[:, 0]) | (spread(c[:, 1]) << 1) | (spread(c[:, 2]) << 2)
    out.append(k.astype(np.uint16))
    r.run(1)
    dev.synchronize()
d = ROOT / "gpurun_out" / "gsort_bench"
d.mkdir(parents=True, exist_ok=True)
np.concatenate(out).tofile(d / "keys.bin")
print("keys", len(out), len(out[0]), "distinct per round", [len(np.unique(k)) for k in out], flush=True)
for o in (r, sb, ds):
    o.close()
dev.close()
