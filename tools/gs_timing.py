"""Per-round timing of the renderer at full C3 size (GPU), with kernel stats."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tests"))
import conftest  # noqa: E402

pt = conftest.load_package()
dev = pt.Device(0)
cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
s = pt.Scene.config(cfg)
W, H = s.info.width, s.info.height
ds = pt.DeviceScene(dev)
ds.update(s)
sb = pt.SampleBuffer(dev, W, H)
r = pt.BasicRenderer(dev, ds, sb)
r.RenderFlags = 3
dev.set_profiling(True, period=1)
t0 = time.time()
r.reset()
dev.synchronize()
print(f"reset {time.time()-t0:.4f}s", flush=True)
for i in range(40):
    dev.reset_kernel_stats()
    t0 = time.time()
    r.run(2 if i == 0 else 1)
    dev.synchronize()
    dt = time.time() - t0
    ks = {k: dev.kernel_stats(v) for k, v in (("ext", 1), ("sh", 2), ("sort", 6))}
    if i < 6 or i % 8 == 0:
        print(i, f"{dt*1e3:.3f} ms", {k: round(v[1] / max(v[0], 1), 4) for k, v in ks.items()}, r.stats(), flush=True)
