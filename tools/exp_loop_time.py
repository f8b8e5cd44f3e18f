"""Times C3 rounds without profiling events: Mrays/s (best of 3 x 64 rounds).

Used for the multi-stream tile-range experiment recorded in DESIGN.md (the
PT_RUN_PARTS code was removed after it measured slower) and for checking the
cost of the kernel-timing events."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))
from exp_reorder import load  # noqa: E402

pt = load()
dev = pt.Device(0)
cid = int(sys.argv[1]) if len(sys.argv) > 1 else 3
scene = pt.Scene.config(cid)
info = scene.info
ds = pt.DeviceScene(dev)
ds.update(scene)
sb = pt.SampleBuffer(dev, info.width, info.height)
r = pt.BasicRenderer(dev, ds, sb)
r.RenderFlags = info.render_flags
r.PathTerminationProbability = info.termination_probability
r.reset()
r.run(2)
for _ in range(8):
    r.run(1)
dev.synchronize()
best = 0.0
for rep in range(3):
    t0 = time.perf_counter()
    for _ in range(64):
        r.run(1)
    dev.synchronize()
    dt = time.perf_counter() - t0
    best = max(best, info.width * info.height * 64 / dt / 1e6)
print(f"C{cid} Mrays/s {best:.1f}", flush=True)
