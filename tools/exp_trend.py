"""C3 throughput by round block after Reset + Run(2) (no profiling events):
how the path population's mix changes the cost of a round."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))
from exp_reorder import load  # noqa: E402

pt = load()
dev = pt.Device(0)
scene = pt.Scene.config(3)
info = scene.info
ds = pt.DeviceScene(dev)
ds.update(scene)
sb = pt.SampleBuffer(dev, info.width, info.height)
r = pt.BasicRenderer(dev, ds, sb)
r.RenderFlags = info.render_flags
r.PathTerminationProbability = info.termination_probability
r.reset()
r.run(2)
dev.synchronize()
done = 2
for blk in range(12):
    t0 = time.perf_counter()
    for _ in range(32):
        r.run(1)
    dev.synchronize()
    dt = time.perf_counter() - t0
    print(f"rounds {done}-{done + 32}: {info.width * info.height * 32 / dt / 1e6:.1f} Mrays/s", flush=True)
    done += 32
