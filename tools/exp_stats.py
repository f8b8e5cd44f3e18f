"""Prints ptExtendStats (traversal counters, wave coherence) for configs 1-5
after Reset + Run(2) + 8 rounds."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))
from exp_reorder import load  # noqa: E402

pt = load()
dev = pt.Device(0)
for cid in [int(c) for c in (sys.argv[1:] or ["1", "2", "3", "5"])]:
    scene = pt.Scene.config(cid)
    info = scene.info
    ds = pt.DeviceScene(dev)
    ds.update(scene)
    sb = pt.SampleBuffer(dev, info.width, info.height)
    r = pt.BasicRenderer(dev, ds, sb)
    r.RenderFlags = info.render_flags
    r.PathTerminationProbability = info.termination_probability
    r.reset()
    r.run(10)
    d = r.extend_stats()
    tot = sum(d[k] for k in d if k.startswith("blas_steps_distinct"))
    d["blas_wave_steps"] = tot
    for k in [k for k in d if k.startswith("blas_steps_distinct")]:
        d[k + "_frac"] = round(d[k] / max(tot, 1), 4)
    print(f"C{cid}", json.dumps(d), flush=True)
    for o in (r, sb, ds):
        o.close()
dev.close()
