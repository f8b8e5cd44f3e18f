"""Debug: the global-sort renderer against the oracle on small frames (GPU)."""
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tests"))
import conftest  # noqa: E402
import oracle_lib  # noqa: E402

pt = conftest.load_package()
dev = pt.Device(0)
for cfg, W, H in ((1, 64, 64), (3, 160, 90)):
    s = pt.Scene.config(cfg)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    r.set_fused_rounds(0)
    o = oracle_lib.OracleRenderer(s.packs(), W, H)
    for x in (r, o):
        x.RenderFlags = 3
        x.reset()
    dev.synchronize()
    print("reset ok", flush=True)
    for i, rounds in enumerate([2, 1, 1]):
        t0 = time.time()
        r.run(rounds)
        dev.synchronize()
        o.run(rounds)
        gs, os_ = r.read_state(), o.state()
        print(cfg, "run", rounds, f"{time.time()-t0:.2f}s", "stats", r.stats(), "oracle", o.counters(), flush=True)
        for f in ("origin", "packed_velocity", "throughput", "probability", "lambda0"):
            bad = np.argwhere(gs[f].view(np.uint32).reshape(H, W, -1).any(-1) != o.state()[f].view(np.uint32).reshape(H, W, -1).any(-1)) if False else None
            d = (gs[f].view(np.uint32) != os_[f].view(np.uint32)).reshape(H, W, -1).any(-1)
            print("  ", f, "differ px", int(d.sum()), np.argwhere(d)[:3].tolist(), flush=True)
        hd = (gs["hit"]["shape_material"] != os_["hit"]["shape_material"])
        print("   hit shape differ", int(hd.sum()), flush=True)
    a, b = sb.read(), o.accum()
    print("accum equal", bool(np.array_equal(a.view(np.uint32), b.view(np.uint32))), flush=True)
    for x in (r, sb, ds):
        x.close()
