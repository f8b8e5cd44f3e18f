"""Debug aid: a renderer's schedule against the oracle after every call --
which call first differs, how many pixels and state fields.

usage: python tools/exp_lists_debug.py CONFIG W H r2,b6,r1,b4 [SPLIT]
       (r = run(k), b = run_rounds(k); SPLIT: tile groups, default 3)"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import __graft_entry__ as ge  # noqa: E402
import oracle_lib  # noqa: E402


def main():
    pt = ge._load_package()
    config, W, H = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    sched = sys.argv[4].split(",")   # e.g. r2,b6,r1,b4  (r = run(k), b = run_rounds(k))
    split = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    s = pt.Scene.config(config)
    dev = pt.Device(0)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    r.RenderFlags = 3
    r.set_fused_rounds(0)
    r.set_split(split)
    print("class lists", r.class_lists(), "split", r.split(), flush=True)
    o = oracle_lib.OracleRenderer(s.packs(), W, H)
    o.RenderFlags = 3
    r.reset()
    o.reset()
    for step in sched:
        k = int(step[1:])
        if step[0] == "r":
            r.run(k)
            o.run(k)
        else:
            r.run_rounds(k)
            for _ in range(k):
                o.run(1)
        dev.synchronize()
        ga, oa = sb.read(), o.accum()
        gs, os_ = r.read_state(), o.state()
        dw = np.argwhere(ga[..., 3] != oa[..., 3])
        dx = np.argwhere(np.any(ga[..., :3].view(np.uint32) != oa[..., :3].view(np.uint32), axis=-1))
        dst = {f: int(np.sum(np.any((gs[f].view(np.uint32) != os_[f].view(np.uint32)).reshape(H, W, -1), axis=-1)))
               for f in ("origin", "throughput", "probability", "lambda0", "packed_velocity")}
        print(step, "count diffs", len(dw), dw[:6].tolist(), "xyz diffs", len(dx), "state diffs", dst,
              "stats", r.stats(), o.counters(), flush=True)
    for x in (r, sb, ds, dev):
        x.close()


if __name__ == "__main__":
    main()
