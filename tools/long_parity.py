"""Long-run parity check: a config at its full size over Reset + Run(2) +
(rounds - 2) x Run(1) (default C3 1920x1080, 64 rounds: four tile-order
re-sorts, the path population turned over many times; round 3 ran 700
rounds, about a 256-spp frame), every slot's state and every accumulated
pixel compared with the CPU oracle bit for bit.  Prints one JSON line.

A random scene of tests/fuzz_scenes.py runs as CONFIG "fuzz:SEED" at
320x240 with the seed's RenderFlags, roulette and camera.

usage: python tools/long_parity.py [CONFIG | fuzz:SEED] [ROUNDS] [CAMERA] [--batched] [--split K]"""
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
import oracle_lib  # noqa: E402


def main():
    # --batched: the GPU side runs its Run(1) rounds through
    # ptRunBasicRendererRounds in chunks of 50 (tile groups on concurrent
    # streams on full frames); the oracle runs the same rounds one by one.
    batched = "--batched" in sys.argv
    if batched:
        sys.argv.remove("--batched")
    split = 0   # --split K: force K tile groups (0: automatic)
    if "--split" in sys.argv:
        i = sys.argv.index("--split")
        split = int(sys.argv[i + 1])
        del sys.argv[i:i + 2]
    pt = load()
    cfg = sys.argv[1] if len(sys.argv) > 1 else "3"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    if cfg.startswith("fuzz:"):
        import fuzz_scenes
        s, st = fuzz_scenes.build(pt, int(cfg[5:]))
        W, H, flags, ptp, camera = 320, 240, st["flags"], st["termination"], st["camera"]
    else:
        cfg = int(cfg)
        s = pt.Scene.config(cfg)
        info = s.info
        W, H, flags, ptp, camera = info.width, info.height, info.render_flags, info.termination_probability, 0
        if len(sys.argv) > 3:
            camera = int(sys.argv[3])
    dev = pt.Device(0)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    r.set_split(split)
    if split > 1:
        r.set_fused_rounds(0)   # forced groups: the small frames' rounds would otherwise run fused
    # The oracle's per-round threads run on this process's share of distinct
    # physical cores of one package (bench.pick_cores; unpinned they spread
    # over both NUMA packages and run ~1.6x slower).
    sys.path.insert(0, str(ROOT))
    import bench
    threads = oracle_lib.default_threads()
    pinned, _ = bench.pick_cores(threads) if threads < len(os.sched_getaffinity(0)) else (None, None)
    if pinned:
        os.sched_setaffinity(0, pinned)
    o = oracle_lib.OracleRenderer(s.packs(), W, H, threads=threads)
    t0 = time.time()
    for x in (r, o):
        x.RenderFlags = flags
        x.PathTerminationProbability = ptp
        x.CameraIndex = camera
        x.reset()
        x.run(2)
    done = 0
    while done < rounds - 2:
        n = min(50, rounds - 2 - done)
        if batched:
            r.run_rounds(n)
        else:
            for _ in range(n):
                r.run(1)
        for _ in range(n):
            o.run(1)
        done += n
        # progress (the oracle takes ~0.3 s a round at C3)
        print(f"round {done + 2} of {rounds}, {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    dev.synchronize()
    g, want = r.read_state(), o.state()
    bad = {}
    for f in ("origin", "packed_velocity", "lambda0", "throughput", "probability", "sample", "active01", "active23"):
        bad[f] = int(np.sum(np.any((g[f].view(np.uint32) != want[f].view(np.uint32)).reshape(H, W, -1), axis=-1)))
    acc_bad = int(np.sum(np.any(sb.read().view(np.uint32) != o.accum().view(np.uint32), axis=-1)))
    print(json.dumps({"config": cfg, "camera": camera, "size": [W, H], "rounds": rounds, "batched": batched,
                      "split": r.split() if batched else None,
                      "class_lists": r.class_lists() if batched else None, "state_mismatch_px": bad,
                      "accum_mismatch_px": acc_bad, "samples": float(o.accum()[..., 3].sum()),
                      "seconds": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
