"""One-off deeper cross-check of the oracle against tests/path_restatement.py:
fuzz seeds given on the command line, 16x12 pixels, Reset + Run(2) + 14 x Run(1),
every slot and pixel compared (CPU; run one process per group of seeds).

usage: python tools/restatement_deep.py SEED [SEED ...]"""
import sys
from pathlib import Path

import numpy as np
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / 'tests'))
from conftest import load_package
import fuzz_scenes, oracle_lib, path_restatement as pr
pt = load_package()
def bits(a): return np.asarray(a, np.float32).view(np.uint32)
for seed in map(int, sys.argv[1:]):
    s, st = fuzz_scenes.build(pt, seed)
    W, H, sched = 16, 12, [2] + [1] * 14
    slots, accum = pr.render(s, W, H, sched, flags=st["flags"], ptp=st["termination"], camera=st["camera"])
    o = oracle_lib.OracleRenderer(s.packs(), W, H)
    o.RenderFlags = st["flags"]; o.PathTerminationProbability = st["termination"]; o.CameraIndex = st["camera"]
    o.reset()
    for r in sched: o.run(r)
    w, oa = o.state(), o.accum(); o.close()
    bad = 0
    for y in range(H):
        for x in range(W):
            sl, ww = slots[y][x], w[y, x]
            act = [a & 0xFFFF for a in sl.active]
            ok = (np.array_equal(bits(sl.O), ww["origin"].view(np.uint32)) and sl.PV == int(ww["packed_velocity"])
                  and np.array_equal(bits(sl.thr), ww["throughput"].view(np.uint32))
                  and np.array_equal(bits(sl.prob), ww["probability"].view(np.uint32))
                  and np.array_equal(bits(sl.sample), ww["sample"].view(np.uint32))
                  and (act[1] << 16 | act[0]) == int(ww["active01"]) and (act[3] << 16 | act[2]) == int(ww["active23"]))
            bad += not ok
    accbad = int(np.sum(np.any(bits(accum) != oa.view(np.uint32), axis=-1)))
    print(seed, "bad", bad, "accbad", accbad, flush=True)
