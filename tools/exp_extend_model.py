"""Per-step cost model of the extend kernel's LaneStep loop,
evaluated on real per-ray step sequences of a settled C3 frame.

1. Step sequences: the oracle renders C3 at 256x128 for Reset + Run(2) + 12
   rounds; each pixel's current ray is traced by tests/trace_restatement.py
   instrumented to record its step kinds in the extend kernel's order:
   I = internal BLAS node (child-pair box test), F = one face (FACE_STEP),
   T = TLAS-level step (scene.glsl.inc:468-520, incl. the BLAS exit).  Pops
   ride on the step that empties a leaf or misses both children (no step of
   their own), as in LaneStep.  Rays are grouped into 16x16-pixel tiles of
   four 64-lane waves (the kernel's tile / wave shape, rows of 16 pixels).
2. Wave-step cost (VALU instructions, gfx950 disassembly of
   extend_kernel<slots, no spill, 5, 20, u16>, tools/r05 asm notes in DESIGN
   §4): internal-node path cI = 115 (12 subtractions, 36 Markstein quotient
   FMAs / multiplies, min/max network, decision and push), face path cF = 74
   (Moller-Trumbore with the exact reciprocal), TLAS path cT = 60, loop
   overhead c0 = 20; a wave step executes every path one of its active lanes
   takes (exec-masked).  Vector memory per step: 4 x dwordx4 (node pair) on
   internal lanes, 3 x dwordx4 (face) on face lanes.
3. Policies evaluated (cost per tile = sum over wave steps):
   * baseline: every active lane advances one step per wave step;
   * postponed faces (k): face lanes wait while fewer than k lanes of the wave
     need a face (the face path then runs for more lanes at once);
   * in-block compaction every K steps (extend_compact_kernel): when the
     block's live rays fit in fewer waves, they move to the lowest threads
     (cost: a count barrier every K steps, 80 instructions per wave per
     exchange), capped at the exchange buffer's 138 rays.

usage: python tools/exp_extend_model.py [tiles]   (prints the table DESIGN.md §4 quotes)
"""
import pickle
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

cI, cF, cT, c0 = 115, 74, 60, 20


def sequences(ntiles, W=256, H=128, seed=3):
    import bench
    import oracle_lib  # test infrastructure (the CPU restatement), not the product path
    import trace_restatement as T
    pt = bench.load_package()
    s = pt.Scene.config(3)
    A = s.arrays()
    o = oracle_lib.OracleRenderer(s.packs(), W, H, threads=8)
    o.RenderFlags = 3
    o.reset()
    o.run(2)
    for _ in range(12):
        o.run(1)
    st = o.state()
    S = T.Scene(A)
    seq = []

    def mesh_node(S, O, V, root, hit):
        stack, node = [], root
        while True:
            if S.mn_end[node] > 0:
                for face in range(S.mn_begin[node], S.mn_end[node]):
                    T.intersect_mesh_face(S, O, V, face, hit)
                    seq.append("F")
            else:
                seq.append("I")
                a = S.mn_begin[node]
                b = a + 1
                ta = T.intersect_bounding_box(O, V, hit.time, S.mn_min[a], S.mn_max[a])
                tb = T.intersect_bounding_box(O, V, hit.time, S.mn_min[b], S.mn_max[b])
                if ta > tb:
                    if ta < T.INFINITY:
                        stack.append(a)
                    node = b
                    continue
                if tb < T.INFINITY:
                    stack.append(b)
                    node = a
                    continue
                if ta < T.INFINITY:
                    node = a
                    continue
            if not stack:
                break
            node = stack.pop()

    shape = T.intersect_shape

    def shape_step(S, O, V, idx, hit):
        seq.append("T")
        return shape(S, O, V, idx, hit)

    T.intersect_mesh_node, T.intersect_shape = mesh_node, shape_step
    rng = np.random.default_rng(seed)
    blocks = [(bx, by) for by in range(H // 16) for bx in range(W // 16)]
    tiles = []
    for bi in rng.choice(len(blocks), ntiles, replace=False):
        bx, by = blocks[bi]
        tile = []
        for y in range(by * 16, by * 16 + 16):
            for x in range(bx * 16, bx * 16 + 16):
                p = st[y, x]
                d = np.zeros(3, np.float32)
                oracle_lib.lib().oracle_unpack_unit_vector(int(p["packed_velocity"]),
                                                           d.ctypes.data_as(oracle_lib.C.POINTER(oracle_lib.C.c_float)))
                seq.clear()
                T.trace(S, T._v(p["origin"]), T._v(d), np.float32(1048576.0))
                tile.append("".join(seq))
        tiles.append(tile)
    o.close()
    return tiles


def step_cost(kinds):
    return c0 + cI * ("I" in kinds) + cF * ("F" in kinds) + cT * ("T" in kinds)


def run_tile(tile, postpone=0, K=0, cap=256, ccomp=80, cbar=10):
    rays = [[s, 0] for s in tile]
    lanes = list(range(256))
    cost = wsteps = lsteps = 0
    steps = comps = 0
    while True:
        live_waves = 0
        for w in range(4):
            idx = [r for r in lanes[w * 64:(w + 1) * 64] if r is not None and rays[r][1] < len(rays[r][0])]
            if not idx:
                continue
            live_waves += 1
            nxt = {r: rays[r][0][rays[r][1]] for r in idx}
            nI = sum(v == "I" for v in nxt.values())
            nF = sum(v == "F" for v in nxt.values())
            nT = sum(v == "T" for v in nxt.values())
            adv = [r for r in idx if nxt[r] == "I"] if (postpone and nI and nF < postpone and not nT) else idx
            cost += step_cost(set(nxt[r] for r in adv))
            wsteps += 1
            lsteps += len(adv)
            for r in adv:
                rays[r][1] += 1
        if live_waves == 0:
            break
        steps += 1
        if K and steps % K == 0:
            cost += 4 * cbar
            alive = [r for r in lanes if r is not None and rays[r][1] < len(rays[r][0])]
            if (len(alive) + 63) // 64 < live_waves and len(alive) <= cap:
                comps += 1
                cost += live_waves * ccomp
                lanes = alive + [None] * (256 - len(alive))
    return cost, wsteps, lsteps, steps, comps


def main():
    ntiles = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    cache = Path("/tmp/pt_extend_model_tiles.pkl")
    if cache.exists():
        tiles = pickle.loads(cache.read_bytes())
    else:
        tiles = sequences(ntiles)
        cache.write_bytes(pickle.dumps(tiles))
    n = len(tiles)
    L = [len(s) for t in tiles for s in t]
    print(f"{n} tiles, {len(L)} rays, {np.mean(L):.2f} steps per ray "
          f"(I {np.mean([s.count('I') for t in tiles for s in t]):.2f}, "
          f"F {np.mean([s.count('F') for t in tiles for s in t]):.2f}, "
          f"T {np.mean([s.count('T') for t in tiles for s in t]):.2f})")
    base = None
    for name, kw in [("baseline", {}), ("postpone faces k=4", {"postpone": 4}), ("postpone faces k=16", {"postpone": 16}),
                     ("compact K=2", {"K": 2, "cap": 138}), ("compact K=4", {"K": 4, "cap": 138}),
                     ("compact K=8", {"K": 8, "cap": 138})]:
        C = W = LS = S = CP = 0
        for t in tiles:
            c, w, ls, s, cp = run_tile(t, **kw)
            C += c; W += w; LS += ls; S += s; CP += cp
        base = base or C
        print(f"{name:22s} VALU/tile {C / n:8.0f} ({C / base - 1:+.1%})  wave steps/tile {W / n:6.1f}  "
              f"SIMD eff {LS / (W * 64):.3f}  block steps {S / n:5.1f}  exchanges/tile {CP / n:.1f}")


if __name__ == "__main__":
    main()
