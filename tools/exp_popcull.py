"""How many BLAS steps would culling popped nodes by their stored entry time
save?  (Round 6 model; nothing here is built into the product.)

The reference pops a set-aside child (scene.glsl.inc:394-397) and visits it
without looking at the hit found since the push: an internal child then tests
its two children against the shorter Reach and, when both boxes now start at
or beyond it, misses both and pops again (:360-390).  With the child's entry
time kept beside its stack entry, such a pop could be skipped without a fetch
-- the same hit, because a parent's box bounds its children's and the slab
quotients are correctly rounded, so a child's EntryT is never below its
parent's.  This tool counts those steps on the same step sequences
tools/exp_extend_model.py uses (settled C3 frame of the oracle at 256x128, per
ray in LaneStep's order) and prices them in the model's wave steps.

usage: python tools/exp_popcull.py [tiles]
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "tools"))

import exp_extend_model as M  # noqa: E402


def sequences(ntiles, W=256, H=128, seed=3, config=3):
    import bench
    import oracle_lib  # test infrastructure (the CPU restatement), not the product path
    import trace_restatement as T
    pt = bench.load_package()
    s = pt.Scene.config(config)
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
    stats = {"pops": 0, "pops_internal": 0, "cullable": 0, "max_depth": 0}

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
                        stack.append((a, ta))
                    node = b
                    stats["max_depth"] = max(stats["max_depth"], len(stack))
                    continue
                if tb < T.INFINITY:
                    stack.append((b, tb))
                    stats["max_depth"] = max(stats["max_depth"], len(stack))
                    node = a
                    continue
                if ta < T.INFINITY:
                    node = a
                    continue
            # pop; mark culled internal pops ("i": the step a stored entry
            # time would skip)
            while stack:
                node, t = stack.pop()
                stats["pops"] += 1
                if S.mn_end[node] == 0:
                    stats["pops_internal"] += 1
                    if t >= hit.time:
                        stats["cullable"] += 1
                        seq.append("i")   # this internal step misses both children
                        # the reference visits it: two box tests, both miss, pop again
                        continue
                break
            else:
                break

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
    return tiles, stats


def main():
    ntiles = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    config = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    tiles, stats = sequences(ntiles, config=config)
    steps = sum(len(s) for t in tiles for s in t)
    culled = sum(s.count("i") for t in tiles for s in t)
    base = [M.run_tile([s.replace("i", "I") for s in t]) for t in tiles]
    skip = [M.run_tile([s.replace("i", "") for s in t]) for t in tiles]
    rays = 256 * len(tiles)
    print(f"config {config}, {len(tiles)} tiles, {rays} rays")
    print(f"steps per ray {steps / rays:.2f}; culled-pop steps per ray {culled / rays:.3f} ({culled / steps:.1%} of steps)")
    print(f"pops {stats['pops']}, internal {stats['pops_internal']}, cullable {stats['cullable']}, max stack {stats['max_depth']}")
    for name, k in (("VALU cost", 0), ("wave steps", 1), ("lane steps", 2)):
        b = sum(x[k] for x in base)
        s = sum(x[k] for x in skip)
        print(f"{name}: {b} -> {s} ({s / b - 1:+.1%})")


if __name__ == "__main__":
    main()
