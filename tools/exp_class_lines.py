"""Where the class-pure shade's extra bytes come from.

The class lists hold a round's ray positions class by class (hit diffuse /
metal / translucent / other, miss), in tile order.  A class-pure wave takes
64 consecutive entries; its path records are read and written by slot, its
ray / hit records by position, 16 B each, and a 128-B cache line holds 8
records.  When a class is rare, 64 entries span many tiles and each line a
wave touches holds few of its records: the rest of the line is fetched for
nothing unless another class's wave reads it while it is still in L2.

This script takes a settled render of the CPU oracle (the rays' outcome
classes; TileOrder's slot permutation within a tile is modelled as a random
permutation), builds the lists, cuts them into waves and counts the distinct
lines each wave touches, against the 64 x 16 B it uses.

usage: python tools/exp_class_lines.py CONFIG W H [ROUNDS]  -> JSON
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

TYPES = {0: 0, 1: 1, 2: 2}   # BASIC_DIFFUSE / METAL / TRANSLUCENT -> outcome class (pt_packed.h); else 3


def main():
    import __graft_entry__ as ge
    import oracle_lib
    pt = ge._load_package()
    config, W, H = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 12
    s = pt.Scene.config(config)
    a = s.arrays()
    mats = a["materials"].reshape(-1, 32)[:, 0]
    shape_mat = a["shapes"]["MaterialIndex"]
    o = oracle_lib.OracleRenderer(s.packs(), W, H)
    o.RenderFlags = 3
    o.reset()
    o.run(2)
    for _ in range(rounds):
        o.run(1)
    st = o.state()
    o.close()
    sm = st["hit"]["shape_material"].reshape(-1)
    miss = sm == 0xFFFFFFFF
    shape = np.where(miss, 0, sm >> 16)
    mtype = mats[shape_mat[shape]]
    cls = np.where(miss, 4, np.vectorize(lambda t: TYPES.get(int(t), 3))(mtype))
    # Pixels -> tiles of 16 x 16 (slot = tile * 256 + row-major within the tile).
    tx = (W + 15) // 16
    y, x = np.divmod(np.arange(W * H), W)
    tile = (y // 16) * tx + (x // 16)
    within = (y % 16) * 16 + (x % 16)
    rng = np.random.default_rng(1)
    ntiles = tile.max() + 1
    perm = np.stack([rng.permutation(256) for _ in range(ntiles)])   # TileOrder: slot -> position
    slot = tile * 256 + within
    pos = tile * 256 + perm[tile, within]
    out = {"config": config, "W": W, "H": H, "rounds": rounds + 2, "classes": {}}
    total_used = total_lines_slot = total_lines_pos = 0
    for c in range(5):
        sel = np.flatnonzero(cls == c)
        if sel.size == 0:
            continue
        order = np.argsort(pos[sel], kind="stable")      # the list: positions in tile order
        sl, ps = slot[sel][order], pos[sel][order]
        nw = (sel.size + 63) // 64
        lines_s = lines_p = 0
        for w in range(nw):
            lines_s += np.unique(sl[w * 64:(w + 1) * 64] // 8).size
            lines_p += np.unique(ps[w * 64:(w + 1) * 64] // 8).size
        used = sel.size
        out["classes"][["diffuse", "metal", "translucent", "other", "miss"][c]] = {
            "fraction": round(sel.size / cls.size, 4), "waves": nw,
            "lines_per_wave_slot_records": round(lines_s / nw, 1),
            "lines_per_wave_position_records": round(lines_p / nw, 1),
            "amplification_slot_records": round(lines_s * 8 / used, 2),
            "amplification_position_records": round(lines_p * 8 / used, 2)}
        total_used += used
        total_lines_slot += lines_s
        total_lines_pos += lines_p
    out["amplification_slot_records"] = round(total_lines_slot * 8 / total_used, 2)
    out["amplification_position_records"] = round(total_lines_pos * 8 / total_used, 2)
    out["note"] = ("lines fetched x 128 B over records used x 16 B, per wave, if no line a wave touches "
                   "is still in L2 from another class's wave (class-major sweeps); tile-local shade: 1.0")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
