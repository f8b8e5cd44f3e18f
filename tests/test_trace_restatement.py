"""Cross-check of the oracle's Trace() against a second restatement written
independently from the GLSL (tests/trace_restatement.py): the whole trace
record bit for bit -- closest-hit time, packed shape / material index,
octahedral normal and tangent, texture U, V -- on random rays
(axis-aligned and tiny-component cases included, tests/rays.py) and on real
path rays -- the rays in flight after a few oracle rounds, which start on
surfaces and graze edges -- for configs 1, 2, 3, 5 and random fuzz scenes.
The two restatements share only the numerics convention of DESIGN.md §2."""
from __future__ import annotations

import numpy as np
import pytest

import fuzz_scenes
import kat
import oracle_lib
import trace_restatement as tr
from rays import random_rays


def path_rays(scene, W, H, n, seed):
    """n of the rays a small oracle render has in flight after Reset, Run(2),
    Run(1) (basic.cpp:285-332), with their packed velocities."""
    o = oracle_lib.OracleRenderer(scene.packs(), W, H)
    o.RenderFlags = 3
    o.reset()
    o.run(2)
    o.run(1)
    st = o.state().reshape(-1)
    o.close()
    pick = np.random.default_rng(seed).choice(len(st), size=min(n, len(st)), replace=False)
    return st["origin"][pick].astype(np.float32), st["packed_velocity"][pick].astype(np.uint32)


def check(arrays, packs, origins, vel, dur):
    rec = oracle_lib.trace_rays(packs, origins, vel, dur)
    V = kat.unpack_unit_vector(vel)
    times, sm, pn, ptg, uv = tr.trace_records(arrays, origins, V, dur)
    assert np.array_equal(sm, rec["shape_material"]), \
        f"shape/material differs at {np.flatnonzero(sm != rec['shape_material'])[:8].tolist()}"
    hit = sm != 0xFFFFFFFF
    assert np.array_equal(times[hit].view(np.uint32), rec["time"][hit].view(np.uint32)), \
        f"hit time differs at {np.flatnonzero(hit & (times.view(np.uint32) != rec['time'].view(np.uint32)))[:8].tolist()}"
    for name, mine in (("packed_normal", pn), ("packed_tangent", ptg)):
        bad = np.flatnonzero(hit & (mine != rec[name]))
        assert bad.size == 0, f"{name} differs at {bad[:8].tolist()}"
    has_uv = hit
    for k, name in enumerate(("u", "v")):
        bad = np.flatnonzero(has_uv & (uv[:, k].view(np.uint32) != rec[name].view(np.uint32)))
        assert bad.size == 0, f"{name} differs at {bad[:8].tolist()}"
    return int(hit.sum())


@pytest.mark.parametrize("config", [1, 2, 3, 5])
def test_trace_matches_independent_restatement(pt, config):
    s = pt.Scene.config(config)
    arrays, packs = s.arrays(), s.packs()
    o, v, d = random_rays(arrays, 300, seed=config)
    hits = check(arrays, packs, o, v, d)
    po, pv = path_rays(s, 64, 48, 200, seed=config)
    hits += check(arrays, packs, po, pv, np.full(len(pv), 1048576.0, np.float32))
    assert hits > 50
    s.close()


@pytest.mark.parametrize("seed", [0, 5, 11])
def test_trace_matches_independent_restatement_fuzz(pt, seed):
    s, _ = fuzz_scenes.build(pt, seed)
    arrays, packs = s.arrays(), s.packs()
    o, v, d = random_rays(arrays, 300, seed=100 + seed)
    hits = check(arrays, packs, o, v, d)
    po, pv = path_rays(s, 48, 32, 150, seed=seed)
    hits += check(arrays, packs, po, pv, np.full(len(pv), 1048576.0, np.float32))
    assert hits > 20
    s.close()
