"""Cross-check of the oracle's rounds against a second restatement written
from the GLSL text apart from it (tests/path_restatement.py, with
tests/trace_restatement.py for Trace): C1's scene (diffuse sphere and plane
with a nearest-filtered checker texture, constant sky) and C3's (the room
mesh with its bilinear-filtered texture) after Reset, Run(2), Run(1), Run(1)
-- every slot's ray, Lambda0, throughput, probability, sample and
active-shape stack, and every accumulated pixel, bit for bit; with and
without jitter, with Russian roulette, accumulate and overwrite."""
from __future__ import annotations

import numpy as np
import pytest

import oracle_lib
import path_restatement as pr


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("flags,ptp", [(3, 0.0), (1, 0.0), (3, 0.3), (2, 0.0)])
def test_c1_rounds_match_independent_restatement(pt, flags, ptp):
    s = pt.Scene.config(1)
    W, H, schedule = 16, 12, [2, 1, 1]
    slots, accum = pr.render(s, W, H, schedule, flags=flags, ptp=ptp)
    o = oracle_lib.OracleRenderer(s.packs(), W, H)
    o.RenderFlags = flags
    o.PathTerminationProbability = ptp
    o.reset()
    for r in schedule:
        o.run(r)
    st, oa = o.state(), o.accum()
    o.close()
    for y in range(H):
        for x in range(W):
            sl, want = slots[y][x], st[y, x]
            where = (x, y)
            assert np.array_equal(bits(sl.O), want["origin"].view(np.uint32)), (where, "origin")
            assert sl.PV == int(want["packed_velocity"]), (where, "velocity")
            assert bits(sl.lam0) == np.float32(want["lambda0"]).view(np.uint32), (where, "lambda0")
            assert np.array_equal(bits(sl.thr), want["throughput"].view(np.uint32)), (where, "throughput")
            assert np.array_equal(bits(sl.prob), want["probability"].view(np.uint32)), (where, "probability")
            assert np.array_equal(bits(sl.sample), want["sample"].view(np.uint32)), (where, "sample")
            act = [a & 0xFFFF for a in sl.active]
            assert (act[1] << 16 | act[0]) == int(want["active01"]), (where, "active01")
            assert (act[3] << 16 | act[2]) == int(want["active23"]), (where, "active23")
    assert np.array_equal(bits(accum), oa.view(np.uint32)), "accumulator"
    assert oa[..., 3].sum() > 0
    s.close()


@pytest.mark.parametrize("flags", [3, 1])
def test_c3_rounds_match_independent_restatement(pt, flags):
    """C3's room: a textured (bilinear) diffuse mesh under a constant sky."""
    s = pt.Scene.config(3)
    W, H, schedule = 12, 8, [2, 1, 1]
    slots, accum = pr.render(s, W, H, schedule, flags=flags)
    o = oracle_lib.OracleRenderer(s.packs(), W, H)
    o.RenderFlags = flags
    o.reset()
    for r in schedule:
        o.run(r)
    st, oa = o.state(), o.accum()
    o.close()
    for y in range(H):
        for x in range(W):
            sl, want = slots[y][x], st[y, x]
            assert sl.PV == int(want["packed_velocity"]), ((x, y), "velocity")
            assert np.array_equal(bits(sl.thr), want["throughput"].view(np.uint32)), ((x, y), "throughput")
            assert np.array_equal(bits(sl.prob), want["probability"].view(np.uint32)), ((x, y), "probability")
            assert np.array_equal(bits(sl.O), want["origin"].view(np.uint32)), ((x, y), "origin")
    assert np.array_equal(bits(accum), oa.view(np.uint32)), "accumulator"
    assert oa[..., 3].sum() > 0 and oa[..., :3].sum() > 0     # escapes reached the sky
    s.close()
