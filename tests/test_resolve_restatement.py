"""Cross-check of the oracle's RenderSampleBuffer restatement against a
second one written apart from it (tests/resolve_restatement.py): float
OutColor bit for bit and the sRGB8 swapchain bytes exactly, for all four tone
mapping modes, several brightness / white levels, on accumulators with empty
pixels, negative and out-of-gamut XYZ, tiny and huge sums, and a real
oracle-rendered frame."""
from __future__ import annotations

import numpy as np
import pytest

import oracle_lib
import resolve_restatement as rr


def accumulators(seed, n=1500):
    rng = np.random.default_rng(seed)
    a = np.empty((n, 4), np.float32)
    a[:, :3] = rng.lognormal(0.0, 2.0, size=(n, 3)) * rng.choice([1.0, 1.0, 1.0, -0.3], size=(n, 3))
    a[:, 3] = rng.choice([0.0, 1.0, 3.0, 1024.0, 1e-3], size=n)
    a[:20, :3] = 0.0                  # black pixels with samples
    a[20:40, :3] = [0.9505, 1.0, 1.089]   # D65 white
    a[40:60] *= np.float32(1e30)      # huge sums
    a[60:80, :3] *= np.float32(1e-30)  # tiny sums
    return a


@pytest.mark.parametrize("mode", [rr.CLAMP, rr.REINHARD, rr.HABLE, rr.ACES])
@pytest.mark.parametrize("brightness,white", [(1.0, 1.0), (2.5, 4.0), (0.125, 0.5)])
def test_resolve_matches_independent_restatement(pt, mode, brightness, white):
    a = accumulators(mode * 10 + int(brightness * 8))
    want, want8 = oracle_lib.resolve(a, brightness=brightness, mode=mode, white=white)
    got, got8 = rr.resolve(a, brightness=brightness, mode=mode, white=white)
    finite = np.isfinite(want)
    assert np.array_equal(finite, np.isfinite(got))
    assert np.array_equal(got[finite].view(np.uint32), want[finite].view(np.uint32)), \
        np.flatnonzero(np.any(got.view(np.uint32) != want.view(np.uint32), axis=1))[:8]
    assert np.array_equal(got8, want8)


def test_resolve_of_a_rendered_frame(pt):
    """C2's 24x16 oracle frame after 12 rounds, every mode."""
    s = pt.Scene.config(2)
    o = oracle_lib.OracleRenderer(s.packs(), 24, 16)
    o.RenderFlags = 3
    o.reset()
    o.run(2)
    for _ in range(10):
        o.run(1)
    acc = o.accum()
    o.close()
    s.close()
    assert acc[..., 3].sum() > 0
    for mode in (rr.CLAMP, rr.REINHARD, rr.HABLE, rr.ACES):
        want, want8 = oracle_lib.resolve(acc, brightness=1.5, mode=mode, white=2.0)
        got, got8 = rr.resolve(acc, brightness=1.5, mode=mode, white=2.0)
        assert np.array_equal(np.isnan(got), np.isnan(want))
        assert np.array_equal(np.nan_to_num(got).view(np.uint32), np.nan_to_num(want).view(np.uint32))
        assert np.array_equal(got8, want8)
        # NaN channels (Reinhard's c * new / old on black pixels) store 0 by
        # the UNORM rule in the oracle, as in the restatement.
        nan = np.isnan(want[..., :3])
        assert np.all(want8[..., :3][nan] == 0)


def test_srgb8_store_of_nan_and_infinities(pt):
    """The sRGB8 store's rule for non-finite channels, pinned on the oracle:
    NaN -> 0, +inf -> 255, -inf -> 0 (UNORM conversion after the clamp)."""
    a = np.zeros((4, 4), np.float32)
    a[:, 3] = 1.0
    a[0, :3] = np.nan
    a[1, :3] = np.inf
    a[2, :3] = -np.inf
    a[3, :3] = [0.25, 0.5, 1.0]
    want, want8 = oracle_lib.resolve(a, brightness=1.0, mode=rr.CLAMP, white=1.0)
    got, got8 = rr.resolve(a, brightness=1.0, mode=rr.CLAMP, white=1.0)
    assert np.array_equal(got8, want8)
    assert np.all(want8[0, :3] == 0)
