"""The slab test's division convention (common.glsl.inc:153-185).

SURVEY.md §7/§8(c) fix the oracle's convention as correctly rounded IEEE
division, and the HIP kernels evaluate the same quotients (exact FMA-corrected
division, pt_device.hpp FastQuot).  Round 2 had moved both sides to the
reciprocal form RN((Min-O)*RN(1/V)); tools/slab_convention.py measured what
that changes (profiles/r03_slab/slab_convention.json: on C3 at 1920x1080, 3 of
8.3 M path rays got another hit, one of them 663 893 ulps away in time, and
the 16-round image moved by 2.6e-4 relative L2 > the 1e-4 bar), so the
IEEE convention was restored on both sides.
"""
from __future__ import annotations

import subprocess
import sys
from pathlib import Path

import numpy as np

import oracle_lib

ROOT = Path(__file__).resolve().parents[1]
INF = np.float32(1e30)


def ieee_slab(o, v, reach, mn, mx):
    """numpy float32 restatement of IntersectBoundingBox with IEEE division
    and GLSL min/max (NaN operands dropped, as fminf/fmaxf)."""
    with np.errstate(divide="ignore", invalid="ignore"):
        a = (mn - o) / v
        b = (mx - o) / v
    e = np.fmax(np.fmax(np.fmin(a[0], b[0]), np.fmin(a[1], b[1])), np.fmin(a[2], b[2]))
    x = np.fmin(np.fmin(np.fmax(a[0], b[0]), np.fmax(a[1], b[1])), np.fmax(a[2], b[2]))
    if x < e or x <= 0 or e >= reach:
        return INF
    return np.float32(e)


def random_boxes(n, seed):
    rng = np.random.default_rng(seed)
    o = rng.uniform(-5, 5, (n, 3)).astype(np.float32)
    v = rng.normal(size=(n, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    v = v.astype(np.float32)
    c = rng.uniform(-5, 5, (n, 3)).astype(np.float32)
    h = rng.uniform(0.01, 3, (n, 3)).astype(np.float32)
    mn, mx = (c - h).astype(np.float32), (c + h).astype(np.float32)
    # special cases: zero velocity components (infinite / NaN slab planes),
    # flat boxes, origin on a plane
    v[:64, 0] = 0.0
    v[64:96, 1:] = 0.0
    mx[96:128, 2] = mn[96:128, 2]
    o[128:160, 0] = mn[128:160, 0]
    reach = np.where(np.arange(n) % 7 == 0, rng.uniform(0.1, 5, n), 1048576.0).astype(np.float32)
    return o, v, reach, mn, mx


def test_oracle_default_is_ieee():
    assert oracle_lib.lib().oracle_slab_division() == 1


def test_ieee_slab_matches_numpy():
    """The oracle's slab test (default convention) equals a float32 IEEE
    restatement bit for bit, special cases included."""
    o, v, reach, mn, mx = random_boxes(4000, 1)
    for i in range(len(o)):
        got = np.float32(oracle_lib.intersect_bounding_box(o[i], v[i], reach[i], mn[i], mx[i]))
        ref = ieee_slab(o[i], v[i], reach[i], mn[i], mx[i])
        assert got.view(np.uint32) == ref.view(np.uint32), (i, got, ref)


def test_reciprocal_form_differs():
    """The reciprocal form is a different evaluation: some entry times differ
    (by an ulp), so the switch the measurement relies on is live."""
    o, v, reach, mn, mx = random_boxes(2000, 2)
    diff = 0
    for i in range(len(o)):
        a = oracle_lib.intersect_bounding_box(o[i], v[i], reach[i], mn[i], mx[i])
        with oracle_lib.slab_division("rcp"):
            b = oracle_lib.intersect_bounding_box(o[i], v[i], reach[i], mn[i], mx[i])
        diff += np.float32(a).view(np.uint32) != np.float32(b).view(np.uint32)
    assert diff > 0
    assert oracle_lib.lib().oracle_slab_division() == 1   # context manager restored the default


def test_measurement_tool_runs(tmp_path):
    """tools/slab_convention.py end to end on a tiny frame (the full-size
    numbers are in profiles/r03_slab)."""
    out = tmp_path / "slab.json"
    subprocess.run([sys.executable, str(ROOT / "tools" / "slab_convention.py"), "--quick", "--configs", "1",
                    "--fuzz", "1", "--out", str(out)], check=True, timeout=600)
    import json
    d = json.loads(out.read_text())
    assert set(d["scenes"]) == {"C1", "fuzz0"}
    c1 = d["scenes"]["C1"]
    assert c1["random_rays"]["rays"] == 20000 and c1["image"]["samples"] > 0
