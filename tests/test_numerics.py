"""Known-answer tests of the numerics convention (include/pt_fp.h) through the
CPU oracle: PCG stream, seeding, octahedral packing, the standard-observer fit
and the deterministic transcendentals.  The expected values come from the
independent numpy restatements in tests/kat.py and from the committed
fixtures under tests/golden/ (regenerate with tests/golden/make_golden.py).
"""
from __future__ import annotations

import ctypes as C
import json
from pathlib import Path

import numpy as np
import pytest

import kat
import oracle_lib

GOLDEN = Path(__file__).resolve().parent / "golden"


def _pcg_oracle(state, n):
    s = C.c_uint32(state)
    return [oracle_lib.lib().oracle_pcg(C.byref(s)) for _ in range(n)]


def test_pcg_golden_vectors():
    """First 16 outputs of Random() (common.glsl.inc:189-196) for fixed seeds."""
    gold = json.loads((GOLDEN / "pcg.json").read_text())
    for entry in gold["streams"]:
        assert kat.pcg_stream(entry["seed"], 16) == entry["outputs"]
        assert _pcg_oracle(entry["seed"], 16) == entry["outputs"]


def test_pcg_random_seeds_match_restatement():
    rng = np.random.default_rng(7)
    for s in rng.integers(0, 2**32, size=64, dtype=np.uint64):
        assert _pcg_oracle(int(s), 8) == kat.pcg_stream(int(s), 8)


def test_seed_formula():
    """gid.y*65537 + gid.x + Seed*277803737 with u32 wrap (basic_scatter.glsl:315-318)."""
    assert kat.seed(0, 0, 0) == 0
    assert kat.seed(1, 0, 0) == 1
    assert kat.seed(0, 1, 0) == 65537
    assert kat.seed(0, 0, 1) == 277803737
    assert kat.seed(1919, 1079, 100) == (1079 * 65537 + 1919 + 100 * 277803737) % 2**32


def _oracle_pack(v):
    out = np.zeros(len(v), dtype=np.uint32)
    for i, x in enumerate(np.asarray(v, dtype=np.float32)):
        out[i] = oracle_lib.lib().oracle_pack_unit_vector(x.ctypes.data_as(C.POINTER(C.c_float)))
    return out


def _oracle_unpack(u):
    out = np.zeros((len(u), 3), dtype=np.float32)
    for i, x in enumerate(u):
        oracle_lib.lib().oracle_unpack_unit_vector(int(x), out[i].ctypes.data_as(C.POINTER(C.c_float)))
    return out


def test_unit_vector_golden():
    g = np.load(GOLDEN / "unit_vectors.npz")
    assert np.array_equal(kat.pack_unit_vector(g["directions"]), g["packed"])
    assert np.array_equal(_oracle_pack(g["directions"]), g["packed"])
    assert np.array_equal(_oracle_unpack(g["packed"]).view(np.uint32), g["unpacked"].view(np.uint32))


def test_unit_vector_random_bit_exact():
    rng = np.random.default_rng(11)
    d = rng.normal(size=(2000, 3)).astype(np.float32)
    d[:50, 2] = 0.0                        # equator: the V.z <= 0 fold
    d[50:60] = [[0, 0, 1]] * 5 + [[0, 0, -1]] * 5
    d[60:70, :2] = 0.0
    packed = kat.pack_unit_vector(d)
    assert np.array_equal(_oracle_pack(d), packed)
    un = _oracle_unpack(packed)
    assert np.array_equal(un.view(np.uint32), kat.unpack_unit_vector(packed).view(np.uint32))
    # round trip error of 16-bit octahedral encoding
    dn = d / np.linalg.norm(d, axis=1, keepdims=True)
    assert np.max(np.abs(un - dn)) < 1e-4


def test_unit_vector_special_values():
    assert kat.pack_unit_vector(np.array([[0, 0, 1]]))[0] == 0
    assert kat.pack_unit_vector(np.array([[1, 0, 0]]))[0] == 32767
    assert kat.pack_unit_vector(np.array([[-1, 0, 0]]))[0] == ((-32767) & 0xFFFF)


def test_standard_observer():
    out = np.zeros(3, dtype=np.float32)
    for lam in np.linspace(360.0, 830.0, 95):
        oracle_lib.lib().oracle_sample_observer(float(lam), out.ctypes.data_as(C.POINTER(C.c_float)))
        assert np.allclose(out, kat.standard_observer(float(lam)), rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize("name,ref,lo,hi,max_ulp", [
    ("exp", np.exp, -80.0, 80.0, 2),
    ("log", np.log, 1e-30, 1e30, 2),
    ("sin", np.sin, -100.0, 100.0, 2),
    ("cos", np.cos, -100.0, 100.0, 2),
    ("asin", np.arcsin, -1.0, 1.0, 3),
])
def test_transcendentals_accuracy(name, ref, lo, hi, max_ulp):
    f = getattr(oracle_lib.lib(), f"oracle_fp_{name}")
    rng = np.random.default_rng(3)
    if name == "log":
        x = np.exp(rng.uniform(np.log(lo), np.log(hi), 4000)).astype(np.float32)
    else:
        x = rng.uniform(lo, hi, 4000).astype(np.float32)
    got = np.array([f(float(v)) for v in x], dtype=np.float32)
    exp = ref(x.astype(np.float64)).astype(np.float32)
    # absolute floor near zeros of sin/cos (argument reduction error)
    close = np.abs(got.astype(np.float64) - exp) <= 4e-7
    assert np.all((kat.ulp_distance(got, exp) <= max_ulp) | close)


def test_atan2_accuracy():
    f = oracle_lib.lib().oracle_fp_atan2
    rng = np.random.default_rng(5)
    y = rng.normal(size=3000).astype(np.float32)
    x = rng.normal(size=3000).astype(np.float32)
    got = np.array([f(float(a), float(b)) for a, b in zip(y, x)], dtype=np.float32)
    exp = np.arctan2(y.astype(np.float64), x.astype(np.float64)).astype(np.float32)
    assert np.all((kat.ulp_distance(got, exp) <= 3) | (np.abs(got - exp) <= 4e-7))
    assert f(0.0, 1.0) == 0.0 and f(1.0, 0.0) > 1.57


def test_transcendentals_golden():
    """Bit patterns of the convention kernels, pinned (device code shares pt_fp.h)."""
    g = np.load(GOLDEN / "fp_convention.npz")
    L = oracle_lib.lib()
    for name in ("exp", "log", "sin", "cos", "asin"):
        f = getattr(L, f"oracle_fp_{name}")
        got = np.array([f(float(v)) for v in g[f"{name}_x"]], dtype=np.float32)
        assert np.array_equal(got.view(np.uint32), g[f"{name}_y"].view(np.uint32)), name


def test_unpack_snorm16_equals_ieee_quotient_exhaustively():
    """pt_unpack_snorm16 evaluates x / 32767 as RN(x * RN(1/32767)) plus one
    FMA residual correction (include/pt_fp.h); for every one of the 65 536
    int16 inputs it must equal the correctly rounded quotient (numpy float32
    division), clamped to [-1, 1] as glm::unpackSnorm2x16 does."""
    L = oracle_lib.lib()
    x = np.arange(-32768, 32768, dtype=np.int64)
    want = np.clip(x.astype(np.float32) / np.float32(32767.0), np.float32(-1), np.float32(1)).astype(np.float32)
    got = np.array([L.oracle_unpack_snorm16(int(v) & 0xFFFF) for v in x], dtype=np.float32)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
