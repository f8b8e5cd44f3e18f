"""RenderSampleBuffer / resolve (resolve.glsl:60-130): the oracle against an
independent numpy float32 restatement, and the image writers."""
from __future__ import annotations

import numpy as np
import pytest

import oracle_lib

F = np.float32
XYZ_TO_SRGB = np.array([[3.2406, -0.9689, 0.0557], [-1.5372, 1.8758, -0.2040], [-0.4986, 0.0415, 1.0570]], F)
ACES_IN = np.array([[0.59719, 0.07600, 0.02840], [0.35458, 0.90834, 0.13383], [0.04823, 0.01566, 0.83777]], F)
ACES_OUT = np.array([[1.60475, -0.10208, -0.00327], [-0.53108, 1.10813, -0.07276], [-0.07367, -0.00605, 1.07602]], F)


def mat3_mul(cols, v):
    """GLSL mat3 (given as columns) * vec3, summed left to right in float32."""
    return np.stack([(cols[0, r] * v[..., 0] + cols[1, r] * v[..., 1]) + cols[2, r] * v[..., 2] for r in range(3)], -1)


def hable_partial(x):
    A, B, C, D, E, Fc = F(0.15), F(0.50), F(0.10), F(0.20), F(0.02), F(0.30)
    return (x * (A * x + C * B) + D * E) / (x * (A * x + B) + D * Fc) - E / Fc


def resolve_np(acc, brightness, mode, white):
    acc = acc.astype(F)
    a = acc[..., 3:4]
    with np.errstate(all="ignore"):
        col = np.where(a > 0, mat3_mul(XYZ_TO_SRGB, (F(brightness) * acc[..., :3]) / a), F(0))
        if mode == 0:
            col = np.clip(np.nan_to_num(col, nan=0.0), 0, 1).astype(F)
        elif mode == 1:
            old = (col[..., 0] * F(0.2126) + col[..., 1] * F(0.7152)) + col[..., 2] * F(0.0722)
            n = old * (F(1) + old / (F(white) * F(white)))
            new = n / (F(1) + old)
            col = col * new[..., None] / old[..., None]
        elif mode == 2:
            col = hable_partial(col * F(2)) * (F(1) / hable_partial(np.full(3, 11.2, F)))
        else:
            v = mat3_mul(ACES_IN, col)
            A = v * (v + F(0.0245786)) - F(0.000090537)
            B = v * (F(0.983729) * v + F(0.4329510)) + F(0.238081)
            col = mat3_mul(ACES_OUT, A / B)
    return col.astype(F)


def accumulators(seed=0):
    rng = np.random.default_rng(seed)
    a = rng.uniform(0, 4, size=(24, 32, 4)).astype(F)
    a[..., 3] = rng.integers(0, 50, size=(24, 32)).astype(F)
    a[0, :8] = 0                                   # no samples -> black
    a[1, :8, :3] = -a[1, :8, :3]                   # negative XYZ sums
    a[2, :8, :3] *= 1e6                            # very bright
    return a


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
@pytest.mark.parametrize("brightness,white", [(1.0, 1.0), (2.5, 4.0)])
def test_oracle_matches_numpy(mode, brightness, white):
    acc = accumulators(mode)
    out, out8 = oracle_lib.resolve(acc, brightness, mode, white)
    exp = resolve_np(acc, brightness, mode, white)
    got = out[..., :3]
    same = (got.view(np.uint32) == exp.view(np.uint32)) | (np.isnan(got) & np.isnan(exp))
    assert same.all(), np.argwhere(~same)[:5]
    assert np.all(out[..., 3] == 1.0) and np.all(out8[..., 3] == 255)


def test_srgb8_encoding():
    acc = accumulators(7)
    out, out8 = oracle_lib.resolve(acc, 1.0, 0, 1.0)
    c = np.clip(out[..., :3].astype(np.float64), 0, 1)
    ref = np.where(c <= 0.0031308, 12.92 * c, 1.055 * np.power(c, 1 / 2.4) - 0.055)
    ref8 = np.floor(ref * 255 + 0.5)
    assert np.max(np.abs(out8[..., :3].astype(int) - ref8)) <= 1
    assert np.mean(out8[..., :3] == ref8) > 0.99
    assert np.all(out8[0, :8, :3] == 0)            # zero samples -> black


def test_png_roundtrip(pt, tmp_path):
    img = np.random.default_rng(3).integers(0, 256, size=(17, 23, 4), dtype=np.uint8)
    pt.write_png(tmp_path / "a.png", img)
    assert np.array_equal(pt.read_png(tmp_path / "a.png"), img)
    pt.write_ppm(tmp_path / "a.ppm", img)
    assert (tmp_path / "a.ppm").read_bytes().startswith(b"P6\n23 17\n255\n")
    pt.write_pfm(tmp_path / "a.pfm", img.astype(np.float32))
    assert (tmp_path / "a.pfm").stat().st_size == len(b"PF\n23 17\n-1.0\n") + 17 * 23 * 12


def test_resolve_parameters_defaults(pt):
    p = pt.ResolveParameters()
    assert (p.Brightness, p.ToneMappingMode, p.ToneMappingWhiteLevel) == (1.0, pt.TONE_MAPPING_CLAMP, 1.0)
