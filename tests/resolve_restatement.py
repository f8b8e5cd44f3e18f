"""A second restatement of RenderSampleBuffer (resolve.glsl:60-130), written
from the GLSL apart from oracle/pt_oracle.cpp (test infrastructure only;
tests/test_resolve_restatement.py): the accumulator's mean XYZ scaled by
Brightness, CIE_XYZ_TO_SRGB (spectrum.glsl.inc:50-55, GLSL mat3 given by
columns), then the Clamp / Reinhard / Hable / ACES tone curves, and the
swapchain's B8G8R8A8_SRGB store (vulkan.cpp:1407): the sRGB transfer curve
and UNORM8 rounding.

Numerics: DESIGN.md §2's convention in numpy float32 (nothing fused, a
mat3 * vec3 and a dot summed left to right, GLSL constant expressions such
as C * B folded in float32); the sRGB curve's power is exp(log(C) / 2.4) on
the convention's exp / log (the oracle's exported pt_exp / pt_log), and
UNORM8 conversion rounds x * 255 half up."""
from __future__ import annotations

import numpy as np

import oracle_lib

f32 = np.float32
CLAMP, REINHARD, HABLE, ACES = 0, 1, 2, 3

# mat3(c0, c1, c2): columns; M @ v = c0 * v.x + c1 * v.y + c2 * v.z.
XYZ_TO_SRGB = np.array([[3.2406, -0.9689, 0.0557], [-1.5372, 1.8758, -0.2040], [-0.4986, 0.0415, 1.0570]], f32)
ACES_IN = np.array([[0.59719, 0.07600, 0.02840], [0.35458, 0.90834, 0.13383], [0.04823, 0.01566, 0.83777]], f32)
ACES_OUT = np.array([[1.60475, -0.10208, -0.00327], [-0.53108, 1.10813, -0.07276], [-0.07367, -0.00605, 1.07602]], f32)


def _mat(cols, v):
    """GLSL mat3 * vec3 over (n, 3) rows of v."""
    return (cols[0][None, :] * v[:, 0:1] + cols[1][None, :] * v[:, 1:2]) + cols[2][None, :] * v[:, 2:3]


def _fp_vec(name, x):
    fn = getattr(oracle_lib.lib(), f"oracle_fp_{name}")
    return np.array([fn(float(v)) for v in x.reshape(-1)], f32).reshape(x.shape)


def tone_map(color, mode, white):
    c = color
    if mode == CLAMP:
        return np.clip(c, f32(0.0), f32(1.0))
    if mode == REINHARD:
        old = (c[:, 0] * f32(0.2126) + c[:, 1] * f32(0.7152)) + c[:, 2] * f32(0.0722)
        mx = f32(white)
        n = old * (f32(1.0) + old / (mx * mx))
        new = n / (f32(1.0) + old)
        return (c * new[:, None]) / old[:, None]
    if mode == HABLE:
        def partial(x):
            a, b, cc, d, e, f = f32(0.15), f32(0.50), f32(0.10), f32(0.20), f32(0.02), f32(0.30)
            return (x * (a * x + cc * b) + d * e) / (x * (a * x + b) + d * f) - e / f
        cur = partial(c * f32(2.0))
        scale = f32(1.0) / partial(np.full((1, 3), f32(11.2)))
        return cur * scale
    if mode == ACES:
        v = _mat(ACES_IN, c)
        a = v * (v + f32(0.0245786)) - f32(0.000090537)
        b = v * (f32(0.983729) * v + f32(0.4329510)) + f32(0.238081)
        return _mat(ACES_OUT, a / b)
    return c


def encode_srgb8(c):
    """B8G8R8A8_SRGB store of a float channel.  Vulkan's UNORM conversion
    takes NaN to 0 (the device's and the oracle's pt_clamp does so by
    min/max), so NaN is mapped to 0 here by rule, not left to numpy's
    platform-defined float -> uint8 cast."""
    c = np.where(np.isnan(c), f32(0.0), c).astype(f32)
    c = np.clip(c, f32(0.0), f32(1.0))
    powed = _fp_vec("exp", _fp_vec("log", c) * (f32(1.0) / f32(2.4)))
    e = np.where(c <= f32(0.0031308), f32(12.92) * c, f32(1.055) * powed - f32(0.055)).astype(f32)
    return np.floor(np.clip(e, f32(0.0), f32(1.0)) * f32(255.0) + f32(0.5)).astype(np.uint8)


def resolve(accum, brightness=1.0, mode=CLAMP, white=1.0):
    """(OutColor float32 (..., 4), sRGB8 bytes (..., 4)) of accumulator pixels.
    IEEE float32 semantics throughout: inf / NaN arithmetic is the restated
    behaviour (e.g. Reinhard on black pixels), so numpy's warnings for it are
    silenced; the one platform-defined step, NaN -> uint8, is ruled out in
    encode_srgb8."""
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        return _resolve(accum, brightness, mode, white)


def _resolve(accum, brightness, mode, white):
    a = np.asarray(accum, f32).reshape(-1, 4)
    color = np.zeros((len(a), 3), f32)
    live = a[:, 3] > 0
    mean = (f32(brightness) * a[live, :3]) / a[live, 3:4]
    color[live] = _mat(XYZ_TO_SRGB, mean)
    color = tone_map(color, mode, white).astype(f32)
    out = np.concatenate([color, np.ones((len(a), 1), f32)], axis=1)
    out8 = np.concatenate([encode_srgb8(color), np.full((len(a), 1), 255, np.uint8)], axis=1)
    shape = np.asarray(accum).shape
    return out.reshape(shape), out8.reshape(shape)
