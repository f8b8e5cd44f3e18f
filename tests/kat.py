"""Independent numpy restatements used as known-answer generators.

These are written from the reference GLSL/C++ formulas directly (not from the
oracle's C code), so agreement with the oracle checks the restatement rather
than restating it twice the same way.  Test infrastructure only.
"""
from __future__ import annotations

import numpy as np

M32 = 0xFFFFFFFF


def pcg(state: int):
    """Random() (reference src/core/common.glsl.inc:189-196).  Returns (value, new_state)."""
    state = (state * 747796405 + 2891336453) & M32
    s = state
    w = (((s >> ((s >> 28) + 4)) ^ s) * 277803737) & M32
    return ((w >> 22) ^ w) & M32, state


def pcg_stream(state: int, n: int):
    out = []
    for _ in range(n):
        v, state = pcg(state)
        out.append(v)
    return out


def seed(x: int, y: int, frame: int) -> int:
    """Per-invocation seed (basic_scatter.glsl:315-318)."""
    return (y * 65537 + x + frame * 277803737) & M32


def _round_half_away(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.float64)
    return np.sign(x) * np.floor(np.abs(x) + 0.5)


def pack_snorm2x16(p: np.ndarray) -> np.ndarray:
    """glm::packSnorm2x16 / GLSL packSnorm2x16: round(clamp(v,-1,1)*32767)."""
    c = np.clip(p.astype(np.float32), np.float32(-1), np.float32(1)) * np.float32(32767.0)
    q = _round_half_away(c.astype(np.float32)).astype(np.int64) & 0xFFFF
    return (q[..., 0] | (q[..., 1] << 16)).astype(np.uint32)


def unpack_snorm2x16(u: np.ndarray) -> np.ndarray:
    u = np.asarray(u, dtype=np.uint32)
    lo = (u & 0xFFFF).astype(np.uint16).view(np.int16).astype(np.float32)
    hi = (u >> 16).astype(np.uint16).view(np.int16).astype(np.float32)
    p = np.stack([lo, hi], axis=-1) / np.float32(32767.0)
    return np.clip(p, np.float32(-1), np.float32(1))


def _sign_not_zero(p: np.ndarray) -> np.ndarray:
    return np.where(p >= 0, np.float32(1), np.float32(-1)).astype(np.float32)


def pack_unit_vector(v: np.ndarray) -> np.ndarray:
    """PackUnitVector (common.glsl.inc:137-142; host common.hpp:100-105), float32 step by step."""
    v = np.asarray(v, dtype=np.float32).reshape(-1, 3)
    l1 = (np.abs(v[:, 0]) + np.abs(v[:, 1])) + np.abs(v[:, 2])
    inv = (np.float32(1.0) / l1).astype(np.float32)
    p = v[:, :2] * inv[:, None]
    fold = (np.float32(1.0) - np.abs(p[:, ::-1])) * _sign_not_zero(p)
    p = np.where((v[:, 2] <= 0)[:, None], fold, p).astype(np.float32)
    return pack_snorm2x16(p)


def unpack_unit_vector(u: np.ndarray) -> np.ndarray:
    """UnpackUnitVector (common.glsl.inc:145-151), normalize = v * (1/sqrt(dot(v,v)))."""
    p = unpack_snorm2x16(u).reshape(-1, 2)
    z = (np.float32(1.0) - np.abs(p[:, 0])) - np.abs(p[:, 1])
    fold = (np.float32(1.0) - np.abs(p[:, ::-1])) * _sign_not_zero(p)
    p = np.where((z < 0)[:, None], fold, p).astype(np.float32)
    v = np.concatenate([p, z[:, None]], axis=1).astype(np.float32)
    d = (v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1]) + v[:, 2] * v[:, 2]
    r = (np.float32(1.0) / np.sqrt(d.astype(np.float32))).astype(np.float32)
    return (v * r[:, None]).astype(np.float32)


def standard_observer(lam: float) -> np.ndarray:
    """Wyman et al. multi-lobe CIE 1931 fit (spectrum.glsl.inc:10-33), float64."""
    def g(x, mu, lo, hi):
        t = (x - mu) * (lo if x < mu else hi)
        return np.exp(-0.5 * t * t)
    x = 0.362 * g(lam, 442.0, 0.0624, 0.0374) + 1.056 * g(lam, 599.8, 0.0264, 0.0323) - 0.065 * g(lam, 501.1, 0.0490, 0.0382)
    y = 0.821 * g(lam, 568.8, 0.0213, 0.0247) + 0.286 * g(lam, 530.9, 0.0613, 0.0322)
    z = 1.217 * g(lam, 437.0, 0.0845, 0.0278) + 0.681 * g(lam, 459.0, 0.0385, 0.0725)
    return np.array([x, y, z])


def ulp_distance(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """|a-b| in float32 ulps (sign-magnitude ordered)."""
    def key(x):
        i = np.asarray(x, dtype=np.float32).view(np.int32).astype(np.int64)
        return np.where(i < 0, -(i & 0x7FFFFFFF), i)
    return np.abs(key(a) - key(b))
