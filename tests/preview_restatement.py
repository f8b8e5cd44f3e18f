"""A second restatement of RenderPreview (preview_render.glsl:96-178),
written from the GLSL apart from oracle/pt_oracle.cpp (test infrastructure
only; tests/test_preview_restatement.py): one primary ray per pixel from the
camera transform, Trace() (tests/trace_restatement.py, with its shape / mesh
node counters), and the seven render modes -- base colour (MaterialBaseColor
dispatch, scene.glsl.inc:254-274,696-701, observed under D65,
spectrum.glsl.inc:159-215), shaded base colour, normal, material and
primitive index palettes, mesh and scene complexity -- the selection tint,
brightness, the pick query and the per-pixel AOVs.

Numerics: DESIGN.md §2's convention in float32 (nothing fused, sums left to
right, normalize = v * (1 / sqrt(dot))); the fragment's ScreenXY is the pixel
centre ((x + 0.5) / W, (y + 0.5) / H) of a W x H viewport; the D65 table is
include/pt_cie.h's."""
from __future__ import annotations

import re
from pathlib import Path

import numpy as np

import path_restatement as pr
import trace_restatement as tr

f32 = np.float32
NONE = 0xFFFFFFFF
COLORS = np.array([
    (0.902, 0.098, 0.294), (0.235, 0.706, 0.294), (1.000, 0.882, 0.098), (0.263, 0.388, 0.847),
    (0.961, 0.510, 0.192), (0.569, 0.118, 0.706), (0.275, 0.941, 0.941), (0.941, 0.196, 0.902),
    (0.737, 0.965, 0.047), (0.980, 0.745, 0.745), (0.000, 0.502, 0.502), (0.902, 0.745, 1.000),
    (0.604, 0.388, 0.141), (1.000, 0.980, 0.784), (0.502, 0.000, 0.000), (0.667, 1.000, 0.765),
    (0.502, 0.502, 0.000), (1.000, 0.847, 0.694), (0.000, 0.000, 0.459), (0.502, 0.502, 0.502)], f32)
XYZ_TO_SRGB = [[f32(3.2406), f32(-0.9689), f32(0.0557)], [f32(-1.5372), f32(1.8758), f32(-0.2040)],
               [f32(-0.4986), f32(0.0415), f32(1.0570)]]   # mat3 columns


def _d65():
    text = (Path(__file__).resolve().parents[1] / "include" / "pt_cie.h").read_text()
    body = text[text.index("#define PT_CIE_D65_VALUES"):]
    vals = re.findall(r"([0-9]+\.[0-9]+)f", body)
    assert len(vals) >= 471
    return np.array(vals[:471], f32)


D65 = _d65()


def _mat3(cols, v):
    return [(cols[0][r] * v[0] + cols[1][r] * v[1]) + cols[2][r] * v[2] for r in range(3)]


def illuminant_d65(nl):
    """SampleIlluminantD65 (spectrum.glsl.inc:159-164)."""
    off = nl * f32(470.0)
    i = min(max(int(off), 0), 469)
    return pr._mix(D65[i], D65[i + 1], off - f32(i))


def observe_d65(beta_w):
    """ObserveParametricSpectrumUnderD65(vec4) (spectrum.glsl.inc:197-210)."""
    delta = (pr.LAMBDA_MAX - pr.LAMBDA_MIN) / f32(16.0)
    c = [f32(0.0)] * 3
    for i in range(16):
        nl = f32(i) / f32(15.0)
        d = illuminant_d65(nl) / f32(10566.864005)
        lam = pr._mix(pr.LAMBDA_MIN, pr.LAMBDA_MAX, nl)
        s = beta_w[3] * pr.parametric(beta_w[:3], lam)
        obs = pr.observer(lam)
        c = [c[k] + ((s * d) * obs[k]) * delta for k in range(3)]
    return c


def base_color(W_, m, uv):
    """MaterialBaseColor: *_BaseColor by type, black for anything else."""
    typ = int(W_.mat[32 * m])
    one = f32(1.0)
    if typ in (0, 1):
        col = observe_d65([W_.mfloat(m, 1), W_.mfloat(m, 2), W_.mfloat(m, 3), one])
        ti = int(W_.mat[32 * m + 4])
        if ti != NONE:
            t = W_.sample_texture(ti, uv)
            tc = observe_d65([t[0], t[1], t[2], one])
            col = [col[k] * tc[k] for k in range(3)]
        return col
    if typ == 2:
        return observe_d65([W_.mfloat(m, 7), W_.mfloat(m, 8), W_.mfloat(m, 9), one])
    return [f32(0.0)] * 3


def preview(scene, camera_to, mode, W, H, brightness=1.0, selected=NONE, mouse=(NONE, NONE)):
    """(OutColor (H, W, 4), AOV dict of (H, W) arrays, query)."""
    W_ = pr.World(scene)
    to = np.asarray(camera_to, f32).reshape(16)
    img = np.zeros((H, W, 4), f32)
    aov = {k: np.zeros((H, W), np.uint32) for k in ("shape_index", "material_index", "primitive_index",
                                                    "mesh_complexity", "scene_complexity")}
    aov.update({k: np.zeros((H, W), f32) for k in ("time", "u", "v")})
    aov["normal"] = np.zeros((H, W, 3), f32)
    query = NONE
    half = f32(0.5)
    for y in range(H):
        for x in range(W):
            sx, sy = (f32(x) + half) / f32(W), (f32(y) + half) / f32(H)
            aspect = f32(W) / f32(H)
            v = pr._normalize([(sx - half) * aspect, half - sy, f32(-1.0)])
            O = pr._mat_vec(to, [f32(0.0)] * 3, 1.0)
            V = pr._mat_vec(to, v, 0.0)
            h = tr.trace(W_.S, O, V, pr.HIT_TIME_LIMIT)
            miss = h.shape == tr.SHAPE_INDEX_NONE
            n = uv = None
            mat = 0
            if not miss:
                n, _, uv = tr.hit_attributes(W_.S, h)
                mat = W_.S.shape_material[h.shape]
            c = [f32(0.0)] * 3
            if mode in (0, 1):
                if miss:
                    c = _mat3(XYZ_TO_SRGB, observe_d65(W_.sky_spectrum(V)))
                else:
                    c = _mat3(XYZ_TO_SRGB, base_color(W_, mat, uv))
                    if mode == 1:
                        dn = pr._dot(n, [-V[0], -V[1], -V[2]])
                        c = [ck * dn for ck in c]
            elif mode == 2:
                c = [half * (f32(1.0) - V[k]) for k in range(3)] if miss else [half * (n[k] + f32(1.0)) for k in range(3)]
            elif mode == 3 and not miss:
                c = list(COLORS[mat % 20])
            elif mode == 4 and not miss:
                c = list(COLORS[h.prim % 20])
            elif mode in (5, 6):
                cnt = f32(h.mesh_complexity if mode == 5 else h.scene_complexity)
                c = [(f32(0.0) * cnt) / f32(256.0), (f32(1.0) * cnt) / f32(256.0), (f32(0.0) * cnt) / f32(256.0)]
            if h.shape == selected:
                c = [c[0] * f32(1.0), c[1] * half, c[2] * half]
            c = [ck * f32(brightness) for ck in c]
            if (x, y) == tuple(mouse):
                query = h.shape
            img[y, x] = [c[0], c[1], c[2], f32(1.0)]
            aov["shape_index"][y, x] = h.shape
            aov["mesh_complexity"][y, x] = h.mesh_complexity
            aov["scene_complexity"][y, x] = h.scene_complexity
            if not miss:
                aov["time"][y, x] = h.time
                aov["material_index"][y, x] = mat
                aov["primitive_index"][y, x] = h.prim
                aov["normal"][y, x] = n
                aov["u"][y, x], aov["v"][y, x] = uv
    return img, aov, query
