"""Cross-check of the oracle's path generation against a second restatement
written from the GLSL text apart from it: after Reset, every pixel's first
ray (origin bits and packed velocity) and normalized Lambda0 must equal a
numpy float32 restatement of

  main's seeding                basic_scatter.glsl:312-318 (tests/kat.py seed / pcg)
  GenerateNewPath               basic_scatter.glsl:7-42
  GenerateCameraRay             scene.glsl.inc:613-655 (pinhole, thin lens, 360)
  RandomPointOnDisk, Random0To1 common.glsl.inc:199-210
  TransformRay, StoreTraceRay   common.glsl.inc:65-72, basic.glsl.inc:133-140

under DESIGN.md §2's convention (normalize = v * (1 / sqrt(dot)), mat4 *
vec4 left to right); sin / cos are the convention's own functions (the
oracle's exported pt_sin / pt_cos), the octahedral packing tests/kat.py's."""
from __future__ import annotations

import numpy as np
import pytest

import fuzz_scenes
import kat
import oracle_lib

f32 = np.float32
TAU = f32(6.283185306)     # common.glsl.inc:7
PI = f32(3.141592653)      # common.glsl.inc:6


def _normalize(v):
    r = f32(1.0) / np.sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2])
    return [v[0] * r, v[1] * r, v[2] * r]


def _mat_vec(m, v, w):
    w = f32(w)
    return [((m[r] * v[0] + m[4 + r] * v[1]) + m[8 + r] * v[2]) + m[12 + r] * w for r in range(3)]


def new_path(cam, x, y, W, H, flags, frame):
    """(origin, packed velocity, lambda0) of GenerateNewPath at pixel (x, y)."""
    L = oracle_lib.lib()
    state = kat.seed(x, y, frame)

    def r01():
        nonlocal state
        v, state = kat.pcg(state)
        return f32(v) / f32(4294967296.0)

    def disk():
        r = np.sqrt(r01())
        theta = r01() * TAU
        return r * f32(L.oracle_fp_cos(theta)), r * f32(L.oracle_fp_sin(theta))

    if flags & 2:                                   # RENDER_FLAG_SAMPLE_JITTER
        jx = r01()
        jy = r01()
        sx, sy = f32(x) + jx, f32(y) + jy
    else:
        sx, sy = f32(x) + f32(0.5), f32(y) + f32(0.5)
    nx, ny = sx / f32(W), sy / f32(H)
    model = int(cam["Model"])
    size = cam["SensorSize"].astype(np.float32)
    if model in (0, 1):
        sp = [-size[0] * (nx - f32(0.5)), -size[1] * (f32(0.5) - ny), f32(cam["SensorDistance"])]
        if model == 0:
            dx, dy = disk()
            a = f32(cam["ApertureRadius"])
            o = [a * dx, a * dy, f32(0.0)]
            v = _normalize([o[0] - sp[0], o[1] - sp[1], o[2] - sp[2]])
        else:
            fl = f32(cam["FocalLength"])
            den = sp[2] - fl
            op = [(-sp[i] * fl) / den for i in range(3)]
            dx, dy = disk()
            a = f32(cam["ApertureRadius"])
            o = [a * dx, a * dy, f32(0.0)]
            v = _normalize([op[0] - o[0], op[1] - o[1], op[2] - o[2]])
    else:
        phi = (nx - f32(0.5)) * TAU
        theta = (f32(0.5) - ny) * PI
        ct, st = f32(L.oracle_fp_cos(theta)), f32(L.oracle_fp_sin(theta))
        o = [f32(0.0)] * 3
        v = [ct * f32(L.oracle_fp_sin(phi)), st, -ct * f32(L.oracle_fp_cos(phi))]
    to = cam["Transform"]["To"].astype(np.float32).reshape(16)
    O = _mat_vec(to, o, 1.0)
    V = _mat_vec(to, v, 0.0)
    lam = r01()
    return np.array(O, np.float32), int(kat.pack_unit_vector(np.array([V], np.float32))[0]), lam


def check(scene, W, H, camera, flags, frame):
    o = oracle_lib.OracleRenderer(scene.packs(), W, H)
    o.CameraIndex = camera
    o.RenderFlags = flags
    o.FrameIndex = frame
    o.reset()
    st = o.state()
    o.close()
    cam = scene.arrays()["cameras"][camera]
    for y in range(H):
        for x in range(W):
            org, pv, lam = new_path(cam, x, y, W, H, flags, frame)
            s = st[y, x]
            assert np.array_equal(s["origin"].view(np.uint32), org.view(np.uint32)), (x, y, "origin")
            assert int(s["packed_velocity"]) == pv, (x, y, "velocity")
            assert np.float32(s["lambda0"]).view(np.uint32) == lam.view(np.uint32), (x, y, "lambda0")
    return int(cam["Model"])


@pytest.mark.parametrize("config,camera,flags", [(1, 0, 3), (1, 0, 1), (3, 0, 3), (5, 0, 3), (5, 1, 2)])
def test_new_paths_match_independent_restatement(pt, config, camera, flags):
    s = pt.Scene.config(config)
    if camera >= len(s.arrays()["cameras"]):
        pytest.skip("config has one camera")
    check(s, 24, 18, camera, flags, frame=7 + config)
    s.close()


def test_new_paths_cover_every_camera_model(pt):
    """Fuzz scenes pick pinhole, thin-lens and 360 cameras: all three models
    restate identically."""
    models = set()
    for seed in range(12):
        s, _ = fuzz_scenes.build(pt, seed)
        models.add(check(s, 12, 8, 0, 3, frame=seed))
        s.close()
        if models == {0, 1, 2}:
            break
    assert models == {0, 1, 2}
