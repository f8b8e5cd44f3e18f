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
import oracle_lib
import path_restatement as pr


def new_path(cam, x, y, W, H, flags, frame):
    """(origin, packed velocity, lambda0) of GenerateNewPath at pixel (x, y)
    from main's seed (tests/path_restatement.py)."""
    O, pv, lam = pr.new_path(None, cam, pr.Rng(x, y, frame), x, y, W, H, flags)
    return np.array(O, np.float32), pv, lam


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
