"""Cross-check of the oracle's rounds against a second restatement written
from the GLSL text apart from it (tests/path_restatement.py, with
tests/trace_restatement.py for Trace): C1's scene (diffuse sphere and plane
with a nearest-filtered checker texture, constant sky) and C3's (the room
mesh with its bilinear-filtered texture) after Reset, Run(2), Run(1), Run(1)
-- every slot's ray, Lambda0, throughput, probability, sample and
active-shape stack, and every accumulated pixel, bit for bit; with and
without jitter, with Russian roulette, accumulate and overwrite.  A metal
room adds the metal BSDF, sky light sampling and the textured sky."""
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


def metal_room(pt):
    """Diffuse floor (nearest checker) and walls, metal shapes -- mirror
    (Dirac), rough, anisotropic, roughness-textured, a metal mesh -- under an
    HDR sky texture (bilinear) sampled by the vMF lobe half the time."""
    import fuzz_scenes
    rng = np.random.default_rng(7)
    s = pt.Scene.empty()
    checker = s.create_checker_texture("Checker", pt.TEXTURE_REFLECTANCE_WITH_ALPHA,
                                       (0.9, 0.9, 0.9, 1.0), (0.2, 0.3, 0.7, 1.0))
    rough_tex = s.create_texture("Noise", pt.TEXTURE_REFLECTANCE_WITH_ALPHA,
                                 fuzz_scenes.random_texture(rng, 16, 8))
    floor = s.create_material(pt.MATERIAL_BASIC_DIFFUSE, "Floor", BaseColor=(0.8, 0.7, 0.6))
    s.set_material_parameter(floor, "BaseTexture", checker)
    wall = s.create_material(pt.MATERIAL_BASIC_DIFFUSE, "Wall", BaseColor=(0.3, 0.6, 0.4))
    mirror = s.create_material(pt.MATERIAL_BASIC_METAL, "Mirror", BaseColor=(0.9, 0.9, 0.95),
                               SpecularColor=(1.0, 1.0, 1.0), Roughness=0.0)
    gold = s.create_material(pt.MATERIAL_BASIC_METAL, "Gold", BaseColor=(1.0, 0.78, 0.34),
                             SpecularColor=(0.9, 0.6, 0.3), Roughness=0.35)
    brushed = s.create_material(pt.MATERIAL_BASIC_METAL, "Brushed", BaseColor=(0.6, 0.6, 0.65),
                                SpecularColor=(0.8, 0.8, 0.9), Roughness=0.25, RoughnessAnisotropy=0.7)
    spotty = s.create_material(pt.MATERIAL_BASIC_METAL, "Spotty", BaseColor=(0.7, 0.4, 0.4),
                               SpecularColor=(0.9, 0.9, 0.9), Roughness=0.5)
    s.set_material_parameter(spotty, "RoughnessTexture", rough_tex)
    s.create_entity(pt.ENTITY_PLANE, position=(0.0, 0.0, -1.0), material=floor)
    s.create_entity(pt.ENTITY_CUBE, position=(2.5, 1.5, 0.0), rotation=(0.0, 0.0, 0.4),
                    scale=(0.4, 1.5, 1.0), material=wall)
    s.create_entity(pt.ENTITY_SPHERE, position=(-1.2, 0.0, 0.0), scale=(0.8, 0.8, 0.8), material=mirror)
    s.create_entity(pt.ENTITY_SPHERE, position=(0.6, -0.6, -0.3), scale=(0.6, 0.6, 0.6), material=gold)
    s.create_entity(pt.ENTITY_CUBE, position=(0.3, 1.4, -0.2), rotation=(0.3, 0.2, 0.5),
                    scale=(0.6, 0.6, 0.6), material=brushed)
    blob = s.create_mesh(*fuzz_scenes.blob_mesh(rng, 8, 12, 0.15), name="Blob")
    e = s.create_entity(pt.ENTITY_MESH_INSTANCE, position=(1.6, -0.2, 0.1), scale=(0.5, 0.5, 0.5), material=spotty)
    s.set_mesh(e, blob)
    sky = s.create_texture("Sky", pt.TEXTURE_RADIANCE, fuzz_scenes.random_sky(rng))
    s.set_root(scatter_rate=0.0, skybox_brightness=1.3, skybox_sampling_probability=0.5, skybox=sky)
    cam = s.create_entity(pt.ENTITY_CAMERA, position=(0.0, -6.0, 1.0), rotation=(1.45, 0.0, 0.0))
    s.set_camera_pinhole(cam, fov_degrees=60.0)
    s.pack()
    return s


@pytest.mark.parametrize("flags,ptp", [(3, 0.0), (1, 0.2)])
def test_metal_room_rounds_match_independent_restatement(pt, flags, ptp):
    """Metal BSDF sampling and evaluation (GGX, F82-tint Fresnel), sky light
    sampling (vMF) and the textured sky, restated apart from the oracle."""
    s = metal_room(pt)
    W, H, schedule = 16, 12, [2, 1, 1]
    pr.STATS.clear()
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
            assert np.array_equal(bits(sl.thr), want["throughput"].view(np.uint32)), (where, "throughput")
            assert np.array_equal(bits(sl.prob), want["probability"].view(np.uint32)), (where, "probability")
            assert np.array_equal(bits(sl.sample), want["sample"].view(np.uint32)), (where, "sample")
    assert np.array_equal(bits(accum), oa.view(np.uint32)), "accumulator"
    assert oa[..., 3].sum() > 0 and oa[..., :3].sum() > 0
    for branch in ("diffuse", "metal", "dirac", "light"):
        assert pr.STATS[branch] > 5, dict(pr.STATS)
    s.close()
