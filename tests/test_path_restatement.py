"""Cross-check of the oracle's rounds against a second restatement written
from the GLSL text apart from it (tests/path_restatement.py, with
tests/trace_restatement.py for Trace): after Reset, Run(2), Run(1), Run(1),
every slot's ray, Lambda0, throughput, probability, sample and active-shape
words, and every accumulated pixel, bit for bit -- on C1 (diffuse sphere and
plane, nearest checker, constant sky), C2 (glass, metal, HDR sky sampled by
the vMF lobe), C5 (both cameras), C3 (the room mesh, bilinear texture), a metal room, and the
random fuzz scenes (OpenPBR fall-through, rough and smooth glass with dispersion,
nested and scattering media, a scattering scene medium, textured roughness,
every camera model); with and without jitter, with Russian roulette,
accumulate and overwrite."""
from __future__ import annotations

import collections

import numpy as np
import pytest

import fuzz_scenes
import oracle_lib
import path_restatement as pr


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


def check(s, W, H, schedule, flags, ptp=0.0, camera=0, openpbr=False):
    """Render with both and compare everything; returns the oracle accumulator."""
    pr.STATS.clear()
    slots, accum = pr.render(s, W, H, schedule, flags=flags, ptp=ptp, camera=camera, openpbr=openpbr)
    o = oracle_lib.OracleRenderer(s.packs(), W, H)
    o.set_openpbr(openpbr)
    o.RenderFlags = flags
    o.PathTerminationProbability = ptp
    o.CameraIndex = camera
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
    return oa


@pytest.mark.parametrize("flags,ptp", [(3, 0.0), (1, 0.0), (3, 0.3), (2, 0.0)])
def test_c1_rounds_match_independent_restatement(pt, flags, ptp):
    s = pt.Scene.config(1)
    oa = check(s, 16, 12, [2, 1, 1], flags, ptp)
    assert oa[..., 3].sum() > 0
    s.close()


@pytest.mark.parametrize("flags", [3, 1])
def test_c3_rounds_match_independent_restatement(pt, flags):
    """C3's room: a textured (bilinear) diffuse mesh under a constant sky."""
    s = pt.Scene.config(3)
    oa = check(s, 12, 8, [2, 1, 1], flags)
    assert oa[..., 3].sum() > 0 and oa[..., :3].sum() > 0     # escapes reached the sky
    s.close()


@pytest.mark.parametrize("config,camera,branches", [
    (2, 0, ("diffuse", "metal", "glass_dirac", "refract", "light")),
    (5, 0, ("diffuse", "metal", "glass_dirac", "refract")),
    (5, 1, ("diffuse", "metal", "refract"))])
def test_config_rounds_match_independent_restatement(pt, config, camera, branches):
    """C2 (a smooth glass sphere, metal and diffuse shapes, the HDR sky) and
    C5 (every basic material, a scattering medium, both of its cameras)."""
    s = pt.Scene.config(config)
    info = s.info
    check(s, 16, 12, [2, 1, 1], info.render_flags, info.termination_probability, camera)
    for branch in branches:
        assert pr.STATS[branch] > 5, dict(pr.STATS)
    s.close()


def test_fuzz_rounds_match_independent_restatement(pt):
    """Fuzz seeds 0-23, each with its own flags, roulette and camera;
    together they take every branch, OpenPBR surfaces (not dispatched by
    the reference, so the path ends there) included."""
    seen = collections.Counter()
    for seed in range(24):
        s, st = fuzz_scenes.build(pt, seed)
        check(s, 12, 8, [2, 1, 1], st["flags"], st["termination"], st["camera"])
        seen.update(pr.STATS)
        s.close()
    for branch in ("diffuse", "metal", "metal_dirac", "glass", "glass_dirac", "reflect", "refract",
                   "medium", "light", "openpbr"):
        assert seen[branch] > 20, dict(seen)


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
    oa = check(s, 16, 12, [2, 1, 1], flags, ptp)
    assert oa[..., 3].sum() > 0 and oa[..., :3].sum() > 0
    for branch in ("diffuse", "metal", "metal_dirac", "light"):
        assert pr.STATS[branch] > 5, dict(pr.STATS)
    s.close()


def fog_glass(pt):
    """Scattering glass: a rough glass block holding forward-scattering fog
    (Henyey-Greenstein g = 0.6) with a smooth, strongly dispersive sphere of
    back-scattering fog (g = -0.5) nested in it, in a hazy scene medium."""
    import fuzz_scenes
    rng = np.random.default_rng(11)
    s = pt.Scene.empty()
    floor = s.create_material(pt.MATERIAL_BASIC_DIFFUSE, "Floor", BaseColor=(0.7, 0.7, 0.7))
    block = s.create_material(pt.MATERIAL_BASIC_TRANSLUCENT, "Block", IOR=1.45, AbbeNumber=40.0, Roughness=0.2,
                              TransmissionColor=(0.9, 0.8, 0.7), TransmissionDepth=0.6)
    s.set_material_parameter(block, "ScatteringColor", (0.8, 0.8, 0.9))
    s.set_material_parameter(block, "ScatteringAnisotropy", 0.6)
    ball = s.create_material(pt.MATERIAL_BASIC_TRANSLUCENT, "Ball", IOR=1.8, AbbeNumber=20.0, Roughness=0.0,
                             TransmissionColor=(0.6, 0.9, 0.8), TransmissionDepth=0.4)
    s.set_material_parameter(ball, "ScatteringColor", (0.5, 0.7, 0.6))
    s.set_material_parameter(ball, "ScatteringAnisotropy", -0.5)
    s.create_entity(pt.ENTITY_PLANE, position=(0.0, 0.0, -1.0), material=floor)
    cube = s.create_entity(pt.ENTITY_CUBE, position=(0.0, 0.0, 0.0), rotation=(0.1, 0.2, 0.3),
                           scale=(1.4, 1.4, 1.0), material=block)
    s.create_entity(pt.ENTITY_SPHERE, parent=cube, scale=(0.55, 0.55, 0.7), material=ball)
    sky = s.create_texture("Sky", pt.TEXTURE_RADIANCE, fuzz_scenes.random_sky(rng))
    s.set_root(scatter_rate=0.02, skybox_brightness=1.0, skybox_sampling_probability=0.5, skybox=sky)
    cam = s.create_entity(pt.ENTITY_CAMERA, position=(0.0, -4.5, 0.6), rotation=(1.45, 0.0, 0.0))
    s.set_camera_pinhole(cam, fov_degrees=50.0)
    s.pack()
    return s


@pytest.mark.parametrize("flags,ptp", [(3, 0.0), (1, 0.1)])
def test_fog_glass_rounds_match_independent_restatement(pt, flags, ptp):
    """Anisotropic medium scattering (SampleDirectionHG), rough refraction
    and reflection with dispersion, nested media, sky light sampling on
    rough glass."""
    s = fog_glass(pt)
    check(s, 16, 12, [2, 1, 1, 1], flags, ptp)
    for branch in ("glass", "glass_dirac", "reflect", "refract", "medium_hg", "light"):
        assert pr.STATS[branch] > 5, sorted(pr.STATS.items())
    s.close()


@pytest.mark.parametrize("flags,ptp", [(3, 0.0), (2, 0.1)])
def test_openpbr_sampler_rounds_match_independent_restatement(pt, flags, ptp):
    """The opt-in OpenPBR sampler (ptSetBasicRendererOpenPBR) on
    tests/test_openpbr.py's scene: parameter draws, coat, metal and
    dielectric base specular, Oren-Nayar diffuse base, the layer walk with a
    bounce limit of 3, OpenPBR media nested with a basic glass."""
    import test_openpbr
    s = test_openpbr.openpbr_scene(pt)
    check(s, 16, 12, [2, 1, 1, 1], flags, ptp, openpbr=True)
    for branch in ("coat_reflect", "coat_refract", "spec_metal", "spec_reflect", "spec_refract", "oren_nayar",
                   "medium_hg", "light"):
        assert pr.STATS[branch] > 10, sorted(pr.STATS.items())
    s.close()
