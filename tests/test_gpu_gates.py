"""GPU: the host-proved shade specialisations, on scenes that pass and on
scenes that FAIL each gate.  The host picks the shade
instantiation from the packs (runtime.hip SceneMaterialMask, kernels.hip
pt_shade_mats); a wrong gate would silently run a kernel that drops terms the
scene needs.  Each case asserts which variant ran (ptGetBasicRendererShadeInfo)
and that the render is bit-exact against the oracle.

Gates:
* PT_SHADE_SKY clear (sky lobe and sky pdf term dropped): needs
  SkyboxSamplingProbability of bit pattern +0 and a finite vMF pdf for every
  direction (concentration <= 1000, |mean direction|^2 <= 1.01);
* PT_SHADE_TEXWRAP clear (the lean kernel's two-select texel wrap): needs every
  atlas placement inside [0, 1];
* the lean diffuse-mesh kernel: diffuse materials only, meshes only, neither
  of the above;
* grey path records: no translucent and no shaded OpenPBR material.

The raw packs are patched through ctypes (values the scene editor would not
write), the same packs going to the device and to the oracle.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

import oracle_lib
from test_gpu_parity import compare_state, scene_for

pytestmark = pytest.mark.gpu

LEAN = 1   # PT_SHADE_DIFFUSE alone: the lean diffuse-mesh instantiation


@pytest.fixture(scope="module")
def dev(pt):
    if pt.device_count() < 1:
        pytest.skip("no HIP device")
    d = pt.Device(0)
    yield d
    d.close()


class PatchedPacks:
    """A scene's packs with the globals and / or texture records replaced
    (arrays owned here; the scene keeps the rest alive)."""

    def __init__(self, pt, scene, globals_edit=None, textures_edit=None):
        N = pt._native
        self.scene = scene
        p = scene.packs()
        self._p = N.pt_scene_packs()
        C.memmove(C.addressof(self._p), C.addressof(p), C.sizeof(p))
        a = scene.arrays()
        self._g = a["globals"].copy()
        if globals_edit:
            globals_edit(self._g[0])
        self._p.globals = self._g.ctypes.data
        self._t = a["textures"].copy()
        if textures_edit:
            textures_edit(self._t)
        if len(self._t):
            self._p.textures = self._t.ctypes.data

    def packs(self):
        return self._p


def render_and_check(pt, dev, source, W=128, H=72, schedule=(2, 1, 1), termination=0.0):
    ds = pt.DeviceScene(dev)
    ds.update(source)
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    o = oracle_lib.OracleRenderer(source.packs(), W, H)
    for x in (r, o):
        x.RenderFlags = 3
        x.PathTerminationProbability = termination
        x.reset()
    info = r.shade_info()
    for x in (r, o):
        for k in schedule:
            x.run(k)
    dev.synchronize()
    compare_state(r.read_state(), o.state())
    oa = o.accum()
    assert np.array_equal(sb.read().view(np.uint32), oa.view(np.uint32))
    assert oa[..., 3].sum() > 0
    o.close()
    for x in (r, sb, ds):
        x.close()
    return info


def test_lean_positive_control(pt, dev):
    """C3 (diffuse meshes, no sky sampling, unit-square atlas): the lean kernel, grey records."""
    info = render_and_check(pt, dev, scene_for(pt, 3))
    assert info["kernel_mask"] == LEAN and info["grey_records"]
    assert not info["scene_mask"] & (pt.SHADE_SKY | pt.SHADE_TEXWRAP | pt.SHADE_PRIMS)


@pytest.mark.parametrize("case", ["negative-zero-probability", "concentration-over-1000", "mean-direction-overflow"])
def test_sky_gate_failures_run_the_sky_terms(pt, dev, case):
    """SkyboxSamplingProbability = -0.0 (-0 * pdf + 1 * MaterialPDF is -0
    where MaterialPDF is -0, but the skipped form MaterialPDF + 0 is +0), +0
    with a concentration above 1000, +0 with a mean direction of length 10
    (its pdf overflows to inf for directions along it, so +0 * pdf is NaN and
    the skipped term would differ): each keeps the sky terms (PT_SHADE_SKY)
    and renders bit-exactly."""
    s = scene_for(pt, 3)

    def edit(g):
        if case == "negative-zero-probability":
            g["SkyboxSamplingProbability"] = np.float32(-0.0)
        elif case == "concentration-over-1000":
            g["SkyboxSamplingProbability"] = 0.0
            g["SkyboxConcentration"] = 5000.0
            g["SkyboxMeanDirection"] = (0.0, 0.6, 0.8)
        else:
            g["SkyboxSamplingProbability"] = 0.0
            g["SkyboxConcentration"] = 50.0
            g["SkyboxMeanDirection"] = (0.0, 0.0, 10.0)
    src = PatchedPacks(pt, s, globals_edit=edit)
    assert np.signbit(src._g[0]["SkyboxSamplingProbability"]) == (case == "negative-zero-probability")
    info = render_and_check(pt, dev, src)
    assert info["scene_mask"] & pt.SHADE_SKY
    assert info["kernel_mask"] != LEAN and info["kernel_mask"] & pt.SHADE_SKY
    assert info["grey_records"]


def test_texwrap_gate_failure_runs_the_remainder_wrap(pt, dev):
    """A diffuse mesh-only scene whose raw packs place a texture beyond the
    unit square of the atlas (coordinates then wrap past the two-select
    range): PT_SHADE_TEXWRAP, the general instantiation, bit-exact."""
    s = scene_for(pt, 3)

    def edit(t):
        assert len(t) > 0
        t[0]["AtlasPlacementMaximum"] = t[0]["AtlasPlacementMinimum"] + 1.375 * (
            t[0]["AtlasPlacementMaximum"] - t[0]["AtlasPlacementMinimum"])
        t[0]["AtlasPlacementMinimum"][0] -= 0.125
    src = PatchedPacks(pt, s, textures_edit=edit)
    info = render_and_check(pt, dev, src)
    assert info["scene_mask"] & pt.SHADE_TEXWRAP
    assert info["kernel_mask"] != LEAN


@pytest.mark.parametrize("material", ["metal", "glass"])
def test_lean_scene_plus_one_shape(pt, dev, material):
    """The C3 room plus one metal (grey records kept: metal pdfs are scalars)
    or one glass sphere (four-float records: refraction fills the stack and
    Fresnel weights are per wavelength)."""
    s = pt.Scene.config(3)
    if material == "metal":
        m = s.create_material(pt.MATERIAL_BASIC_METAL, "Brass", BaseColor=(0.9, 0.7, 0.3), Roughness=0.2)
    else:
        m = s.create_material(pt.MATERIAL_BASIC_TRANSLUCENT, "Glass", IOR=1.5, Roughness=0.05)
    cam = s.arrays()["cameras"][0]["Transform"]["To"].reshape(4, 4).T
    eye, fwd = cam[:3, 3], -cam[:3, 2]
    s.create_entity(pt.ENTITY_SPHERE, position=tuple(eye + 1.5 * fwd), scale=(0.6, 0.6, 0.6), material=m)
    s.pack()
    info = render_and_check(pt, dev, s)
    want = pt.SHADE_METAL if material == "metal" else pt.SHADE_TRANSLUCENT
    assert info["scene_mask"] & want and info["kernel_mask"] & want
    assert info["grey_records"] == (material == "metal")
    s.close()


@pytest.mark.parametrize("config,metal", [(1, False), (3, False), (3, True)])
def test_fog_without_glass_keeps_four_float_records(pt, dev, config, metal):
    """SceneScatterRate > 0 in a scene with no glass: the
    scene mask (diffuse [+ metal] + scatter) has no translucent bit, but the
    shade instantiation it maps to (PT_MATS_ALL) does and reads the four-float
    record, so the renderer must not take the grey form.  Bit-exact against
    the oracle on the accumulator and on every read_state field, Probability
    included.  In fog that fills the scene no path escapes (a ray to the sky
    always scatters first), so roulette (termination 0.2) ends paths and new
    ones start from the camera."""
    s = scene_for(pt, config)
    owned = None
    if metal:
        owned = s = pt.Scene.config(config)
        m = s.create_material(pt.MATERIAL_BASIC_METAL, "Brass", BaseColor=(0.9, 0.7, 0.3), Roughness=0.2)
        cam = s.arrays()["cameras"][0]["Transform"]["To"].reshape(4, 4).T
        eye, fwd = cam[:3, 3], -cam[:3, 2]
        s.create_entity(pt.ENTITY_SPHERE, position=tuple(eye + 1.5 * fwd), scale=(0.6, 0.6, 0.6), material=m)
        s.pack()

    def edit(g):
        g["SceneScatterRate"] = np.float32(0.35)
    src = PatchedPacks(pt, s, globals_edit=edit)
    info = render_and_check(pt, dev, src, schedule=(2, 1, 1, 1), termination=0.2)
    assert info["scene_mask"] & pt.SHADE_SCATTER
    assert not info["scene_mask"] & pt.SHADE_TRANSLUCENT
    assert info["kernel_mask"] & pt.SHADE_TRANSLUCENT
    assert not info["grey_records"]
    if owned is not None:
        owned.close()


@pytest.mark.parametrize("config,grey", [(1, True), (2, False), (5, False)])
def test_config_variants(pt, dev, config, grey):
    """The other configs' variants: C1 (diffuse sphere + plane) grey, C2 / C5
    (glass) four-float records."""
    info = render_and_check(pt, dev, scene_for(pt, config), W=64, H=48)
    assert info["grey_records"] == grey
    assert info["kernel_mask"] != LEAN


def test_node_cache_layout_is_result_neutral(pt, dev):
    """The LDS node cache's device BVH layout (the top child pairs first,
    every index remapped; runtime.hip NodeCacheLayout): on for the u16-stack
    scenes, off when the stack needs 32-bit entries, and the same hits and
    frames either way -- against the oracle, which traverses the packs'
    original numbering."""
    from test_gpu_parity import compare_hits, random_rays
    for config in (3, 5):
        s = scene_for(pt, config)
        for fmt, cached in ((0, True), (1, False)):
            ds = pt.DeviceScene(dev)
            ds.set_stack_format(fmt)
            ds.update(s)
            assert (ds.node_cache_pairs > 0) == cached
            if cached and config == 3:
                assert ds.node_cache_pairs == 160
            o, v, d = random_rays(s.arrays(), 20000, seed=40 + config)
            compare_hits(ds.trace_rays(o, v, d), oracle_lib.trace_rays(s.packs(), o, v, d))
            ds.close()
