"""Editor preview (preview_render.glsl:96-178) restated by the oracle:
structural checks of the seven modes, AOVs, selection tint and pick query."""
from __future__ import annotations

import numpy as np
import pytest

import oracle_lib

NONE = 0xFFFFFFFF


def camera_to(scene):
    return scene.arrays()["cameras"][0]["Transform"]["To"]


@pytest.fixture(scope="module")
def scenes(pt):
    out = {c: pt.Scene.config(c) for c in (1, 3, 5)}
    yield out
    for s in out.values():
        s.close()


def run(pt, scene, mode, W=48, H=32, **kw):
    p = pt.PreviewParameters(camera_to(scene), RenderMode=mode, RenderSizeX=W, RenderSizeY=H, **kw)
    return oracle_lib.preview(scene.packs(), p)


def test_normal_mode_matches_aovs(pt, scenes):
    img, aov, _ = run(pt, scenes[5], pt.PREVIEW_RENDER_MODE_NORMAL)
    hit = aov["shape_index"] != NONE
    assert hit.any() and (~hit).any() is not None
    assert np.allclose(img[hit][:, :3], 0.5 * (aov["normal"][hit] + 1), atol=1e-6)
    assert np.allclose(np.linalg.norm(aov["normal"][hit], axis=1), 1, atol=1e-5)
    assert np.all(img[..., 3] == 1)


def test_id_modes_use_palette(pt, scenes):
    img, aov, _ = run(pt, scenes[5], pt.PREVIEW_RENDER_MODE_MATERIAL_INDEX)
    hit = aov["shape_index"] != NONE
    assert np.all(img[~hit][:, :3] == 0)
    colors = {tuple(np.round(c, 3)) for c in img[hit][:, :3]}
    assert len(colors) >= 2
    img2, aov2, _ = run(pt, scenes[3], pt.PREVIEW_RENDER_MODE_PRIMITIVE_INDEX)
    assert len(np.unique(aov2["primitive_index"][aov2["shape_index"] != NONE])) > 20


def test_complexity_counts(pt, scenes):
    _, aov, _ = run(pt, scenes[3], pt.PREVIEW_RENDER_MODE_MESH_COMPLEXITY)
    assert np.all(aov["scene_complexity"] == 1)        # one shape: the TLAS root is its leaf
    assert np.all(aov["mesh_complexity"] >= 1)
    img, aov5, _ = run(pt, scenes[5], pt.PREVIEW_RENDER_MODE_SCENE_COMPLEXITY)
    # with nothing selected (0xFFFFFFFF) the sky counts as "selected" and is
    # tinted by (1, 0.5, 0.5) — faithful to preview_render.glsl:164-165
    tint = np.where(aov5["shape_index"] == NONE, 0.5, 1.0)
    assert np.allclose(img[..., 1], aov5["scene_complexity"] / 256.0 * tint)
    assert np.all(img[..., 0] == 0) and np.all(img[..., 2] == 0)


def test_selection_tint_and_pick(pt, scenes):
    s = scenes[5]
    # select an index no pixel has, so the sky is not tinted in the base image
    base, aov, q = run(pt, s, pt.PREVIEW_RENDER_MODE_BASE_COLOR_SHADED, MouseX=24, MouseY=16,
                       SelectedShapeIndex=0xFFFFFFFE)
    assert q == aov["shape_index"][16, 24]
    sel = int(aov["shape_index"][16, 24])
    tinted, _, _ = run(pt, s, pt.PREVIEW_RENDER_MODE_BASE_COLOR_SHADED, SelectedShapeIndex=sel, Brightness=2.0)
    m = aov["shape_index"] == sel
    assert np.allclose(tinted[m][:, :3], 2.0 * base[m][:, :3] * [1.0, 0.5, 0.5], rtol=1e-6, atol=1e-7)
    assert np.allclose(tinted[~m][:, :3], 2.0 * base[~m][:, :3], rtol=1e-6, atol=1e-7)
    _, _, q2 = run(pt, s, 0, MouseX=10_000, MouseY=10_000)
    assert q2 == NONE                                   # outside the image: query untouched


def test_base_color_of_white_sky(pt, scenes):
    """No skybox texture: the sky spectrum is (0, 0, 100, 1), i.e. a
    reflectance of ~1 everywhere, observed under D65 -> near-white sRGB."""
    img, aov, _ = run(pt, scenes[1], pt.PREVIEW_RENDER_MODE_BASE_COLOR, W=32, H=16, SelectedShapeIndex=0xFFFFFFFE)
    sky = aov["shape_index"] == NONE
    if sky.any():
        c = img[sky][:, :3]
        assert np.all(c > 0.8) and np.all(c < 1.2)
