"""Cross-check of the oracle's RenderPreview restatement against a second one
written apart from it (tests/preview_restatement.py): the image bit for bit,
every AOV field and the pick query, for all seven render modes on configs 1,
2, 3 and 5 (the C2 sky spectrum, C3's bilinear texture, C5's translucent
base colours) and a fuzz scene."""
from __future__ import annotations

import numpy as np
import pytest

import fuzz_scenes
import oracle_lib
import preview_restatement as prv


def check(pt, s, mode, W=40, H=24):
    cam = s.arrays()["cameras"][0]["Transform"]["To"]
    p = pt.PreviewParameters(cam, RenderMode=mode, RenderSizeX=W, RenderSizeY=H, Brightness=1.5,
                             SelectedShapeIndex=1, MouseX=17, MouseY=11)
    want, want_aov, want_q = oracle_lib.preview(s.packs(), p)
    got, aov, q = prv.preview(s, p.camera_to, mode, W, H, brightness=1.5, selected=1, mouse=(17, 11))
    same = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
    assert same.all(), np.argwhere(~same)[:5]
    for name in ("shape_index", "material_index", "primitive_index", "mesh_complexity", "scene_complexity"):
        assert np.array_equal(aov[name], want_aov[name].astype(np.uint32)), name
    for name in ("time", "u", "v", "normal"):
        assert np.array_equal(aov[name].view(np.uint32), np.ascontiguousarray(want_aov[name]).view(np.uint32)), name
    assert q == want_q
    return want_aov


@pytest.mark.parametrize("config", [1, 2, 3, 5])
@pytest.mark.parametrize("mode", range(7))
def test_preview_matches_independent_restatement(pt, config, mode):
    s = pt.Scene.config(config)
    aov = check(pt, s, mode)
    assert (aov["shape_index"] != 0xFFFFFFFF).sum() > 20
    s.close()


@pytest.mark.parametrize("seed", [2, 9])
def test_preview_fuzz_matches_independent_restatement(pt, seed):
    s, _ = fuzz_scenes.build(pt, seed)
    for mode in (0, 1, 4, 6):
        check(pt, s, mode, 32, 20)
    s.close()
