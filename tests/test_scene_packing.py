"""Host scene packing (restatement of PackSceneData, scene.cpp:1115-1621):
BVH invariants of the BLAS (BuildMeshNode, scene.cpp:435-599) and TLAS
(scene.cpp:1346-1498), material / texture / camera packing, and a regression
pin of the packed bytes (tests/golden/scene_packs.json)."""
from __future__ import annotations

import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

GOLDEN = Path(__file__).resolve().parent / "golden"


@pytest.fixture(scope="module")
def scenes(pt):
    out = {c: pt.Scene.config(c) for c in (1, 2, 3, 5)}
    yield out
    for s in out.values():
        s.close()


def _contains(outer_min, outer_max, inner_min, inner_max):
    return np.all(outer_min <= inner_min) and np.all(inner_max <= outer_max)


def check_blas(nodes, faces, root, face_range):
    """Walks one mesh's BLAS from `root`; returns (depth, faces seen)."""
    seen = []
    depth = 0
    stack = [(root, 1)]
    while stack:
        i, d = stack.pop()
        depth = max(depth, d)
        n = nodes[i]
        lo, hi = n["Minimum"], n["Maximum"]
        if n["FaceEndIndex"] > 0:
            b, e = int(n["FaceBeginOrNodeIndex"]), int(n["FaceEndIndex"])
            assert face_range[0] <= b < e <= face_range[1]
            for f in range(b, e):
                P = np.stack([faces[f]["Position0"], faces[f]["Position1"], faces[f]["Position2"]])
                assert _contains(lo, hi, P.min(0), P.max(0)), f"face {f} outside leaf {i}"
            seen.extend(range(b, e))
        else:
            a = int(n["FaceBeginOrNodeIndex"])
            for c in (a, a + 1):
                assert _contains(lo, hi, nodes[c]["Minimum"], nodes[c]["Maximum"]), f"child {c} outside {i}"
                stack.append((c, d + 1))
    return depth, seen


@pytest.mark.parametrize("cfg", [3, 5])
def test_blas_invariants(scenes, cfg):
    a = scenes[cfg].arrays()
    shapes, nodes, faces = a["shapes"], a["mesh_nodes"], a["mesh_faces"]
    mesh_shapes = shapes[shapes["Type"] == 0]   # SHAPE_TYPE_MESH_INSTANCE
    assert len(mesh_shapes) >= 1
    root = int(mesh_shapes[0]["MeshRootNodeIndex"])
    depth, seen = check_blas(nodes, faces, root, (0, len(faces)))
    assert sorted(seen) == list(range(len(faces))), "leaves must partition the faces"
    assert depth <= 32
    assert len(nodes) == 2 * np.count_nonzero(nodes["FaceEndIndex"] > 0) - 1


def test_room_mesh_shape(scenes):
    a = scenes[3].arrays()
    assert len(a["mesh_faces"]) == 3976
    assert len(a["mesh_nodes"]) == 6243
    v = a["mesh_vertices"]
    assert np.all(np.concatenate([a["mesh_faces"][f"VertexIndex{k}"] for k in range(3)]) < len(v))


@pytest.mark.parametrize("cfg", [1, 2, 3, 5])
def test_tlas_invariants(scenes, cfg):
    a = scenes[cfg].arrays()
    nodes, shapes = a["shape_nodes"], a["shapes"]
    g = a["globals"][0]
    assert g["ShapeCount"] == len(shapes)
    leaves = []
    stack = [0]
    while stack:
        i = stack.pop()
        n = nodes[i]
        ch = int(n["ChildNodeIndices"])
        if ch == 0:
            leaves.append(int(n["ShapeIndex"]))
            continue
        for c in (ch & 0xFFFF, ch >> 16):
            assert 0 < c < len(nodes)
            assert _contains(n["Minimum"], n["Maximum"], nodes[c]["Minimum"], nodes[c]["Maximum"])
            stack.append(c)
    assert sorted(leaves) == list(range(len(shapes))), "every shape reachable exactly once"
    assert len(nodes) == 2 * len(shapes) - 1


@pytest.mark.parametrize("cfg", [1, 2, 3, 5])
def test_material_and_texture_references(scenes, cfg):
    a = scenes[cfg].arrays()
    words = a["materials"]
    n_mat = len(words) // 32
    assert len(words) % 32 == 0 and n_mat >= 2
    # fallback OpenPBR occupies slots 0-1 (scene.cpp:1236-1263)
    assert words[0] == 3
    assert np.all(a["shapes"]["MaterialIndex"] < n_mat)
    tex = a["textures"]
    lo, hi = tex["AtlasPlacementMinimum"], tex["AtlasPlacementMaximum"]
    # v is flipped: Minimum.y is the bottom texel row (scene.cpp:1168-1176)
    assert np.all((lo >= 0) & (lo <= 1) & (hi >= 0) & (hi <= 1))
    assert np.all(lo[:, 0] < hi[:, 0]) and np.all(lo[:, 1] > hi[:, 1])


def test_atlas_placements_disjoint(scenes):
    tex = scenes[5].arrays()["textures"]
    for i in range(len(tex)):
        for j in range(i + 1, len(tex)):
            if tex[i]["AtlasImageIndex"] != tex[j]["AtlasImageIndex"]:
                continue
            pa = np.stack([tex[i]["AtlasPlacementMinimum"], tex[i]["AtlasPlacementMaximum"]])
            pb = np.stack([tex[j]["AtlasPlacementMinimum"], tex[j]["AtlasPlacementMaximum"]])
            a0, a1, b0, b1 = pa.min(0), pa.max(0), pb.min(0), pb.max(0)
            overlap = np.all(np.minimum(a1, b1) > np.maximum(a0, b0))
            assert not overlap, (i, j)


def test_camera_packing(scenes):
    cams = scenes[5].arrays()["cameras"]
    assert len(cams) == 2
    thin, pano = cams
    assert thin["Model"] == 1 and pano["Model"] == 2
    # thin lens: 32x16 mm sensor, f = 50 mm, aperture 20 mm (diameter), focus 3 m
    assert np.allclose(thin["SensorSize"], [0.032, 0.016])
    assert np.isclose(thin["FocalLength"], 0.050)
    assert np.isclose(thin["ApertureRadius"], 0.010)


def test_pinhole_sensor_is_two_to_one(scenes):
    """SensorSize.y = SensorSize.x / 2 hard-coded (scene.cpp:1518-1522)."""
    c = scenes[1].arrays()["cameras"][0]
    assert c["Model"] == 0
    assert np.isclose(c["SensorSize"][1], c["SensorSize"][0] / 2)


def test_packing_is_deterministic(pt):
    h = []
    for _ in range(2):
        s = pt.Scene.config(2)
        h.append({k: hashlib.sha256(v.tobytes()).hexdigest() for k, v in s.arrays().items()})
        s.close()
    assert h[0] == h[1]


@pytest.mark.parametrize("cfg", [1, 2, 3, 5])
def test_packed_bytes_match_golden(scenes, cfg):
    gold = json.loads((GOLDEN / "scene_packs.json").read_text())[str(cfg)]
    for k, v in scenes[cfg].arrays().items():
        assert len(v) == gold["counts"][k], k
        assert hashlib.sha256(v.tobytes()).hexdigest() == gold[k], k


def test_custom_mesh_bvh(pt):
    """BuildMeshNode on a random triangle soup: invariants hold and the flat
    node count is 2*leaves-1."""
    rng = np.random.default_rng(4)
    F = 300
    centers = rng.uniform(-3, 3, size=(F, 1, 3))
    pos = (centers + rng.normal(scale=0.2, size=(F, 3, 3))).reshape(-1, 3).astype(np.float32)
    idx = np.arange(3 * F, dtype=np.uint32)
    s = pt.Scene.create()
    mesh = s.create_mesh(pos, idx)
    s.create_entity(pt.ENTITY_MESH_INSTANCE, position=(0, 0, 1))
    e = s.create_entity(pt.ENTITY_MESH_INSTANCE, position=(0, 0, 1))
    s.set_mesh(e, mesh)
    s.pack()
    a = s.arrays()
    shapes = a["shapes"][a["shapes"]["Type"] == 0]
    root = int(shapes[-1]["MeshRootNodeIndex"])
    depth, seen = check_blas(a["mesh_nodes"], a["mesh_faces"], root, (0, len(a["mesh_faces"])))
    assert sorted(seen) == list(range(F))
    assert depth - 1 == pt.mesh_depth(mesh)   # mesh::Depth counts edges (scene.cpp:595)
    s.close()


def test_spectrum_coefficients_properties(pt):
    """RGB -> parametric spectrum (spectrum.cpp:439-479, evaluated as in
    spectrum.glsl.inc:169-173): gray is flat, white/black saturate, red rises
    toward long wavelengths."""
    lam = np.linspace(400, 700, 31)

    def ev(rgb):
        c = pt.spectrum_coefficients(rgb).astype(np.float64)
        x = (c[0] * lam + c[1]) * lam + c[2]
        return 0.5 + x / (2 * np.sqrt(1 + x * x))
    assert np.all(np.abs(ev([0.5, 0.5, 0.5]) - 0.5) < 0.02)
    assert np.all(ev([1, 1, 1]) > 0.9)
    assert np.all(ev([0, 0, 0]) < 0.1)
    red = ev([0.8, 0.3, 0.3])
    assert red[-1] > red[5] + 0.3
