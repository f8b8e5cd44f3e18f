"""The product's BVH builders (csrc/scene/scene.cpp: BuildMeshNode, mesh
packing, the TLAS pairing) against a second restatement written separately
from the reference's text (tests/builder_restatement.py): packed mesh nodes,
face order and shape nodes bit for bit.  CPU only."""
from __future__ import annotations

import numpy as np
import pytest

import builder_restatement as BR


def packed_mesh_of(pt, P, F):
    s = pt.Scene.empty()
    m = s.create_mesh(P, F)
    s.create_entity(pt.ENTITY_MESH_INSTANCE)
    e = s.create_entity(pt.ENTITY_MESH_INSTANCE)
    s.set_mesh(e, m)
    s.pack()
    a = s.arrays()
    s.close()
    return a


def check_mesh(pt, P, F):
    P = np.ascontiguousarray(P, dtype=np.float32)
    F = np.ascontiguousarray(F, dtype=np.uint32).reshape(-1, 3)
    a = packed_mesh_of(pt, P, F)
    nodes, faces = BR.build_mesh(P, F)
    ref = BR.pack_mesh_nodes(nodes)
    got = a["mesh_nodes"]
    assert len(got) == len(ref), f"{len(got)} nodes vs {len(ref)}"
    gf = np.stack([a["mesh_faces"]["VertexIndex0"], a["mesh_faces"]["VertexIndex1"], a["mesh_faces"]["VertexIndex2"]], 1)
    assert np.array_equal(gf, faces), "face order differs"
    for i, (mn, fb, mx, fe) in enumerate(ref):
        g = got[i]
        assert np.array_equal(g["Minimum"].view(np.uint32), np.array(mn, np.float32).view(np.uint32)), f"node {i} min"
        assert np.array_equal(g["Maximum"].view(np.uint32), np.array(mx, np.float32).view(np.uint32)), f"node {i} max"
        assert (int(g["FaceBeginOrNodeIndex"]), int(g["FaceEndIndex"])) == (fb, fe), f"node {i} indices"
    return len(ref)


def soup(seed, n, axis_aligned=False):
    rng = np.random.default_rng(seed)
    if axis_aligned:
        # coplanar, shared-coordinate triangles on a coarse lattice (ties in
        # bins, centroids and bounds; signed zeros)
        P = rng.integers(-4, 5, size=(3 * n, 3)).astype(np.float32) * np.float32(0.25)
        P[rng.random(3 * n) < 0.1, 2] = np.float32(-0.0)
        P[::7, 0] = 0.0
    else:
        c = rng.normal(size=(n, 3)).astype(np.float32) * 3
        P = (np.repeat(c, 3, 0) + rng.normal(size=(3 * n, 3)).astype(np.float32) * 0.2).astype(np.float32)
    F = np.arange(3 * n, dtype=np.uint32).reshape(-1, 3)
    F = F[rng.permutation(n)]
    return P, F


@pytest.mark.parametrize("seed,n,aa", [(1, 40, False), (2, 700, False), (3, 300, True), (4, 1500, True), (5, 3, False)])
def test_mesh_builder_matches_restatement(pt, seed, n, aa):
    P, F = soup(seed, n, aa)
    assert check_mesh(pt, P, F) >= 1


def mesh_from_packs(a, root):
    """A config scene's mesh as (positions, faces) from its packed faces."""
    f = a["mesh_faces"]
    vi = np.stack([f["VertexIndex0"], f["VertexIndex1"], f["VertexIndex2"]], 1).astype(np.int64)
    P = np.zeros((vi.max() + 1, 3), np.float32)
    for k, name in enumerate(("Position0", "Position1", "Position2")):
        P[vi[:, k]] = f[name]
    return P, vi


@pytest.mark.parametrize("config", [3, 5])
def test_config_meshes_match_restatement(pt, config):
    """The C3 room mesh (3 976 faces) and C5's mesh, rebuilt from their packed
    faces (in the built face order, as a new input order)."""
    s = pt.Scene.config(config)
    a = s.arrays()
    s.close()
    P, F = mesh_from_packs(a, 0)
    assert check_mesh(pt, P, F) > 100


def check_tlas(a):
    ref = BR.build_tlas(a["shapes"], a["mesh_nodes"])
    got = a["shape_nodes"]
    assert len(got) == len(ref)
    for i, (mn, ch, mx, si) in enumerate(ref):
        g = got[i]
        assert np.array_equal(g["Minimum"].view(np.uint32), np.array(mn, np.float32).view(np.uint32)), f"node {i} min"
        assert np.array_equal(g["Maximum"].view(np.uint32), np.array(mx, np.float32).view(np.uint32)), f"node {i} max"
        assert (int(g["ChildNodeIndices"]), int(g["ShapeIndex"])) == (ch, si), f"node {i} links"


@pytest.mark.parametrize("config", [1, 2, 3, 5])
def test_config_tlas_matches_restatement(pt, config):
    s = pt.Scene.config(config)
    check_tlas(s.arrays())
    s.close()


@pytest.mark.parametrize("seed", [7, 8, 9])
def test_random_tlas_matches_restatement(pt, seed):
    """40 shapes of every type, random transforms (rotated, scaled, nested),
    and instances of two meshes."""
    rng = np.random.default_rng(seed)
    s = pt.Scene.empty()
    P, F = soup(seed, 60)
    m1 = s.create_mesh(P, F)
    P2, F2 = soup(seed + 100, 30, True)
    m2 = s.create_mesh(P2, F2)
    parent = None
    for i in range(40):
        t = [pt.ENTITY_SPHERE, pt.ENTITY_CUBE, pt.ENTITY_PLANE, pt.ENTITY_MESH_INSTANCE][rng.integers(0, 4) if i % 9 else 3]
        e = s.create_entity(t, parent=parent if i % 5 == 4 else None,
                            position=tuple(rng.uniform(-20, 20, 3)), rotation=tuple(rng.uniform(-3, 3, 3)),
                            scale=tuple(rng.uniform(0.2, 3, 3)))
        if t == pt.ENTITY_MESH_INSTANCE:
            s.set_mesh(e, m1 if i % 2 else m2)
        if i % 7 == 0:
            parent = e
    s.pack()
    check_tlas(s.arrays())
    s.close()
