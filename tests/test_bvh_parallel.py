"""The threaded mesh BVH build (BuildMeshSubtree / SplitMeshNode in
csrc/scene/scene.cpp) equals the reference's sequential BuildMeshNode
recursion (scene.cpp:435-599) byte for byte: node array, face order and
depth.  PT_BVH_THREADS=1 runs the sequential recursion."""
from __future__ import annotations

import os

import numpy as np
import pytest

import fuzz_scenes


def build(pt, mesh, threads):
    old = os.environ.get("PT_BVH_THREADS")
    os.environ["PT_BVH_THREADS"] = str(threads)
    try:
        s = pt.Scene.empty()
        m = s.create_mesh(*mesh)
        e = s.create_entity(pt.ENTITY_MESH_INSTANCE)
        s.set_mesh(e, m)
        s.pack()
        a = s.arrays()
        out = (a["mesh_nodes"].tobytes(), a["mesh_faces"].tobytes(), pt.mesh_depth(m))
        s.close()
        return out
    finally:
        if old is None:
            del os.environ["PT_BVH_THREADS"]
        else:
            os.environ["PT_BVH_THREADS"] = old


def meshes():
    rng = np.random.default_rng(5)
    soup = fuzz_scenes.soup_mesh(rng, 120000, 3.0)                  # > 2^16 faces: chunked passes at the top
    blob = fuzz_scenes.blob_mesh(rng, 180, 360, 0.05)
    pos, idx, nrm, uv = fuzz_scenes.blob_mesh(rng, 160, 320, 0.0)
    pos = np.round(pos * 4) / 4                                      # many equal centroids and bounds
    pos[::5] *= -1.0
    pos[pos == 0] = np.where(np.arange((pos == 0).sum()) % 2, 0.0, -0.0)   # signed zeros on the bounds
    quant = (pos.astype(np.float32), idx, nrm, uv)
    flat = (np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]] * 70000, np.float32),
            np.arange(210000, dtype=np.uint32).reshape(-1, 3), None, None)  # identical faces: one leaf
    return {"soup": soup, "blob": blob, "quantized": quant, "identical_faces": flat}


@pytest.mark.parametrize("name", ["soup", "blob", "quantized", "identical_faces"])
def test_threaded_build_equals_sequential(pt, name):
    mesh = meshes()[name]
    seq = build(pt, mesh, 1)
    for threads in (3, 8):
        assert build(pt, mesh, threads) == seq, f"{name}: {threads} threads"
