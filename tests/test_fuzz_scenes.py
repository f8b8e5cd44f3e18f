"""CPU side of the fuzz parity tests: the random scenes build and pack, their
TLAS / BLAS arrays are consistent, and the oracle renders them to finite
values (the GPU comparison itself is tests/test_gpu_fuzz.py)."""
from __future__ import annotations

import numpy as np
import pytest

import fuzz_scenes
import oracle_lib


@pytest.mark.parametrize("seed", [0, 3, 7])
def test_random_scene_packs_and_renders(pt, seed):
    s, st = fuzz_scenes.build(pt, seed)
    a = s.arrays()
    shapes = a["shapes"]
    assert len(shapes) >= 4
    assert len(a["shape_nodes"]) == 2 * len(shapes) - 1          # binary TLAS over the shapes
    mesh = shapes[shapes["Type"] == 0]          # PT_SHAPE_TYPE_MESH_INSTANCE
    assert len(mesh) >= 1 and (mesh["MeshRootNodeIndex"] < len(a["mesh_nodes"])).all()
    o = oracle_lib.OracleRenderer(s.packs(), 16, 8, threads=4)
    o.RenderFlags = st["flags"]
    o.PathTerminationProbability = st["termination"]
    o.reset()
    o.run(2)
    o.run(1)
    state, acc = o.state(), o.accum()
    assert np.isfinite(acc).all()
    assert np.isfinite(state["throughput"]).all() and np.isfinite(state["probability"]).all()
    o.close()
    s.close()


def test_random_scenes_differ_by_seed(pt):
    a, _ = fuzz_scenes.build(pt, 1)
    b, _ = fuzz_scenes.build(pt, 2)
    assert a.arrays()["mesh_faces"].tobytes() != b.arrays()["mesh_faces"].tobytes()
    a.close()
    b.close()
