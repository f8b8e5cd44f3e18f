"""Fuzz parity: random scenes (tests/fuzz_scenes.py) rendered by
libpathtracer.so and by the CPU oracle from the same packs must agree bit for
bit -- every slot's state, every accumulated pixel and the hit records of
random rays.  The scenes combine what the fixed configs keep apart: several
mesh instances under one TLAS, entity hierarchies with rotated and
non-uniformly scaled parents, textured diffuse / anisotropic metal /
dispersive and scattering translucent materials, nested shapes (the
active-shape priority stack), OpenPBR hits, HDR skies with and without vMF
light sampling, all three camera models and the renderer's flag / roulette
settings (basic_scatter.glsl:7-360, scene.glsl.inc:304-762).
"""
from __future__ import annotations

import numpy as np
import pytest

import fuzz_scenes
import oracle_lib
from test_gpu_parity import compare_hits, compare_state, random_rays, render_pair

pytestmark = pytest.mark.gpu

SEEDS = list(range(24))


@pytest.fixture(scope="module")
def dev(pt):
    if pt.device_count() < 1:
        pytest.skip("no HIP device")
    d = pt.Device(0)
    yield d
    d.close()


@pytest.mark.parametrize("seed", SEEDS)
def test_random_scene_bit_exact(pt, dev, seed):
    s, st = fuzz_scenes.build(pt, seed)
    # Separate extend/shade launches for even seeds, the fused round kernel
    # for odd ones (both must equal the oracle).
    fused = 0 if seed % 2 == 0 else 2
    W, H = (72, 40) if seed % 3 else (33, 17)
    gs, os_, ga, oa = render_pair(pt, dev, None, W, H, [2, 1, 1, 1], flags=st["flags"],
                                  termination=st["termination"], scene=s, fused=fused)
    compare_state(gs, os_)
    assert np.array_equal(ga.view(np.uint32), oa.view(np.uint32))
    ds = pt.DeviceScene(dev)
    ds.update(s)
    o, v, d = random_rays(s.arrays(), 8192, seed=seed)
    compare_hits(ds.trace_rays(o, v, d), oracle_lib.trace_rays(s.packs(), o, v, d))
    ds.close()
    s.close()


@pytest.mark.parametrize("seed", SEEDS[::3])
def test_random_scene_round_batches_bit_exact(pt, dev, seed):
    """Round batches (rounds_kernel: several Run(1) rounds of a tile in one
    launch) on the random scenes: Reset, Run(2), then 5 rounds in batches of
    3 (a partial last batch) against 5 oracle Run(1) calls."""
    s, st = fuzz_scenes.build(pt, seed)
    W, H = 72, 40
    ds = pt.DeviceScene(dev)
    ds.update(s)
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    r.set_round_batch(3)
    o = oracle_lib.OracleRenderer(s.packs(), W, H)
    for x in (r, o):
        x.RenderFlags = st["flags"]
        x.PathTerminationProbability = st["termination"]
        x.reset()
        x.run(2)
    r.run_rounds(5)
    for _ in range(5):
        o.run(1)
    dev.synchronize()
    compare_state(r.read_state(), o.state())
    assert np.array_equal(sb.read().view(np.uint32), o.accum().view(np.uint32))
    o.close()
    for x in (r, sb, ds):
        x.close()
    s.close()
