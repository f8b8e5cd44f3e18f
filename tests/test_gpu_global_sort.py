"""Global ray sort mode (PT_GLOBAL_SORT=1, kernels.hip "Global ray sort"):
extend traces the frame's rays in (octant, origin cell) key order through a
per-round count / scan / scatter pass, instead of tile by tile.  The order
changes only which rays share a wave, so state, hits and the image must stay
bit-identical to the oracle (basic_trace.glsl / basic_scatter.glsl)."""
from __future__ import annotations

import numpy as np
import pytest

import fuzz_scenes
from test_gpu_parity import compare_state, render_pair

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev(pt):
    if pt.device_count() < 1:
        pytest.skip("no HIP device")
    d = pt.Device(0)
    yield d
    d.close()


@pytest.fixture
def gsort(monkeypatch):
    monkeypatch.setenv("PT_GLOBAL_SORT", "1")


@pytest.mark.parametrize("config,W,H,schedule,camera", [
    (1, 64, 64, [2, 1, 1], 0),
    (2, 96, 96, [2, 1], 0),
    (3, 1920, 1080, [2, 1, 1, 1], 0),   # C3 at full size: 8100 tiles over 254 sort chunks
    (5, 300, 33, [2, 1], 1),            # ragged tiles, 360 camera, all material types
])
def test_global_sort_bit_exact(pt, dev, gsort, config, W, H, schedule, camera):
    gs, os_, ga, oa = render_pair(pt, dev, config, W, H, schedule, camera=camera, fused=0)
    compare_state(gs, os_)
    assert oa[..., 3].sum() > 0
    assert np.array_equal(ga.view(np.uint32), oa.view(np.uint32))


@pytest.mark.parametrize("seed", [1, 4, 7])
def test_global_sort_fuzz_scenes(pt, dev, gsort, seed):
    s, st = fuzz_scenes.build(pt, seed)
    gs, os_, ga, oa = render_pair(pt, dev, None, 72, 40, [2, 1, 1], flags=st["flags"],
                                  termination=st["termination"], scene=s, fused=0)
    compare_state(gs, os_)
    assert np.array_equal(ga.view(np.uint32), oa.view(np.uint32))
    s.close()


def test_global_sort_partition_and_stats(pt, dev, gsort):
    """A band partition in sort mode, and ptExtendStats between rounds (it
    traces the slots' rays without storing): the next rounds still match."""
    import oracle_lib
    s = pt.Scene.config(3)
    W, H = 160, 90
    ds = pt.DeviceScene(dev)
    ds.update(s)
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb, rank=1, nranks=2)
    o = oracle_lib.OracleRenderer(s.packs(), W, H, rank=1, nranks=2)
    for x in (r, o):
        x.RenderFlags = 3
        x.reset()
        x.run(2)
    st = r.extend_stats()
    assert st["rays"] == int(np.sum(pt.owned_pixels(W, H, 1, 2)))
    for x in (r, o):
        x.run(1)
    dev.synchronize()
    compare_state(r.read_state(), o.state())
    assert np.array_equal(sb.read().view(np.uint32), o.accum().view(np.uint32))
    for x in (r, sb, ds):
        x.close()
