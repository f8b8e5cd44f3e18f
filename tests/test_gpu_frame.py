"""GPU: ptRenderFrame's read-back schedule (runtime.hip: the first batch
after Run(2) without a read-back, the last rounds guarded on the device).
Whatever the schedule, a frame is Reset, Run(2), then Run(1) rounds until the
completed paths reach the target or max_rounds rounds ran
(application.cpp:100-115 with an spp target): the same rounds, FrameIndex,
state and accumulator as that loop issued one round at a time."""
from __future__ import annotations

import numpy as np
import pytest

from test_gpu_parity import compare_state, scene_for

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev(pt):
    if pt.device_count() < 1:
        pytest.skip("no HIP device")
    d = pt.Device(0)
    yield d
    d.close()


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def manual(pt, dev, ds, W, H, target, max_rounds, fused):
    """The frame loop one round at a time, a read-back after each."""
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    r.RenderFlags = 3
    r.set_fused_rounds(fused)
    r.set_round_batch(1)
    r.reset()
    r.run(2)
    rounds = 2
    while True:
        _, samples = r.stats()
        if samples >= target or rounds >= max_rounds:
            break
        r.run(1)
        rounds += 1
    out = rounds, samples, r.FrameIndex, r.read_state(), sb.read()
    r.close()
    sb.close()
    return out


def framed(pt, dev, ds, W, H, target, max_rounds, fused):
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    r.RenderFlags = 3
    r.set_fused_rounds(fused)
    rounds, samples = r.render_frame(target, max_rounds)
    out = rounds, samples, r.FrameIndex, r.read_state(), sb.read()
    r.close()
    sb.close()
    return out


@pytest.mark.parametrize("config,W,H,fused", [(1, 256, 256, 1), (3, 320, 180, 0), (2, 128, 128, 0)])
@pytest.mark.parametrize("spp,max_rounds", [(16, 1 << 30), (16, 9), (16, 5), (16, 20), (16, 22), (3, 1 << 30)])
def test_frame_equals_round_by_round_loop(pt, dev, config, W, H, fused, spp, max_rounds):
    s = scene_for(pt, config)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    target = spp * W * H
    a = framed(pt, dev, ds, W, H, target, max_rounds, fused)
    b = manual(pt, dev, ds, W, H, target, max_rounds, fused)
    assert a[:3] == b[:3], (a[:3], b[:3])
    if max_rounds < (1 << 30):
        assert a[0] == max_rounds
    else:
        assert a[1] >= target
    compare_state(a[3], b[3])
    assert np.array_equal(bits(a[4]), bits(b[4]))
    ds.close()
