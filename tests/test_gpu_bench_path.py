"""GPU: the exact schedule bench.py times, against the CPU oracle at the
configs' full sizes (VERDICT r05, next-round task 1).

The headline runs ptRenderFrame on the C3 frame at 1920x1080.  Its rounds
run in three tile groups on concurrent HIP streams (RunRoundsSplit).  On C2
and C5 the groups shade through per-class lists (shade_classq_kernel).
Nothing here forces a mode: every renderer keeps the product defaults, and
each test asserts that the defaults take the path under test.  Each is then
compared bit for bit with the oracle running the reference's schedule:
Reset, Run(2), then one Run(1) per round (application.cpp:100-115,
basic.cpp:306-332).  The comparison covers every state field of every slot,
every accumulated pixel, and the ray and path counters.

The frame tests also check the frame-end round.  One round before the
frame's last, the oracle has not reached the target; after the last round it
has (the first round whose total reaches the target, application.cpp:100-115
as SURVEY §8(d) reads it).
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle_lib
from test_gpu_parity import compare_state, scene_for

pytestmark = pytest.mark.gpu

FULL = {2: (1024, 1024), 3: (1920, 1080), 4: (3840, 2160), 5: (2048, 1024)}


@pytest.fixture(scope="module")
def dev(pt):
    if pt.device_count() < 1:
        pytest.skip("no HIP device")
    d = pt.Device(0)
    yield d
    d.close()


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def product_renderer(pt, dev, ds, config, W, H):
    """A renderer with the bench's settings (bench.py: flags and termination
    from the config; every scheduling mode automatic), asserting the modes
    the automatic choice takes at the full size."""
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    info = scene_for(pt, config).info
    r.RenderFlags = info.render_flags
    r.PathTerminationProbability = info.termination_probability
    sp = r.split()
    assert sp["groups"] == 3, sp
    assert r.class_lists() == (config in (2, 5))
    return r, sb


def oracle_for(pt, config, W, H):
    s = scene_for(pt, config)
    o = oracle_lib.OracleRenderer(s.packs(), W, H)
    o.RenderFlags = s.info.render_flags
    o.PathTerminationProbability = s.info.termination_probability
    return o


@pytest.mark.parametrize("config", [3, 2, 5, 4])
def test_split_rounds_full_size_vs_oracle(pt, dev, config):
    """Reset, Run(2), then run_rounds(7) and run_rounds(5): two split batches
    (fork and join on the group streams, a tile-order re-sort inside them,
    class-list parities across the batch boundary) against 2 + 12 oracle
    rounds.  C4 is the 4K room on one GPU (8.3 M slots, 32 400 tiles)."""
    W, H = FULL[config]
    s = scene_for(pt, config)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    r, sb = product_renderer(pt, dev, ds, config, W, H)
    r.reset()
    r.run(2)
    r.run_rounds(7)
    r.run_rounds(5)
    dev.synchronize()
    gs, ga, gstats = r.read_state(), sb.read(), r.stats()
    for x in (r, sb, ds):
        x.close()
    o = oracle_for(pt, config, W, H)
    o.reset()
    o.run(2)
    for _ in range(12):
        o.run(1)
    compare_state(gs, o.state())
    oa = o.accum()
    assert oa[..., 3].sum() > 0
    assert np.array_equal(bits(ga), bits(oa)), "accumulator differs"
    assert gstats == o.counters(), (gstats, o.counters())
    o.close()


@pytest.mark.parametrize("config,spp", [(3, 6), (2, 4)])
def test_render_frame_split_path_ends_at_the_reference_round(pt, dev, config, spp):
    """ptRenderFrame with the automatic tile groups (and class lists on C2):
    a frame of spp samples per pixel at the full size.  Its batches run
    split, its last rounds guarded.  The frame ends at the first round whose
    completed-path total reaches the target, and its pixels equal the
    oracle's after the same rounds."""
    W, H = FULL[config]
    target = spp * W * H
    s = scene_for(pt, config)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    r, sb = product_renderer(pt, dev, ds, config, W, H)
    rounds, samples = r.render_frame(target)
    ga = sb.read()
    for x in (r, sb, ds):
        x.close()
    assert samples >= target and rounds > 4
    o = oracle_for(pt, config, W, H)
    o.reset()
    o.run(2)
    for _ in range(rounds - 3):
        o.run(1)
    _, before_last = o.counters()
    assert before_last < target, f"the oracle reached the target one round before the frame's end ({rounds})"
    o.run(1)
    _, osamples = o.counters()
    assert osamples == samples
    assert np.array_equal(bits(ga), bits(o.accum())), "accumulator differs"
    o.close()
