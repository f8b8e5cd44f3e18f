"""GPU: the step-capped extend with compaction across launches
(ptSetBasicRendererExtendCap; DESIGN §4 "Compaction across launches").

A capped extend stops each wave after S wave steps; the lanes still
traversing save their traversal state (level ray, closest hit so far, node
words, level, stack depths and entries) to a packed queue, and a
continuation launch resumes them.  Trace() is a deterministic state machine
(scene.glsl.inc:468-611), so the resumed traversal must end at the same hit
bit for bit: checked here against the uncapped extend and the oracle, for
caps from 2 steps (nearly every ray queued, deep stacks saved) up to the
automatic 32, on every scene type, in single-stream rounds, tile groups,
guarded frame ends and after a resume.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle_lib
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


def render(pt, dev, ds, W, H, cap, split, batches, flags=3, termination=0.0):
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    r.RenderFlags = flags
    r.PathTerminationProbability = termination
    r.set_fused_rounds(0)
    r.set_split(split)
    r.set_extend_cap(cap)
    used = r.extend_cap()
    r.reset()
    r.run(2)
    for b in batches:
        r.run_rounds(b)
    dev.synchronize()
    out = (r.read_state(), sb.read(), r.stats(), used)
    r.close()
    sb.close()
    return out


def same(a, b):
    compare_state(a[0], b[0])
    assert np.array_equal(bits(a[1]), bits(b[1])), "accumulator differs"
    assert a[2] == b[2], f"stats differ: {a[2]} vs {b[2]}"


@pytest.mark.parametrize("config,W,H", [(3, 160, 90), (2, 96, 96), (1, 64, 64)])
def test_capped_extend_equals_uncapped_and_oracle(pt, dev, config, W, H):
    s = scene_for(pt, config)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    batches = [5, 4]
    ref = render(pt, dev, ds, W, H, 1, 1, batches)
    assert ref[3] == 0                      # mode 1: uncapped
    for cap in (2, 3, 7, 32):
        for split in (1, 3):
            out = render(pt, dev, ds, W, H, cap, split, batches)
            assert out[3] == cap
            same(out, ref)
    o = oracle_lib.OracleRenderer(s.packs(), W, H)
    o.RenderFlags = 3
    o.reset()
    o.run(2)
    for _ in range(sum(batches)):
        o.run(1)
    compare_state(ref[0], o.state())
    assert np.array_equal(bits(ref[1]), bits(o.accum()))
    o.close()
    ds.close()


def test_smallest_cap_queues_nearly_every_ray(pt, dev):
    """S = 2 is the smallest settable cap (1 is "off"); on the C3 room nearly
    every ray outlives two steps, so the continuation traces almost the whole
    launch from saved state, TLAS and BLAS entries and all."""
    s = scene_for(pt, 3)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    ref = render(pt, dev, ds, 320, 180, 1, 1, [3, 3])
    same(render(pt, dev, ds, 320, 180, 2, 3, [3, 3]), ref)
    ds.close()


def test_capped_extend_with_roulette(pt, dev):
    """Paths ended by roulette (termination 0.25) under a small cap: the C2
    box (glass: medium events) and the C3 room."""
    for config, W, H in ((2, 96, 96), (3, 96, 64)):
        s = scene_for(pt, config)
        ds = pt.DeviceScene(dev)
        ds.update(s)
        ref = render(pt, dev, ds, W, H, 1, 1, [4, 3], termination=0.25)
        same(render(pt, dev, ds, W, H, 4, 3, [4, 3], termination=0.25), ref)
        ds.close()


def test_spilled_stack_runs_uncapped(pt, dev):
    """Scenes whose traversal stack needs spill rows keep the one-launch
    extend in automatic mode (the queue holds the LDS stack only) and still
    render bit-exactly."""
    s = scene_for(pt, 5)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    W, H = 128, 64
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    spill = ds.stack_needed > 20           # PT_EXTEND_CAP LDS entries (kernels.hip)
    assert (r.extend_cap() == 0) == spill
    assert r.extend_cap() in (0, 32)
    r.close()
    sb.close()
    ds.close()


@pytest.mark.parametrize("config,spp", [(3, 4), (2, 3)])
def test_capped_frames_end_at_the_same_round(pt, dev, config, spp):
    """ptRenderFrame (split batches, guarded last rounds: the continuation
    zeroes the next round's counter even in a round the guard stops) with
    and without the cap: same rounds, samples, state and pixels."""
    s = scene_for(pt, config)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    W, H = (640, 360) if config == 3 else (512, 512)
    out = []
    for cap in (1, 0, 5):
        sb = pt.SampleBuffer(dev, W, H)
        r = pt.BasicRenderer(dev, ds, sb)
        r.RenderFlags = 3
        r.set_fused_rounds(0)
        r.set_split(3)
        r.set_extend_cap(cap)
        res = r.render_frame(spp * W * H)
        # A second frame on the same renderer: the counters' parity
        # carried over from the guarded end.
        r.FrameIndex = 0
        res2 = r.render_frame(spp * W * H)
        out.append((res, res2, r.read_state(), sb.read()))
        r.close()
        sb.close()
    ds.close()
    for o in out[1:]:
        assert o[0] == out[0][0] and o[1] == out[0][1]
        compare_state(o[2], out[0][2])
        assert np.array_equal(bits(o[3]), bits(out[0][3]))
    assert out[0][0] == out[0][1]


def test_cap_changes_between_batches_and_resume(pt, dev):
    """The cap and the group count changing between batches, then a resume
    into a new capped renderer: equal to the uncapped uninterrupted render."""
    s = scene_for(pt, 3)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    W, H = 160, 96
    ref = render(pt, dev, ds, W, H, 1, 1, [3, 4, 5])
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    r.RenderFlags = 3
    r.set_fused_rounds(0)
    r.reset()
    r.run(2)
    r.set_extend_cap(3)
    r.set_split(2)
    r.run_rounds(3)
    r.set_extend_cap(9)
    r.set_split(1)
    r.run_rounds(4)
    saved, acc, frame = r.read_state(), sb.read(), r.FrameIndex
    r.close()
    sb.close()
    sb = pt.SampleBuffer(dev, W, H)
    b = pt.BasicRenderer(dev, ds, sb)
    b.RenderFlags = 3
    b.set_fused_rounds(0)
    b.set_split(3)
    b.set_extend_cap(6)
    sb.write(acc)
    b.FrameIndex = frame
    b.write_state(saved)
    b.run_rounds(5)
    dev.synchronize()
    compare_state(b.read_state(), ref[0])
    assert np.array_equal(bits(sb.read()), bits(ref[1]))
    b.close()
    sb.close()
    ds.close()
