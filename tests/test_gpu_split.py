"""GPU: tile groups on concurrent streams (ptSetBasicRendererSplit).

Consecutive rounds (ptRunBasicRendererRounds, ptRenderFrame) split the tiles
into K groups, each running the batch's rounds on its own HIP stream.  A
slot's round depends only on its own previous round and the round's
FrameIndex (basic_trace.glsl / basic_scatter.glsl run per slot), so every K
must give the unsplit rounds' state and accumulator bit for bit -- checked
here against K = 1 and against the CPU oracle (Run(1) per round,
application.cpp:100-115)."""
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


def render(pt, dev, ds, W, H, groups, batches, flags=3, termination=0.0, fused=0):
    """Reset, Run(2), then run_rounds(b) for each b of batches with the given
    split (a list: one K per batch, so K can change between batches)."""
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    r.RenderFlags = flags
    r.PathTerminationProbability = termination
    r.set_fused_rounds(fused)
    r.reset()
    r.run(2)
    for k, b in zip(groups, batches):
        r.set_split(k)
        r.run_rounds(b)
    dev.synchronize()
    out = r.read_state(), sb.read(), r.stats()
    r.close()
    sb.close()
    return out


def same(a, b):
    sa, aa, ta = a
    sb_, ab, tb = b
    compare_state(sa, sb_)
    assert np.array_equal(bits(aa), bits(ab)), "accumulator differs"
    assert ta == tb, f"stats differ: {ta} vs {tb}"


@pytest.mark.parametrize("config,W,H,batches", [
    (3, 160, 90, [9, 7]),      # grey records, node cache; tile-order re-sorts inside the batches
    (2, 96, 96, [6, 5]),       # sky sampling, metal, glass, completion queue
    (5, 128, 64, [5, 4]),      # fog, dielectrics, spilled traversal stack
])
def test_split_equals_unsplit_and_oracle(pt, dev, config, W, H, batches):
    s = scene_for(pt, config)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    ref = render(pt, dev, ds, W, H, [1] * len(batches), batches)
    for K in (2, 3, 4):
        same(render(pt, dev, ds, W, H, [K] * len(batches), batches), ref)
    # K changing between batches (the order array is regrouped).
    same(render(pt, dev, ds, W, H, [2, 3], batches), ref)
    o = oracle_lib.OracleRenderer(s.packs(), W, H)
    o.RenderFlags = 3
    o.PathTerminationProbability = 0.0
    o.reset()
    o.run(2)
    for _ in range(sum(batches)):
        o.run(1)
    compare_state(ref[0], o.state())
    assert np.array_equal(bits(ref[1]), bits(o.accum()))
    ds.close()


@pytest.mark.parametrize("config,W,H,spp", [(2, 1024, 1024, 4), (5, 2048, 1024, 2), (3, 1920, 1080, 2)])
def test_automatic_split_full_frames(pt, dev, config, W, H, spp):
    """The configs' full frames take three groups automatically; a
    ptRenderFrame with them equals the unsplit frame bit for bit."""
    s = scene_for(pt, config)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    info = s.info
    out = []
    for k in (0, 1):
        sb = pt.SampleBuffer(dev, W, H)
        r = pt.BasicRenderer(dev, ds, sb)
        r.RenderFlags = info.render_flags
        r.PathTerminationProbability = info.termination_probability
        r.set_split(k)
        sp = r.split()
        if k == 0:
            assert sp["groups"] == 3 and sp["tiles"] >= 2048, sp
            assert sp["timed_tiles"] == (sp["tiles"] + 2) // 3
        else:
            assert sp["groups"] == 1
        rounds, samples = r.render_frame(spp * W * H)
        out.append((rounds, samples, r.read_state(), sb.read()))
        r.close()
        sb.close()
    (ra, sa, sta, aa), (rb, sb_, stb, ab) = out
    assert (ra, sa) == (rb, sb_)
    compare_state(sta, stb)
    assert np.array_equal(bits(aa), bits(ab))
    ds.close()


def test_split_off_for_fused_and_small(pt, dev):
    """Automatic mode leaves renderers whose rounds run fused (every tile fits
    on the GPU at once) or whose frames are small unsplit; a forced K is
    capped at the tile count; bad values are rejected."""
    s = scene_for(pt, 1)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    sb = pt.SampleBuffer(dev, 256, 256)
    r = pt.BasicRenderer(dev, ds, sb)
    assert r.split()["groups"] == 1
    r.set_fused_rounds(0)
    assert r.split()["groups"] == 1          # 256 tiles < 2048
    r.set_split(4)
    assert r.split()["groups"] == 4
    with pytest.raises(pt.PathTracerError):
        r.set_split(pt.MAX_SPLIT + 1)
    r.close()
    sb.close()
    sb = pt.SampleBuffer(dev, 16, 16)         # one tile
    r = pt.BasicRenderer(dev, ds, sb)
    r.set_split(3)
    assert r.split()["groups"] == 1
    r.close()
    sb.close()
    ds.close()


def test_split_profiling_times_group_zero(pt, dev):
    """Kernel profiling times group 0's launches: one extend and one shade
    launch per round of a split batch."""
    s = scene_for(pt, 3)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    sb = pt.SampleBuffer(dev, 320, 180)
    r = pt.BasicRenderer(dev, ds, sb)
    r.set_fused_rounds(0)
    r.set_split(2)
    r.reset()
    r.run(2)
    dev.set_profiling(True, period=1)
    dev.reset_kernel_stats()
    r.run_rounds(8)
    dev.synchronize()
    n_ext, _ = dev.kernel_stats(1)   # PT_KERNEL_EXTEND
    n_sh, _ = dev.kernel_stats(2)    # PT_KERNEL_SHADE
    dev.set_profiling(False)
    assert n_ext == 8 and n_sh == 8, (n_ext, n_sh)
    r.close()
    sb.close()
    ds.close()


def test_split_band_partition_with_path_streams(pt, dev):
    """A band partition (rank 1 of 3) carrying two path streams per pixel:
    every stream's state and own accumulator equal under three tile groups
    and unsplit."""
    s = scene_for(pt, 3)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    W, H = 320, 180
    out = []
    for k in (1, 3):
        sb = pt.SampleBuffer(dev, W, H)
        r = pt.BasicRenderer(dev, ds, sb, rank=1, nranks=3, streams=2)
        r.RenderFlags = 3
        r.set_fused_rounds(0)
        r.set_split(k)
        r.reset()
        r.run(2)
        r.run_rounds(9)
        r.merge_streams()
        dev.synchronize()
        out.append(([r.read_state(j) for j in range(2)], [r.read_accumulator(j) for j in range(2)], sb.read()))
        r.close()
        sb.close()
    (sa, aa, ma), (sb2, ab, mb) = out
    for j in range(2):
        compare_state(sa[j], sb2[j])
        assert np.array_equal(bits(aa[j]), bits(ab[j])), f"stream {j} accumulator differs"
    assert np.array_equal(bits(ma), bits(mb))
    ds.close()


def test_split_after_resume(pt, dev):
    """Resume into a new renderer (state, accumulator, FrameIndex), then
    rounds in three tile groups: equal to the uninterrupted unsplit render."""
    s = scene_for(pt, 2)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    W, H = 128, 128
    ref = render(pt, dev, ds, W, H, [1, 1], [4, 6])
    sb = pt.SampleBuffer(dev, W, H)
    a = pt.BasicRenderer(dev, ds, sb)
    a.RenderFlags = 3
    a.set_fused_rounds(0)
    a.reset()
    a.run(2)
    a.run_rounds(4)
    saved, acc, frame = a.read_state(), sb.read(), a.FrameIndex
    a.close()
    sb.close()
    sb = pt.SampleBuffer(dev, W, H)
    b = pt.BasicRenderer(dev, ds, sb)
    b.RenderFlags = 3
    b.set_fused_rounds(0)
    b.set_split(3)
    sb.write(acc)
    b.FrameIndex = frame
    b.write_state(saved)
    b.run_rounds(6)
    dev.synchronize()
    compare_state(b.read_state(), ref[0])
    assert np.array_equal(bits(sb.read()), bits(ref[1]))
    b.close()
    sb.close()
    ds.close()


@pytest.mark.parametrize("config,W,H", [(2, 96, 96), (5, 128, 64)])
def test_class_lists_in_groups(pt, dev, config, W, H):
    """Class-pure shade (per-class lists) inside tile groups, on scenes with
    several material types: on and off give the same bits, both equal to the
    unsplit rounds; the query reports when the lists are used."""
    s = scene_for(pt, config)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    ref = render(pt, dev, ds, W, H, [1, 1], [6, 5])
    out = {}
    for mode in (0, 1):
        sb = pt.SampleBuffer(dev, W, H)
        r = pt.BasicRenderer(dev, ds, sb)
        r.RenderFlags = 3
        r.set_fused_rounds(0)
        r.set_class_lists(mode)
        r.set_split(3)
        assert r.class_lists() == (mode == 0)
        r.set_split(1)
        assert not r.class_lists()
        r.set_split(3)
        r.reset()
        r.run(2)
        r.run_rounds(6)
        r.run_rounds(5)
        dev.synchronize()
        out[mode] = (r.read_state(), sb.read(), r.stats())
        r.close()
        sb.close()
    for mode in (0, 1):
        same(out[mode], ref)
    with pytest.raises(pt.PathTracerError):
        sb = pt.SampleBuffer(dev, W, H)
        r = pt.BasicRenderer(dev, ds, sb)
        try:
            r.set_class_lists(2)
        finally:
            r.close()
            sb.close()
    ds.close()


def test_class_lists_not_for_single_material(pt, dev):
    """The C3 room (one material type) never takes the lists."""
    s = scene_for(pt, 3)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    sb = pt.SampleBuffer(dev, 1920, 1080)
    r = pt.BasicRenderer(dev, ds, sb)
    assert r.split()["groups"] == 3 and not r.class_lists()
    r.close()
    sb.close()
    ds.close()


@pytest.mark.parametrize("config,W,H", [(2, 160, 128), (5, 192, 96)])
def test_class_lists_uneven_groups_and_single_rounds(pt, dev, config, W, H):
    """Class lists with tile groups that do not divide the tiles evenly (80
    and 72 tiles in three groups: the list buffers grow from the
    single-stream size to three group regions) and single-stream list rounds
    between split batches: the same bits as the unsplit tile-local rounds."""
    s = scene_for(pt, config)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    ref = render(pt, dev, ds, W, H, [1, 1], [6, 5])
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    r.RenderFlags = 3
    r.set_fused_rounds(0)
    r.set_split(3)
    assert r.class_lists()
    r.reset()
    r.run(2)          # single-stream rounds through the lists
    r.run_rounds(6)
    r.run(1)
    r.run_rounds(4)
    dev.synchronize()
    same((r.read_state(), sb.read(), r.stats()), ref)
    r.close()
    sb.close()
    ds.close()
