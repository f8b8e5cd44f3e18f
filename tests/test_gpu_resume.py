"""GPU: bit-exact resume of a render (SURVEY.md §5 checkpoint/resume row) and
the grey path-record form's switches (kernels.hip StorePathVertex), all
through libpathtracer.so against uninterrupted renders and the CPU oracle.

Resume = the live paths (ptWriteBasicRendererState: next ray + path record,
basic.glsl.inc:159-198), the accumulator (ptWriteSampleBuffer, or each
stream's own) and FrameIndex, restored into a new renderer.  The trace
record is not part of the resumable state: every round traces before it
scatters (basic_trace.glsl, then basic_scatter.glsl), so the next Run
replaces it first.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle_lib
from test_gpu_parity import compare_state, scene_for

pytestmark = pytest.mark.gpu

PATH_FIELDS = ("origin", "packed_velocity", "lambda0", "throughput", "probability", "sample", "active01", "active23")


@pytest.fixture(scope="module")
def dev(pt):
    if pt.device_count() < 1:
        pytest.skip("no HIP device")
    d = pt.Device(0)
    yield d
    d.close()


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def same_path_fields(a, b, mask=None):
    for f in PATH_FIELDS:
        x, y = a[f], b[f]
        if mask is not None:
            x, y = x[mask], y[mask]
        assert np.array_equal(bits(x), bits(y)), f"path field {f} differs"


def renderer(pt, dev, ds, W, H, flags=3, termination=0.0, **kw):
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb, **kw)
    r.RenderFlags = flags
    r.PathTerminationProbability = termination
    return r, sb


@pytest.mark.parametrize("config,W,H,before,after", [
    (3, 1920, 1080, 2, 3),     # the bench workload at full size (grey records)
    (2, 96, 96, 3, 3),         # glass + metal + sky: four-float records, non-empty active stacks
    (5, 128, 64, 2, 2),        # medium + dielectrics
])
def test_resume_equals_uninterrupted_and_oracle(pt, dev, config, W, H, before, after):
    """Reset + Run(2) + `before` x Run(1); save state, accumulator and
    FrameIndex; destroy the renderer; restore into a new one and run `after`
    more rounds: equal to the uninterrupted render and to the oracle, slot
    state and every accumulated pixel bit for bit."""
    s = scene_for(pt, config)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    a, sba = renderer(pt, dev, ds, W, H)
    a.reset()
    a.run(2)
    for _ in range(before):
        a.run(1)
    saved, acc, frame = a.read_state(), sba.read(), a.FrameIndex
    a.close()
    sba.close()
    if config == 2:
        act = saved["active01"] != 0xFFFFFFFF
        assert act.any(), "some saved path is inside a glass shape"
    b, sbb = renderer(pt, dev, ds, W, H)
    sbb.write(acc)
    b.FrameIndex = frame
    b.write_state(saved)
    restored = b.read_state()
    same_path_fields(restored, saved)
    assert np.all(restored["hit"]["shape_material"] == 0xFFFFFFFF)   # no trace of the restored rays yet
    for _ in range(after):
        b.run(1)
    c, sbc = renderer(pt, dev, ds, W, H)
    c.reset()
    c.run(2)
    for _ in range(before + after):
        c.run(1)
    dev.synchronize()
    gb, gc = b.read_state(), c.read_state()
    compare_state(gb, gc)
    assert np.array_equal(bits(sbb.read()), bits(sbc.read()))
    assert b.FrameIndex == c.FrameIndex
    o = oracle_lib.OracleRenderer(s.packs(), W, H)
    o.RenderFlags = 3
    o.reset()
    o.run(2)
    for _ in range(before + after):
        o.run(1)
    compare_state(gb, o.state())
    oa = o.accum()
    assert np.array_equal(bits(sbb.read()), bits(oa)) and oa[..., 3].sum() > 0
    o.close()
    for x in (b, sbb, c, sbc, ds):
        x.close()


def test_resume_band_streams(pt, dev):
    """A band partition with two path streams: every stream's state and own
    accumulator saved and restored; after more rounds the merged frame equals
    the uninterrupted renderer's bit for bit."""
    s = scene_for(pt, 1)
    W, H, K = 64, 80, 2
    ds = pt.DeviceScene(dev)
    ds.update(s)
    a, sba = renderer(pt, dev, ds, W, H, rank=1, nranks=2, streams=K)
    a.reset()
    a.run(2)
    a.run(1)
    saved = [(a.read_state(k), a.read_accumulator(k)) for k in range(K)]
    frame = a.FrameIndex
    a.close()
    sba.close()
    b, sbb = renderer(pt, dev, ds, W, H, rank=1, nranks=2, streams=K)
    b.FrameIndex = frame
    for k, (st, acc) in enumerate(saved):
        b.write_state(st, k)
        b.write_accumulator(acc, k)
    c, sbc = renderer(pt, dev, ds, W, H, rank=1, nranks=2, streams=K)
    c.reset()
    c.run(2)
    c.run(1)
    for x in (b, c):
        x.run(1)
        x.run(1)
        x.merge_streams()
    dev.synchronize()
    owned = pt.owned_pixels(W, H, 1, 2)
    for k in range(K):
        compare_state(b.read_state(k)[owned], c.read_state(k)[owned])
        assert np.array_equal(bits(b.read_accumulator(k)), bits(c.read_accumulator(k)))
    got, want = sbb.read(), sbc.read()
    assert np.array_equal(bits(got[owned]), bits(want[owned])) and want[owned][:, 3].sum() > 0
    for x in (b, sbb, c, sbc, ds):
        x.close()


def test_state_write_rejects_invalid_paths(pt, dev):
    """Nothing is written when a path is not one a renderer can hold between
    rounds: a non-zero Sample, lambda0 outside [0, 1], an active shape index
    beyond the scene."""
    s = scene_for(pt, 2)
    W, H = 48, 32
    ds = pt.DeviceScene(dev)
    ds.update(s)
    r, sb = renderer(pt, dev, ds, W, H)
    r.reset()
    r.run(2)
    good = r.read_state()
    shapes = len(s.arrays()["shapes"])
    bad_cases = []
    x = good.copy(); x["sample"][3, 5, 1] = 0.5; bad_cases.append((x, "sample"))
    x = good.copy(); x["lambda0"][0, 0] = 1.5; bad_cases.append((x, "lambda0"))
    x = good.copy(); x["active01"][2, 2] = 0xFFFF0000 | shapes; bad_cases.append((x, "active shape"))
    for st, what in bad_cases:
        with pytest.raises(pt.PathTracerError, match=what):
            r.write_state(st)
    same_path_fields(r.read_state(), good)      # untouched
    r.write_state(good)
    r.run(1)
    o = oracle_lib.OracleRenderer(s.packs(), W, H)
    o.RenderFlags = 3
    o.reset()
    o.run(2)
    o.run(1)
    dev.synchronize()
    compare_state(r.read_state(), o.state())
    o.close()
    for x in (r, sb, ds):
        x.close()


def test_record_form_switches_with_openpbr(pt, dev, tmp_path):
    """The grey record form follows the shade mask between rounds: a diffuse
    scene with imported OpenPBR shapes runs grey while OpenPBR shading is off
    (their hits end the path), leaves it when shading is switched on mid-render
    (OpenPBR's spectral weights and media), and returns to it when switched
    off again if every live path allows it.  Every step bit-exact against the
    oracle switching at the same rounds."""
    import test_ingestion as ti
    path = ti.write_model(tmp_path)
    s = pt.Scene.config(1)
    e = s.instantiate_prefab(s.load_model_as_prefab(path, openpbr_as_diffuse=False))
    s.set_transform(e, position=(0.1, 0.1, 0.3), rotation=(0.3, 0.2, 0.1), scale=(0.4, 0.4, 0.4))
    s.pack()
    W, H = 64, 48
    ds = pt.DeviceScene(dev)
    ds.update(s)
    r, sb = renderer(pt, dev, ds, W, H)
    o = oracle_lib.OracleRenderer(s.packs(), W, H)
    o.RenderFlags = 3
    for x in (r, o):
        x.reset()
        x.run(2)
    assert r.shade_info()["grey_records"]
    seen = []
    for enable in (True, False, True, False):
        r.set_openpbr(enable)
        o.set_openpbr(enable)
        for x in (r, o):
            x.run(1)
            x.run(1)
        dev.synchronize()
        info = r.shade_info()
        seen.append(info["grey_records"])
        assert info["grey_records"] is False or not enable
        compare_state(r.read_state(), o.state())
        assert np.array_equal(bits(sb.read()), bits(o.accum()))
    assert seen[0] is False and seen[2] is False
    o.close()
    for x in (r, sb, ds):
        x.close()
    s.close()


@pytest.mark.parametrize("seed", [0, 5, 10, 15, 19, 23])
def test_resume_random_scenes(pt, dev, seed):
    """Resume on the fuzz scenes (tests/fuzz_scenes.py: nested and scattering
    glass, OpenPBR hits, textured skies, every camera, random flags and
    roulette), the resumed renderer running its rounds as a round batch for
    odd seeds: state and image equal the uninterrupted render and the oracle."""
    import fuzz_scenes
    s, st = fuzz_scenes.build(pt, seed)
    W, H = 48, 32
    ds = pt.DeviceScene(dev)
    ds.update(s)
    kw = dict(flags=st["flags"], termination=st["termination"])
    a, sba = renderer(pt, dev, ds, W, H, **kw)
    a.reset()
    a.run(2)
    a.run(1)
    saved, acc, frame = a.read_state(), sba.read(), a.FrameIndex
    a.close()
    sba.close()
    b, sbb = renderer(pt, dev, ds, W, H, **kw)
    sbb.write(acc)
    b.FrameIndex = frame
    b.write_state(saved)
    if seed % 2:
        b.set_round_batch(2)
        b.run_rounds(3)
    else:
        for _ in range(3):
            b.run(1)
    o = oracle_lib.OracleRenderer(s.packs(), W, H)
    o.RenderFlags = st["flags"]
    o.PathTerminationProbability = st["termination"]
    o.reset()
    o.run(2)
    for _ in range(4):
        o.run(1)
    dev.synchronize()
    compare_state(b.read_state(), o.state())
    assert np.array_equal(bits(sbb.read()), bits(o.accum()))
    o.close()
    for x in (b, sbb, ds):
        x.close()
    s.close()


def test_resume_fused_small_frame(pt, dev):
    """C1 at 256x256 (every tile resident at once: the fused round kernel and
    automatic 16-round batches), saved after Run(2) + 5 rounds and resumed for
    20 consecutive Run(1) rounds (batched), against the oracle."""
    s = scene_for(pt, 1)
    W, H = 256, 256
    ds = pt.DeviceScene(dev)
    ds.update(s)
    a, sba = renderer(pt, dev, ds, W, H)
    a.reset()
    a.run(2)
    a.run_rounds(5)
    saved, acc, frame = a.read_state(), sba.read(), a.FrameIndex
    info = a.shade_info()
    a.close()
    sba.close()
    assert info["grey_records"]
    b, sbb = renderer(pt, dev, ds, W, H)
    sbb.write(acc)
    b.FrameIndex = frame
    b.write_state(saved)
    assert not b.shade_info()["grey_records"]       # written records are four-float ones ...
    b.run_rounds(20)
    assert b.shade_info()["grey_records"]           # ... and grey again after the next run
    o = oracle_lib.OracleRenderer(s.packs(), W, H)
    o.RenderFlags = 3
    o.reset()
    o.run(2)
    for _ in range(25):
        o.run(1)
    dev.synchronize()
    compare_state(b.read_state(), o.state())
    assert np.array_equal(bits(sbb.read()), bits(o.accum()))
    o.close()
    for x in (b, sbb, ds):
        x.close()
