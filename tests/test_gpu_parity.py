"""GPU parity: the HIP wavefront kernels against the CPU oracle.

Bars (BASELINE.json north_star): hit records bit-exact (shape/material index,
time, packed normal/tangent, UV); per-pixel slot state bit-exact after the
reference's Reset / Run(2) / Run(1) schedule; accumulated image relative L2
<= 1e-4 after several rounds.  All calls go through libpathtracer.so.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle_lib
from rays import random_rays  # noqa: F401  (re-exported for test_gpu_fuzz)

pytestmark = pytest.mark.gpu

REL_L2_TOL = 1e-4   # north_star: per-pixel radiance within 1e-4 relative L2

# (config, width, height) — reduced resolutions keep the oracle fast; the
# renderer code path is resolution independent.
CASES = [(1, 64, 64), (2, 96, 96), (3, 160, 90), (5, 128, 64)]


@pytest.fixture(scope="module")
def dev(pt):
    if pt.device_count() < 1:
        pytest.skip("no HIP device")
    d = pt.Device(0)
    yield d
    d.close()


_scenes = {}


def scene_for(pt, config):
    if config not in _scenes:
        _scenes[config] = pt.Scene.config(config)
    return _scenes[config]


def compare_hits(g, o):
    assert np.array_equal(g["shape_material"], o["shape_material"]), "shape/material index mismatch"
    hit = o["shape_material"] != 0xFFFFFFFF
    for f in ("time", "packed_normal", "packed_tangent", "u", "v"):
        gv = g[f][hit].view(np.uint32)
        ov = o[f][hit].view(np.uint32)
        bad = np.flatnonzero(gv != ov)
        assert bad.size == 0, f"{f}: {bad.size} of {hit.sum()} hits differ"


@pytest.mark.parametrize("config", [1, 2, 3, 5])
def test_trace_rays_bit_exact(pt, dev, config):
    s = scene_for(pt, config)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    o, v, d = random_rays(s.arrays(), 20000, seed=config)
    g = ds.trace_rays(o, v, d)
    ref = oracle_lib.trace_rays(s.packs(), o, v, d)
    compare_hits(g, ref)
    ds.close()


@pytest.mark.parametrize("fmt", [0, 1, 2], ids=["stack16", "stack32-packed", "stack32-node-index"])
def test_stack_formats_bit_exact(pt, dev, fmt):
    """Every traversal-stack entry format (chosen per scene at upload: 16-bit
    packed words, 32-bit packed words, node indices; ptSetSceneStackFormat
    forces the wider ones) gives the same hits."""
    for config in (3, 5):
        s = scene_for(pt, config)
        ds = pt.DeviceScene(dev)
        ds.set_stack_format(fmt)
        ds.update(s)
        o, v, d = random_rays(s.arrays(), 20000, seed=10 + config)
        compare_hits(ds.trace_rays(o, v, d), oracle_lib.trace_rays(s.packs(), o, v, d))
        ds.close()
    gs, os_, ga, oa = render_pair(pt, dev, 5, 128, 64, [2, 1], stack_format=fmt)
    compare_state(gs, os_)
    assert np.array_equal(ga.view(np.uint32), oa.view(np.uint32))


def test_deep_stack_spills_bit_exact(pt, dev, tmp_path):
    """A scene whose traversal stack outgrows the 20 LDS entries: 24 spheres,
    each twice the size and distance of the last, build a chain-shaped TLAS
    (depth 25); rays fired along the chain push every far child, so entries
    20+ go through the global spill rows.  Hits stay bit-exact."""
    from test_ingestion import write_model
    s = pt.Scene.create()
    for i in range(24):
        s.create_entity(pt.ENTITY_SPHERE, position=(3.0 * 2.0 ** i, 0.0, 1.0), scale=(0.5 * 2.0 ** i,) * 3)
    s.instantiate_prefab(s.load_model_as_prefab(write_model(tmp_path)))
    s.pack()
    ds = pt.DeviceScene(dev)
    ds.update(s)
    assert ds.stack_needed > 20
    rng = np.random.default_rng(5)
    n = 4096
    o = np.zeros((n, 3), np.float32)
    o[:, 0] = rng.uniform(-40.0, -2.0, n)
    o[:, 1:] = rng.normal(0.0, 0.3, (n, 2)) + [0.0, 1.0]
    d = np.zeros((n, 3))
    d[:, 0] = 1.0
    d[:, 1:] = rng.normal(0.0, 0.02, (n, 2))
    d[n // 2:] = rng.normal(size=(n - n // 2, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    vel = oracle_lib.pack_unit_vectors(d.astype(np.float32))
    dur = np.full(n, 1048576.0, np.float32)
    compare_hits(ds.trace_rays(o, vel, dur), oracle_lib.trace_rays(s.packs(), o, vel, dur))
    ds.close()
    s.close()


def render_pair(pt, dev, config, W, H, schedule, camera=0, flags=3, termination=0.0, rank=0, nranks=1,
                scene=None, fused=None, stack_format=0, hit_record=0):
    """The same Reset + Run(schedule...) on the HIP renderer and the oracle:
    (GPU state, oracle state, GPU accumulator, oracle accumulator).
    fused: the renderer's fused-rounds mode (None: its default);
    stack_format / hit_record: the device scene's encodings (PT_STACK_FORMAT_*,
    PT_HIT_RECORD_*; 0 = automatic)."""
    s = scene if scene is not None else scene_for(pt, config)
    ds = pt.DeviceScene(dev)
    ds.set_stack_format(stack_format)
    ds.set_hit_record_form(hit_record)
    ds.update(s)
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb, rank=rank, nranks=nranks)
    o = oracle_lib.OracleRenderer(s.packs(), W, H, rank=rank, nranks=nranks)
    if fused is not None:
        r.set_fused_rounds(fused)
    for x in (r, o):
        x.RenderFlags = flags
        x.PathTerminationProbability = termination
        x.CameraIndex = camera
        x.reset()
        for rounds in schedule:
            x.run(rounds)
    dev.synchronize()
    out = (r.read_state(), o.state(), sb.read(), o.accum())
    for x in (r, sb, ds):
        x.close()
    return out


STATE_FIELDS_F = ["origin", "lambda0", "throughput", "probability", "sample"]
STATE_FIELDS_U = ["packed_velocity", "active01", "active23"]


def compare_state(g, o):
    for f in STATE_FIELDS_U:
        assert np.array_equal(g[f], o[f]), f"state field {f} differs at {np.argwhere(g[f] != o[f])[:4].tolist()}"
    for f in STATE_FIELDS_F:
        gv, ov = g[f].view(np.uint32), o[f].view(np.uint32)
        bad = np.argwhere(gv != ov)
        assert bad.size == 0, f"state field {f} differs at {bad[:4].tolist()}"
    compare_hits(g["hit"].reshape(-1), o["hit"].reshape(-1))


@pytest.mark.parametrize("config,W,H", CASES)
def test_slot_state_bit_exact(pt, dev, config, W, H):
    """Reset, Run(2), Run(1): the application's schedule (application.cpp:109-114)."""
    gs, os_, ga, oa = render_pair(pt, dev, config, W, H, [2, 1])
    compare_state(gs, os_)
    assert np.array_equal(ga.view(np.uint32), oa.view(np.uint32))


@pytest.mark.parametrize("config,W,H", CASES)
def test_image_rel_l2(pt, dev, config, W, H):
    gs, os_, ga, oa = render_pair(pt, dev, config, W, H, [2] + [1] * 14)
    rel = np.linalg.norm(ga - oa) / max(np.linalg.norm(oa), 1e-30)
    assert oa[..., 3].sum() > 0
    assert rel <= REL_L2_TOL, f"relative L2 {rel:.3e}"


@pytest.mark.parametrize("config,W,H,schedule,camera", [
    (1, 256, 256, [2] + [1] * 14, 0),    # C1 at its full 256x256, 16 spp
    (2, 1024, 1024, [2, 1], 0),          # C2 at its full 1024x1024
    (3, 1920, 1080, [2] + [1] * 6, 0),   # C3 (the bench workload) at its full 1920x1080, 8 rounds
    (5, 2048, 1024, [2, 1], 0),          # C5 at its declared 2048x1024, thin-lens camera
    (5, 2048, 1024, [2, 1], 1),          # C5 360 camera
])
def test_full_size_bit_exact(pt, dev, config, W, H, schedule, camera):
    """The configs' declared resolutions (configs.cpp): every
    slot's state and every accumulated pixel bit-exact, over the tile /
    TileOrder / ShadeOrder layout of a full frame (8100 tiles at 1080p, ragged
    last tile row).  C4's 3840x2160 frame is covered per rank in
    test_gpu_coverage.py."""
    gs, os_, ga, oa = render_pair(pt, dev, config, W, H, schedule, camera=camera)
    compare_state(gs, os_)
    assert oa[..., 3].sum() > 0
    assert np.array_equal(ga.view(np.uint32), oa.view(np.uint32))


@pytest.mark.parametrize("W,H", [(16, 40), (17, 9), (300, 33)])
def test_narrow_and_ragged_frames(pt, dev, W, H):
    """One tile column (the tile-row reciprocal's special case), ragged tile
    edges in both directions."""
    gs, os_, ga, oa = render_pair(pt, dev, 1, W, H, [2, 1])
    compare_state(gs, os_)
    assert np.array_equal(ga.view(np.uint32), oa.view(np.uint32))


def test_c5_360_camera(pt, dev):
    gs, os_, ga, oa = render_pair(pt, dev, 5, 96, 48, [2, 1, 1], camera=1)
    compare_state(gs, os_)
    rel = np.linalg.norm(ga - oa) / max(np.linalg.norm(oa), 1e-30)
    assert rel <= REL_L2_TOL


def test_partitioned_union_equals_full(pt, dev):
    """Band-partitioned renderers (one per rank) sum to the 1-GPU image exactly."""
    s = scene_for(pt, 1)
    W, H, N = 64, 80, 3
    ds = pt.DeviceScene(dev)
    ds.update(s)
    full_sb = pt.SampleBuffer(dev, W, H)
    full = pt.BasicRenderer(dev, ds, full_sb)
    parts = []
    for rank in range(N):
        sb = pt.SampleBuffer(dev, W, H)
        parts.append((pt.BasicRenderer(dev, ds, sb, rank=rank, nranks=N), sb))
    for r in [full] + [p[0] for p in parts]:
        r.RenderFlags = 3
        r.reset()
        r.run(2)
        r.run(1)
    total = sum(sb.read() for _, sb in parts)
    assert np.array_equal(total.view(np.uint32), full_sb.read().view(np.uint32))
    for r, sb in parts:
        r.close(); sb.close()
    full.close(); full_sb.close(); ds.close()


def test_profiling_counts_kernels(pt, dev):
    s = scene_for(pt, 1)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    sb = pt.SampleBuffer(dev, 64, 64)
    r = pt.BasicRenderer(dev, ds, sb)
    dev.set_profiling(True)
    dev.reset_kernel_stats()
    r.RenderFlags = 3
    r.reset()
    r.set_fused_rounds(0)
    r.run(3)
    n_ext, ms_ext = dev.kernel_stats(1)
    n_sh, ms_sh = dev.kernel_stats(2)
    # one extend + one shade per round
    assert n_ext == n_sh == 3 and ms_ext > 0 and ms_sh > 0
    assert dev.kernel_rounds(1) == 3 and dev.kernel_rounds(2) == 3
    # a 64x64 frame fits the GPU at once: the automatic mode fuses a round
    # into one launch (kernel 5), and the rounds of one Run(R) into one
    # round batch (kernel 6, seed step 0)
    dev.reset_kernel_stats()
    r.set_fused_rounds(1)
    r.run(1)
    n_rd, ms_rd = dev.kernel_stats(5)
    assert dev.kernel_stats(1)[0] == 0 and dev.kernel_stats(2)[0] == 0
    assert n_rd == 1 and dev.kernel_rounds(5) == 1 and ms_rd > 0
    dev.reset_kernel_stats()
    r.run(2)
    n_rb, ms_rb = dev.kernel_stats(6)
    assert dev.kernel_stats(5)[0] == 0 and dev.kernel_stats(1)[0] == 0
    assert n_rb == 1 and dev.kernel_rounds(6) == 2 and ms_rb > 0
    # consecutive Run(1) rounds of such a frame run as 16-round batches
    # (kernel 6, PT_KERNEL_ROUNDS): a timed batch counts its rounds, and the
    # profiling period counts rounds (period 8: every batch holds a sampled
    # round), so time per round = total / rounds.
    dev.set_profiling(True, period=8)
    dev.reset_kernel_stats()
    r.run_rounds(40)
    n_b, ms_b = dev.kernel_stats(6)
    assert n_b == 3 and dev.kernel_rounds(6) == 40 and ms_b > 0
    dev.set_profiling(True, period=32)
    dev.reset_kernel_stats()
    r.run_rounds(64)    # batches of rounds 0-15, 16-31, 32-47, 48-63: rounds 0 and 32 sampled
    assert dev.kernel_stats(6)[0] == 2 and dev.kernel_rounds(6) == 32
    dev.set_profiling(False)
    r.close(); sb.close(); ds.close()


def test_bad_camera_index_rejected(pt, dev):
    s = scene_for(pt, 1)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    sb = pt.SampleBuffer(dev, 32, 32)
    r = pt.BasicRenderer(dev, ds, sb)
    r.CameraIndex = 7
    with pytest.raises(pt.PathTracerError):
        r.reset()
    r.close(); sb.close(); ds.close()


def test_fast_division_matches_ieee(pt, dev):
    """The FMA-corrected division helper (XDiv) is bit-identical to a / b."""
    for seed in (1, 2, 3, 4):
        assert dev.check_fast_division(1 << 28, seed) == 0


def test_fast_reciprocal_matches_ieee_exhaustively(pt, dev):
    """FastRcp (v_rcp_f32 + one FMA Newton step) equals 1.0f / d bit for bit
    on all 2^32 inputs in its range 2^-126 <= |d| < 2^126."""
    assert dev.check_fast_reciprocal() == 0


def test_extend_stats_does_not_perturb(pt, dev):
    """ptExtendStats traces the current rays (as the next Run's extend would),
    so a render that calls it between rounds matches one that does not."""
    s = scene_for(pt, 3)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    out = []
    for with_stats in (False, True):
        sb = pt.SampleBuffer(dev, 96, 64)
        r = pt.BasicRenderer(dev, ds, sb)
        r.RenderFlags = 3
        r.reset()
        r.run(2)
        if with_stats:
            st = r.extend_stats()
            assert st["rays"] == 96 * 64 and st["waves"] == 96 * 64 // 64
            assert 0 < st["simd_efficiency"] <= 1.0
            assert st["internal_nodes"] > 0 and st["faces"] >= st["blas_leaves"] > 0
        r.run(1)
        out.append((r.read_state(), sb.read()))
        r.close(); sb.close()
    assert np.array_equal(out[0][0].view(np.uint8), out[1][0].view(np.uint8))
    assert np.array_equal(out[0][1].view(np.uint32), out[1][1].view(np.uint32))
    ds.close()


def test_diffuse_metal_scene_bit_exact(pt, dev):
    """A scene with only diffuse + metal materials runs the diffuse|metal shade
    instantiation; it must match the oracle like the full one."""
    s = pt.Scene.create()
    m1 = s.create_material(pt.MATERIAL_BASIC_METAL, "Rough", BaseColor=(0.9, 0.6, 0.3), Roughness=0.3)
    m2 = s.create_material(pt.MATERIAL_BASIC_METAL, "Mirror", BaseColor=(0.8, 0.8, 0.9), Roughness=0.0)
    # CreateScene's camera sits at (0,0,1) looking down at the plane
    s.create_entity(pt.ENTITY_SPHERE, position=(0.5, 0.2, 0.35), scale=(0.3, 0.3, 0.3), material=m1)
    s.create_entity(pt.ENTITY_CUBE, position=(-0.6, -0.3, 0.2), scale=(0.2, 0.2, 0.2), material=m2)
    s.set_root(skybox_sampling_probability=0.3)
    s.pack()
    ds = pt.DeviceScene(dev)
    ds.update(s)
    W, H = 64, 48
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    o = oracle_lib.OracleRenderer(s.packs(), W, H)
    for x in (r, o):
        x.RenderFlags = 3
        x.reset()
        x.run(2)
        x.run(1)
        x.run(1)
    dev.synchronize()
    compare_state(r.read_state(), o.state())
    assert np.array_equal(sb.read().view(np.uint32), o.accum().view(np.uint32))
    for x in (r, sb, ds):
        x.close()
    s.close()


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_resolve_bit_exact(pt, dev, mode):
    """RenderSampleBuffer on the device vs the oracle: OutColor and sRGB8."""
    rng = np.random.default_rng(mode)
    W, H = 96, 40
    acc = rng.uniform(0, 4, size=(H, W, 4)).astype(np.float32)
    acc[..., 3] = rng.integers(0, 50, size=(H, W)).astype(np.float32)
    acc[0, :8] = 0
    acc[1, :8, :3] *= -1
    acc[2, :8, :3] *= 1e6
    sb = pt.SampleBuffer(dev, W, H)
    sb.write(acc)
    assert np.array_equal(sb.read(), acc)
    sb.render(pt.ResolveParameters(Brightness=1.7, ToneMappingMode=mode, ToneMappingWhiteLevel=3.0))
    out, out8 = sb.read_resolved(), sb.read_srgb8()
    ref, ref8 = oracle_lib.resolve(acc, 1.7, mode, 3.0)
    same = (out.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(out) & np.isnan(ref))
    assert same.all(), np.argwhere(~same)[:5]
    assert np.array_equal(out8, ref8)
    sb.close()


@pytest.mark.parametrize("config", [1, 3, 5])
@pytest.mark.parametrize("mode", range(7))
def test_preview_bit_exact(pt, dev, config, mode):
    """RenderPreview on the device vs the oracle: image, AOVs, pick query."""
    s = scene_for(pt, config)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    cam = s.arrays()["cameras"][0]["Transform"]["To"]
    p = pt.PreviewParameters(cam, RenderMode=mode, RenderSizeX=72, RenderSizeY=40, Brightness=1.5,
                             SelectedShapeIndex=1, MouseX=30, MouseY=21)
    ctx = pt.PreviewRenderContext(dev, ds)
    ctx.render(p)
    img, aov, q = ctx.image(), ctx.aovs(), ctx.query()
    ref_img, ref_aov, ref_q = oracle_lib.preview(s.packs(), p)
    same = (img.view(np.uint32) == ref_img.view(np.uint32)) | (np.isnan(img) & np.isnan(ref_img))
    assert same.all(), np.argwhere(~same)[:5]
    assert np.array_equal(aov.view(np.uint8), ref_aov.view(np.uint8))
    assert q == ref_q
    ctx.close()
    ds.close()


def test_imported_model_bit_exact(pt, dev, tmp_path):
    """OBJ + MTL + PNG texture through LoadModelAsPrefab (BasicDiffuse
    conversion) renders identically on the GPU and in the oracle."""
    import test_ingestion as ti
    path = ti.write_model(tmp_path)
    s = pt.Scene.create()
    e = s.instantiate_prefab(s.load_model_as_prefab(path, openpbr_as_diffuse=True))
    s.set_transform(e, position=(0.2, 0.1, 0.4), rotation=(0.3, 0.2, 0.1), scale=(0.3, 0.3, 0.3))
    s.pack()
    ds = pt.DeviceScene(dev)
    ds.update(s)
    W, H = 64, 48
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    o = oracle_lib.OracleRenderer(s.packs(), W, H)
    for x in (r, o):
        x.RenderFlags = 3
        x.reset()
        x.run(2)
        x.run(1)
    dev.synchronize()
    compare_state(r.read_state(), o.state())
    assert np.array_equal(sb.read().view(np.uint32), o.accum().view(np.uint32))
    for x in (r, sb, ds):
        x.close()
    s.close()
