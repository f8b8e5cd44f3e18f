"""GPU parity of the renderer parameters and the callers' flows that
test_gpu_parity.py does not exercise (all through libpathtracer.so, checked
against the CPU oracle bit for bit):

* C4 (3840x2160, BASELINE configs[3]) as the 1/8 pixel-band partitions the
  8-GPU run gives ranks 0 and 7 (basic.glsl.inc:9-10: the reference itself
  cannot hold this frame);
* every RenderFlags combination (basic_scatter.glsl:15-18 no-jitter sample
  position, :354-357 overwrite instead of accumulate) and Russian roulette
  with PathTerminationProbability > 0 (:295-298);
* OBJ materials left as OpenPBR, whose hits end the path with no
  contribution (scene.glsl.inc:685-693);
* the editor's camera move: PackSceneData re-packs only the cameras,
  UpdateVulkanScene uploads only them, then Reset + Run(2) + Run(1)
  (application.cpp:52-66,88-115);
* ptGetStats and the RCCL frame-end reduce (idempotent over progressive
  frames);
* fused rounds (one extend+shade launch per round, round_kernel) against
  the separate launches and the oracle, including a full C3 frame forced
  through the fused kernel;
* two processes rendering their bands with the product renderer and summing
  over gloo (the CPU stand-in for the RCCL reduce; RCCL refuses two ranks on
  one device), equal to the single-process frame.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

import oracle_lib
from test_gpu_parity import compare_hits, compare_state, random_rays, render_pair

pytestmark = pytest.mark.gpu

HERE = Path(__file__).resolve().parent


@pytest.fixture(scope="module")
def dev(pt):
    if pt.device_count() < 1:
        pytest.skip("no HIP device")
    d = pt.Device(0)
    yield d
    d.close()


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


@pytest.mark.parametrize("rank", [0, 7])
def test_c4_rank_of_8_partition_bit_exact(pt, dev, rank):
    """One rank's share of the C4 frame: 3840x2160 = 135 bands of 16 rows over
    8 ranks (ranks 0-6 own 17 bands = 1,044,480 slots, rank 7 owns 16)."""
    s = pt.Scene.config(4)
    W, H = s.info.width, s.info.height
    assert (W, H) == (3840, 2160)
    gs, os_, ga, oa = render_pair(pt, dev, 4, W, H, [2, 1], rank=rank, nranks=8, scene=s)
    owned = pt.owned_pixels(W, H, rank, 8)
    assert owned.sum() == 3840 * 16 * (17 if rank == 0 else 16)
    compare_state(gs, os_)
    assert np.array_equal(bits(ga), bits(oa))
    assert oa[owned][:, 3].sum() > 0 and not oa[~owned].any()
    s.close()


@pytest.mark.parametrize("config,rank,streams", [(4, 0, 2), (4, 7, 2), (3, 5, 8)])
def test_band_path_streams_bit_exact(pt, dev, config, rank, streams):
    """Path streams: a rank-of-8 band partition carrying
    `streams` paths per owned pixel.  Every stream's slot state equals the
    oracle's one-stream render of the same bands started at FrameIndex
    k << 24, and after ptMergeBasicRendererStreams the sample buffer holds the
    streams' accumulators summed in stream order, bit for bit; a merge after
    more rounds gives the new totals the same way.  C4
    at full size (ranks 0 and 7, two streams: 2.09 M slots per launch), C3
    rank 5 of 8 with eight streams (2.2 M slots)."""
    s = pt.Scene.config(config)
    W, H = s.info.width, s.info.height
    ds = pt.DeviceScene(dev)
    ds.update(s)
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb, rank=rank, nranks=8, streams=streams)
    bands = len(range(rank, (H + 15) // 16, 8))
    assert r.slot_count == streams * bands * ((W + 15) // 16) * 256
    r.RenderFlags = 3
    r.reset()
    r.run(2)
    r.run(1)
    r.merge_streams()
    dev.synchronize()
    got1 = sb.read()
    states = [r.read_state(k) for k in range(streams)]
    r.run(1)
    r.merge_streams()
    dev.synchronize()
    got2 = sb.read()
    owned = pt.owned_pixels(W, H, rank, 8)
    want1 = np.zeros((H, W, 4), np.float32)
    want2 = np.zeros((H, W, 4), np.float32)
    for k in range(streams):
        o = oracle_lib.OracleRenderer(s.packs(), W, H, rank=rank, nranks=8)
        o.RenderFlags = 3
        o.FrameIndex = k << 24
        o.reset()
        o.run(2)
        o.run(1)
        compare_state(states[k][owned], o.state()[owned])
        want1 = want1 + o.accum()          # float32, stream order
        o.run(1)
        want2 = want2 + o.accum()
        o.close()
    assert np.array_equal(bits(got1[owned]), bits(want1[owned]))
    assert np.array_equal(bits(got2[owned]), bits(want2[owned]))
    assert got2[owned][:, 3].sum() == want2[owned][:, 3].sum() > 0
    r2, samples = r.stats()
    assert r2 == 4 * streams * int(owned.sum())           # every stream's slot traces a ray per round
    for x in (r, sb, ds):
        x.close()
    s.close()


# (config, W, H, RenderFlags, PathTerminationProbability)
PARAM_CASES = [
    (1, 64, 64, 3, 0.1),     # roulette on, few terminations
    (1, 64, 64, 3, 0.5),     # roulette on, most paths end by roulette
    (1, 64, 64, 0, 0.0),     # no jitter (pixel centres), overwrite
    (1, 64, 64, 1, 0.0),     # no jitter, accumulate
    (1, 64, 64, 2, 0.0),     # jitter, overwrite
    (2, 96, 96, 3, 0.5),     # sky + metal + glass with roulette
    (5, 128, 64, 0, 0.3),    # mixed scene + medium, no jitter, overwrite, roulette
    (5, 128, 64, 1, 0.1),
    (3, 160, 90, 2, 0.2),    # mesh scene
]


@pytest.mark.parametrize("config,W,H,flags,p", PARAM_CASES)
def test_render_flags_and_roulette_bit_exact(pt, dev, config, W, H, flags, p):
    gs, os_, ga, oa = render_pair(pt, dev, config, W, H, [2, 1, 1], flags=flags, termination=p)
    compare_state(gs, os_)
    assert np.array_equal(bits(ga), bits(oa))
    assert oa[..., 3].sum() > 0
    if not flags & pt.RENDER_FLAG_ACCUMULATE:
        # overwrite: a pixel holds its last completed sample only
        assert oa[..., 3].max() == 1.0


def test_openpbr_materials_end_paths(pt, dev, tmp_path):
    """An imported OBJ keeps its OpenPBR materials (the reference's import,
    scene.cpp:671-729): a path that hits them ends with no contribution
    (scene.glsl.inc:685-693)."""
    import test_ingestion as ti
    path = ti.write_model(tmp_path)
    s = pt.Scene.create()
    e = s.instantiate_prefab(s.load_model_as_prefab(path, openpbr_as_diffuse=False))
    s.set_transform(e, position=(0.2, 0.1, 0.4), rotation=(0.3, 0.2, 0.1), scale=(0.3, 0.3, 0.3))
    s.pack()
    mats = s.arrays()["materials"].reshape(-1, 32)[:, 0]
    types = {int(mats[int(sh["MaterialIndex"])]) for sh in s.arrays()["shapes"]}
    assert 3 in types                      # OpenPBR shapes present
    gs, os_, ga, oa = render_pair(pt, dev, None, 64, 48, [2, 1, 1], scene=s)
    compare_state(gs, os_)
    assert np.array_equal(bits(ga), bits(oa))
    assert oa[..., 3].sum() > 0
    s.close()


def test_camera_move_dirty_update_bit_exact(pt, dev):
    """The application's camera move: only the cameras are re-packed and
    uploaded, then Reset + Run(2) + Run(1) on the same renderer; bit-exact
    against a fresh oracle on the updated packs at the same FrameIndex."""
    s = pt.Scene.config(3)
    W, H = 160, 90
    ds = pt.DeviceScene(dev)
    ds.update(s)
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    r.RenderFlags = 3
    r.reset()
    r.run(2)
    r.run(1)
    cam = s.find_camera(0)
    before = s.arrays()["cameras"][0].copy()
    s.move_camera(cam, position=(0.3, -1.2, 1.4), rotation=(1.45, 0.0, 0.35))
    dirty = s.pack()
    assert dirty == pt.SCENE_DIRTY_CAMERAS
    assert not np.array_equal(s.arrays()["cameras"][0]["Transform"]["To"], before["Transform"]["To"])
    ds.update(s, dirty)
    frame = r.FrameIndex
    r.reset()
    r.run(2)
    r.run(1)
    o = oracle_lib.OracleRenderer(s.packs(), W, H)
    o.RenderFlags = 3
    o.FrameIndex = frame
    o.reset()
    o.run(2)
    o.run(1)
    dev.synchronize()
    compare_state(r.read_state(), o.state())
    assert np.array_equal(bits(sb.read()), bits(o.accum()))
    o.close()
    for x in (r, sb, ds):
        x.close()
    s.close()


def test_get_stats_counts_rays_and_samples(pt, dev):
    s = pt.Scene.config(2)
    W, H, N = 96, 80, 2
    ds = pt.DeviceScene(dev)
    ds.update(s)
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb, rank=1, nranks=N)
    r.RenderFlags = 3
    r.reset()
    assert r.stats() == (0, 0)
    r.run(2)
    r.run(3)
    owned = int(pt.owned_pixels(W, H, 1, N).sum())
    rays, samples = r.stats()
    assert rays == 5 * owned
    assert samples == int(sb.read()[..., 3].sum())      # ACCUMULATE: one alpha increment per sample
    assert 0 < samples < rays
    r.reset()
    assert r.stats() == (0, 0)
    for x in (r, sb, ds):
        x.close()
    s.close()


def test_comm_reduce_is_idempotent_over_progressive_frames(pt, dev):
    """ptCommReduceSampleBuffer on a one-rank RCCL communicator: rows outside
    the renderer's bands never enter the sum, even when they hold stale totals
    (the root's buffer after an earlier reduce)."""
    s = pt.Scene.config(1)
    W, H = 64, 80
    ds = pt.DeviceScene(dev)
    ds.update(s)
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb, rank=0, nranks=2)
    o = oracle_lib.OracleRenderer(s.packs(), W, H, rank=0, nranks=2)
    comm = pt.Comm(dev, 1, 0, pt.Comm.unique_id())
    owned = pt.owned_pixels(W, H, 0, 2)
    for x in (r, o):
        x.RenderFlags = 3
        x.reset()
        x.run(2)
    for frame in range(2):
        a = sb.read()
        a[~owned] = 7.0 + frame                      # stale totals in the other rank's bands
        sb.write(a)
        comm.reduce_sample_buffer(sb, 0)
        dev.synchronize()
        assert np.array_equal(bits(sb.read()), bits(o.accum())), f"frame {frame}"
        for x in (r, o):
            x.run(1)
    comm.close()
    o.close()
    for x in (r, sb, ds):
        x.close()
    s.close()


# (config, W, H, schedule): small frames (automatic mode fuses them), a C5
# mixed-material frame with a medium, and the full C3 frame (8160 tiles, more
# than the GPU holds at once: forced with mode 2).
FUSED_CASES = [(3, 160, 96, [2, 1, 3]), (5, 128, 64, [2, 1, 2]), (2, 96, 96, [2, 1, 2]), (3, 1920, 1080, [2, 1])]


@pytest.mark.parametrize("config,W,H,schedule", FUSED_CASES)
def test_fused_rounds_bit_exact(pt, dev, config, W, H, schedule):
    """round_kernel (extend + shade of a tile in one block) gives the same
    state and image as extend_kernel then shade_kernel, and as the oracle."""
    out = {m: render_pair(pt, dev, config, W, H, schedule, fused=m) for m in (0, 2)}
    for m in (0, 2):
        gs, os_, ga, oa = out[m]
        compare_state(gs, os_)
        assert np.array_equal(bits(ga), bits(oa)), f"fused mode {m}"
    assert oa[..., 3].sum() > 0


# (config, W, H, batch, count): count consecutive Run(1) rounds in batches of
# `batch` per launch (a partial last batch when batch does not divide count),
# small frames, C5's mixed materials and medium, and the full C3 frame.
BATCH_CASES = [(3, 160, 96, 4, 7), (5, 128, 64, 3, 5), (2, 96, 96, 16, 9), (1, 64, 64, 2, 2),
               (3, 1920, 1080, 4, 6), (5, 2048, 1024, 8, 8)]


@pytest.mark.parametrize("config,W,H,batch,count", BATCH_CASES)
def test_round_batches_bit_exact(pt, dev, config, W, H, batch, count):
    """ptRunBasicRendererRounds with round batches (rounds_kernel: each tile
    runs several rounds in one launch, seeds FrameIndex+1..+count) equals
    `count` Run(1) calls on the oracle, state and image bit for bit; a Run(1)
    through the per-round kernels follows the batches."""
    from test_gpu_parity import scene_for
    s = scene_for(pt, config)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    r.set_fused_rounds(0)
    r.set_round_batch(batch)
    o = oracle_lib.OracleRenderer(s.packs(), W, H)
    for x in (r, o):
        x.RenderFlags = 3
        x.reset()
        x.run(2)
    r.run_rounds(count)
    for _ in range(count):
        o.run(1)
    dev.synchronize()
    compare_state(r.read_state(), o.state())
    assert np.array_equal(bits(sb.read()), bits(o.accum())), "after the batches"
    r.run(1)
    o.run(1)
    dev.synchronize()
    compare_state(r.read_state(), o.state())
    ga, oa = sb.read(), o.accum()
    assert np.array_equal(bits(ga), bits(oa)), "after a per-round Run(1)"
    assert oa[..., 3].sum() > 0
    for x in (r, sb, ds):
        x.close()


def test_render_frame_round_batches_equal_per_round(pt, dev):
    """ptRenderFrame with round batches (16, and automatic: this frame's 240
    tiles fit on the GPU at once) ends at the same round with the same
    accumulator as with per-round launches (C3 scene, 320x192, 48 spp)."""
    from test_gpu_parity import scene_for
    s = scene_for(pt, 3)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    out = {}
    for batch in (1, 0, 16):
        sb = pt.SampleBuffer(dev, 320, 192)
        r = pt.BasicRenderer(dev, ds, sb)
        r.set_round_batch(batch)
        r.RenderFlags = 3
        rounds, samples = r.render_frame(48 * 320 * 192)
        out[batch] = (rounds, samples, sb.read())
        for x in (r, sb):
            x.close()
    ds.close()
    for batch in (0, 16):
        assert out[1][:2] == out[batch][:2]
        assert np.array_equal(bits(out[1][2]), bits(out[batch][2])), f"batch {batch}"


def test_fused_rounds_mode_argument(pt, dev):
    s = pt.Scene.config(1)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    sb = pt.SampleBuffer(dev, 32, 32)
    r = pt.BasicRenderer(dev, ds, sb)
    with pytest.raises(pt.PathTracerError):
        r.set_fused_rounds(3)
    r.set_fused_rounds(1)
    for x in (r, sb, ds):
        x.close()
    s.close()


def free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def test_two_process_band_render_equals_single_process(pt, dev, tmp_path):
    """Two ranks (processes) on this GPU, each rendering its bands of a C5
    frame with the product renderer over two progressive frames, summed to
    rank 0 over gloo; equal bit for bit to this process's 1-rank frames."""
    cfg, W, H = 5, 128, 80
    out = tmp_path / "reduced.npz"
    env = dict(os.environ, OMP_NUM_THREADS="2", HSA_ENABLE_IPC_MODE_LEGACY="0", PT_DIST_RENDERER="gpu")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}",
           str(HERE / "dist_worker.py"), str(out), str(cfg), str(W), str(H)]
    res = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr[-3000:]
    got = np.load(out)
    s = pt.Scene.config(cfg)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    r.RenderFlags = 3
    r.reset()
    r.run(2)
    r.run(1)
    frame0 = sb.read()
    r.run(1)
    frame1 = sb.read()
    assert int(got["owned"][0]) == W * H
    assert np.array_equal(bits(got["accum"]), bits(frame0))
    assert np.array_equal(bits(got["accum2"]), bits(frame1))
    for x in (r, sb, ds):
        x.close()
    s.close()


def test_comm_gather_single_rank_and_partition_check(pt, dev):
    """ptCommGatherSampleBuffer: a one-rank communicator has nothing to move
    (the buffer is unchanged); a buffer partitioned for another rank count
    is rejected before any RCCL call."""
    s = pt.Scene.config(1)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    sb = pt.SampleBuffer(dev, 48, 40)
    r = pt.BasicRenderer(dev, ds, sb)
    r.RenderFlags = 3
    r.reset()
    r.run(2)
    comm = pt.Comm(dev, 1, 0, pt.Comm.unique_id())
    before = sb.read()
    comm.gather_sample_buffer(sb, 0)
    assert np.array_equal(bits(sb.read()), bits(before))
    r2 = pt.BasicRenderer(dev, ds, sb, rank=1, nranks=2)   # the buffer is now partitioned 1 of 2
    with pytest.raises(pt.PathTracerError):
        comm.gather_sample_buffer(sb, 0)
    comm.close()
    for x in (r2, r, sb, ds):
        x.close()
    s.close()


def test_comm_error_contract_single_rank(pt, dev):
    """The exchange's failure contract on a one-rank communicator (INTEGRATION
    §3): a failed argument check (bad root, mismatched partition, missing total
    buffer) fails the call before any collective and leaves the communicator
    usable; ptCommSetTimeout rejects a non-positive deadline; with the
    communicator live, waits go through the polling path and still complete."""
    s = pt.Scene.config(1)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    sb = pt.SampleBuffer(dev, 48, 40)
    total = pt.SampleBuffer(dev, 48, 40)
    r = pt.BasicRenderer(dev, ds, sb)
    r.RenderFlags = 3
    comm = pt.Comm(dev, 1, 0, pt.Comm.unique_id())
    comm.set_timeout(120.0)
    with pytest.raises(pt.PathTracerError):
        comm.set_timeout(0.0)
    r.reset()
    r.run(2)
    dev.synchronize()                                       # polling wait (live communicator)
    with pytest.raises(pt.PathTracerError, match="bad root"):
        comm.reduce_sample_buffer_into(sb, total, 1)
    with pytest.raises(pt.PathTracerError, match="total buffer"):
        comm.reduce_sample_buffer_into(sb, None, 0)
    with pytest.raises(pt.PathTracerError, match="bad root"):
        comm.gather_sample_buffer(sb, 3)
    comm.reduce_sample_buffer_into(sb, total, 0)            # still usable
    dev.synchronize()
    assert np.array_equal(bits(total.read()), bits(sb.read()))
    rounds, samples = r.render_frame(4 * 48 * 40, 1000)     # ptRenderFrame's waits poll too
    assert samples >= 4 * 48 * 40
    comm.close()
    for x in (r, total, sb, ds):
        x.close()
    s.close()


def test_sample_shard_offset_and_reduce_into(pt, dev):
    """Sample sharding (bench.py's default multi-GPU split): a renderer whose
    RNG stream starts at FrameIndex 1 << 24 (rank 1's) is bit-exact against the
    oracle from the same offset; ptCommReduceSampleBufferInto on a one-rank
    communicator copies the accumulator into the total, leaving it intact,
    and is repeatable after more rounds."""
    s = pt.Scene.config(5)
    W, H = 128, 64
    ds = pt.DeviceScene(dev)
    ds.update(s)
    sb = pt.SampleBuffer(dev, W, H)
    total = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    o = oracle_lib.OracleRenderer(s.packs(), W, H)
    comm = pt.Comm(dev, 1, 0, pt.Comm.unique_id())
    for x in (r, o):
        x.RenderFlags = 3
        x.FrameIndex = 1 << 24
        x.reset()
        x.run(2)
        x.run(1)
    for frame in range(2):
        comm.reduce_sample_buffer_into(sb, total, 0)
        dev.synchronize()
        compare_state(r.read_state(), o.state())
        assert np.array_equal(bits(sb.read()), bits(o.accum()))
        assert np.array_equal(bits(total.read()), bits(o.accum()))
        for x in (r, o):
            x.run(1)
    assert r.FrameIndex == (1 << 24) + 4          # Run(2), Run(1) and two more Run(1)
    with pytest.raises(pt.PathTracerError):
        comm.reduce_sample_buffer_into(sb, None, 0)     # the root needs a total buffer
    comm.close()
    o.close()
    for x in (r, total, sb, ds):
        x.close()
    s.close()


def test_two_process_sample_shards_equal_summed_renders(pt, dev, tmp_path):
    """Two processes on this GPU, each rendering the whole C5 frame from its
    own FrameIndex offset with the product renderer, summed over gloo (the
    CPU stand-in for the RCCL reduce): equal to this process's two offset
    renders added."""
    cfg, W, H = 5, 96, 64
    out = tmp_path / "reduced.npz"
    env = dict(os.environ, OMP_NUM_THREADS="2", HSA_ENABLE_IPC_MODE_LEGACY="0", PT_DIST_RENDERER="gpu",
               PT_DIST_SHARD="samples")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}",
           str(HERE / "dist_worker.py"), str(out), str(cfg), str(W), str(H)]
    res = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr[-3000:]
    got = np.load(out)
    s = pt.Scene.config(cfg)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    want = [np.zeros((H, W, 4), np.float32), np.zeros((H, W, 4), np.float32)]
    for rank in range(2):
        sb = pt.SampleBuffer(dev, W, H)
        r = pt.BasicRenderer(dev, ds, sb)
        r.RenderFlags = 3
        r.FrameIndex = rank << 24
        r.reset()
        r.run(2)
        r.run(1)
        want[0] = want[0] + sb.read()
        r.run(1)
        want[1] = want[1] + sb.read()
        r.close()
        sb.close()
    assert np.array_equal(bits(got["accum"]), bits(want[0]))
    assert np.array_equal(bits(got["accum2"]), bits(want[1]))
    ds.close()
    s.close()


@pytest.mark.parametrize("form", [1, 0], ids=["face-index", "vertex-indices"])
def test_hit_record_forms_bit_exact(pt, dev, form):
    """Both compact hit-record forms (packed vertex indices, the default for
    scenes whose vertex indices fit 21 bits, and the face-index form that
    larger scenes use; ptSetSceneHitRecordForm forces it) give the oracle's
    state and image, meshes and analytic shapes alike (C5 mixes both)."""
    for cfg, W, H in ((3, 160, 96), (5, 128, 64)):
        s = pt.Scene.config(cfg)
        gs, os_, ga, oa = render_pair(pt, dev, cfg, W, H, [2, 1, 1], scene=s, hit_record=form)
        compare_state(gs, os_)
        assert np.array_equal(bits(ga), bits(oa))
        s.close()


def edge_scene(pt, kind):
    """Scenes at the traversal's edges: no shapes at all (every ray misses;
    the reference would read an uninitialised node buffer here, so the
    oracle's all-miss reading is the contract), one analytic shape (the TLAS
    root is a shape leaf), one single-triangle mesh (the BLAS root is a leaf)."""
    s = pt.Scene.empty()
    s.create_entity(pt.ENTITY_CAMERA, position=(0.0, -2.0, 1.0), rotation=(1.2, 0.0, 0.0))
    if kind == "sphere":
        s.create_entity(pt.ENTITY_SPHERE, position=(0.0, 0.0, 1.0), scale=(0.5,) * 3)
    elif kind == "triangle":
        m = s.create_mesh([[-1, 0, 0], [1, 0, 0], [0, 0, 2]], [[0, 1, 2]])
        e = s.create_entity(pt.ENTITY_MESH_INSTANCE)
        s.set_mesh(e, m)
    s.set_root(skybox_sampling_probability=0.5, skybox_brightness=2.0)
    s.pack()
    return s


@pytest.mark.parametrize("kind", ["empty", "sphere", "triangle"])
@pytest.mark.parametrize("W,H", [(1, 1), (37, 21)])
def test_edge_scenes_bit_exact(pt, dev, kind, W, H):
    s = edge_scene(pt, kind)
    gs, os_, ga, oa = render_pair(pt, dev, None, W, H, [2, 1, 1], scene=s)
    compare_state(gs, os_)
    assert np.array_equal(ga.view(np.uint32), oa.view(np.uint32))
    assert oa[..., 3].sum() > 0
    ds = pt.DeviceScene(dev)
    ds.update(s)
    o, v, d = random_rays(s.arrays(), 4096, seed=71)
    compare_hits(ds.trace_rays(o, v, d), oracle_lib.trace_rays(s.packs(), o, v, d))
    ds.close()
    s.close()


def test_large_mesh_bit_exact(pt, dev):
    """A mesh past the compact forms' limits: 740k unconnected triangles =
    2.22 M vertices (> 2^21, so hit records carry the face index instead of
    packed vertex indices) and ~1.5 M BLAS nodes (child-pair indices beyond
    16 bits, so the traversal stack holds packed 32-bit entries, not u16),
    under a TLAS with analytic shapes; state, image and random-ray hits
    bit-exact against the oracle."""
    import fuzz_scenes
    rng = np.random.default_rng(17)
    pos, idx, nrm, uv = fuzz_scenes.soup_mesh(rng, 740000, 2.5)
    assert len(pos) > (1 << 21)
    s = pt.Scene.empty()
    m = s.create_mesh(pos, idx, nrm, uv, name="BigSoup")
    e = s.create_entity(pt.ENTITY_MESH_INSTANCE, position=(0.0, 0.0, 1.5))
    s.set_mesh(e, m)
    s.create_entity(pt.ENTITY_PLANE, position=(0.0, 0.0, -1.0))
    s.create_entity(pt.ENTITY_SPHERE, position=(2.0, -3.0, 0.5), scale=(0.7, 0.7, 0.7))
    s.create_entity(pt.ENTITY_CAMERA, position=(0.0, -8.0, 1.5), rotation=(1.57, 0.0, 0.0))
    s.set_root(skybox_brightness=1.5)
    s.pack()
    a = s.arrays()
    assert len(a["mesh_nodes"]) > (1 << 16)
    gs, os_, ga, oa = render_pair(pt, dev, None, 80, 48, [2, 1, 1], scene=s)
    compare_state(gs, os_)
    assert np.array_equal(bits(ga), bits(oa))
    ds = pt.DeviceScene(dev)
    ds.update(s)
    o, v, d = random_rays(a, 8192, seed=23)
    compare_hits(ds.trace_rays(o, v, d), oracle_lib.trace_rays(s.packs(), o, v, d))
    ds.close()
    s.close()


def test_editor_updates_bit_exact(pt, dev):
    """The editor's other edits, each followed by PackSceneData's dirty flags,
    a partial ptUpdateScene with them, and Reset + Run(2) + Run(1) on the same
    renderer (application.cpp:100-115, scene.hpp:323-333): a material
    parameter, an entity transform (TLAS rebuild), a new deeper mesh instance
    (meshes + shapes; the traversal stack bound grows), the sky.  Each state
    is bit-exact against a fresh oracle on the updated packs."""
    import fuzz_scenes
    rng = np.random.default_rng(29)
    s = pt.Scene.empty()
    red = s.create_material(pt.MATERIAL_BASIC_DIFFUSE, "Red", BaseColor=(0.8, 0.2, 0.2))
    metal = s.create_material(pt.MATERIAL_BASIC_METAL, "Metal", BaseColor=(0.9, 0.8, 0.5), Roughness=0.2)
    glass = s.create_material(pt.MATERIAL_BASIC_TRANSLUCENT, "Glass", IOR=1.5, Roughness=0.0)
    s.create_entity(pt.ENTITY_PLANE, material=red)
    ball = s.create_entity(pt.ENTITY_SPHERE, position=(0.0, 0.0, 1.0), material=glass)
    s.create_entity(pt.ENTITY_CUBE, position=(1.5, 1.0, 0.5), scale=(0.5, 0.5, 0.5), material=metal)
    blob = s.create_mesh(*fuzz_scenes.blob_mesh(rng, 6, 10, 0.1))
    e = s.create_entity(pt.ENTITY_MESH_INSTANCE, position=(-1.5, 0.5, 0.8), scale=(0.6, 0.6, 0.6), material=metal)
    s.set_mesh(e, blob)
    s.create_entity(pt.ENTITY_CAMERA, position=(0.0, -5.0, 1.5), rotation=(1.4, 0.0, 0.0))
    s.set_root(skybox_brightness=1.0)
    s.pack()
    W, H = 96, 64
    ds = pt.DeviceScene(dev)
    ds.update(s)
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    r.RenderFlags = 3

    def render_and_check():
        frame = r.FrameIndex
        r.reset()
        r.run(2)
        r.run(1)
        o = oracle_lib.OracleRenderer(s.packs(), W, H)
        o.RenderFlags = 3
        o.FrameIndex = frame
        o.reset()
        o.run(2)
        o.run(1)
        dev.synchronize()
        compare_state(r.read_state(), o.state())
        assert np.array_equal(bits(sb.read()), bits(o.accum()))
        o.close()

    render_and_check()
    edits = [
        lambda: s.set_material_parameter(red, "BaseColor", (0.2, 0.7, 0.3)),
        lambda: s.set_transform(ball, position=(0.4, 0.3, 1.2), rotation=(0.0, 0.3, 0.0), scale=(0.8, 1.0, 1.2)),
        lambda: s.set_mesh(s.create_entity(pt.ENTITY_MESH_INSTANCE, position=(0.0, 1.5, 0.6), material=red),
                           s.create_mesh(*fuzz_scenes.soup_mesh(rng, 3000, 0.6))),
        lambda: s.set_root(skybox_brightness=2.5, scatter_rate=0.02),
    ]
    stack0 = ds.stack_needed
    for edit in edits:
        edit()
        dirty = s.pack()
        assert dirty != 0
        ds.update(s, dirty)
        render_and_check()
    assert ds.stack_needed > stack0        # the soup's BVH is deeper than the blob's
    for x in (r, sb, ds):
        x.close()
    s.close()


def test_whole_1024spp_frame_bit_exact(pt, dev):
    """A complete benchmark-mode frame (ptRenderFrame: Reset, Run(2), Run(1)
    until the accumulator holds 1024 samples per pixel) of the
    C3 scene at 480x270 (510 tiles: every tile resident at once, so the
    automatic round batches run it; a ragged bottom band), with and without
    round batches, against the oracle running the same schedule for the same
    number of rounds: every accumulated pixel bit-identical."""
    from test_gpu_parity import scene_for
    s = scene_for(pt, 3)
    W, H = 480, 270
    target = 1024 * W * H
    ds = pt.DeviceScene(dev)
    ds.update(s)
    out = {}
    for batch in (0, 1):
        sb = pt.SampleBuffer(dev, W, H)
        r = pt.BasicRenderer(dev, ds, sb)
        r.set_round_batch(batch)
        r.RenderFlags = 3
        out[batch] = r.render_frame(target) + (sb.read(),)
        for x in (r, sb):
            x.close()
    ds.close()
    rounds, samples, ga = out[0]
    assert out[1][:2] == (rounds, samples)
    assert samples >= target and rounds > 1000
    o = oracle_lib.OracleRenderer(s.packs(), W, H)
    o.RenderFlags = 3
    o.reset()
    o.run(2)
    for _ in range(rounds - 3):
        o.run(1)
    # The frame ends at the reference's round: one round earlier the target
    # was not yet reached (the batches sized from the completion
    # rate must not run past it).
    _, before_last = o.counters()
    assert before_last < target
    o.run(1)
    _, osamples = o.counters()
    oa = o.accum()
    o.close()
    assert osamples == samples
    assert int(oa[..., 3].astype(np.float64).sum()) == samples
    for batch in (0, 1):
        assert np.array_equal(bits(out[batch][2]), bits(oa)), f"round batch mode {batch}"


def test_comm_deadline_aborts_and_device_recovers(pt, dev):
    """The wait's deadline branch with a live RCCL communicator (runtime.hip
    DeviceWait): with a 1 ms deadline, waiting on 150 queued
    full-size C3 rounds (~60 ms) gives up with PT_ERROR_TIMEOUT and aborts the
    communicator (ncclCommAbort); exchanges on it then fail with
    PT_ERROR_COMM_ABORTED; once the stream drains, waits succeed again and the
    renderer's work is intact (its rays/samples counters keep counting)."""
    s = pt.Scene.config(3)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    sb = pt.SampleBuffer(dev, 1920, 1080)
    r = pt.BasicRenderer(dev, ds, sb)
    r.RenderFlags = 3
    r.reset()
    r.run(2)
    dev.synchronize()
    comm = pt.Comm(dev, 1, 0, pt.Comm.unique_id())
    comm.set_timeout(1e-3)
    for _ in range(150):
        r.run(1)
    with pytest.raises(pt.PathTracerError, match=r"status -3"):
        dev.synchronize()
    with pytest.raises(pt.PathTracerError, match=r"status -2"):
        comm.reduce_sample_buffer(sb, 0)
    dev.synchronize()                      # no live communicator: drains, then succeeds
    rays, samples = r.stats()
    assert rays == 152 * 1920 * 1080 and samples > 0
    comm.close()
    r.run(1)
    dev.synchronize()
    for x in (r, sb, ds):
        x.close()
    s.close()
