"""Integrator entry points (mirror of src/integrator/basic.hpp:28-32 and
src/integrator/integrator.hpp:51-60) over libpathtracer.so.

    CreateSampleBuffer(device, W, H)          integrator.hpp:51
    CreateBasicRenderer(device, scene, sb)     basic.hpp:28
    ResetBasicRenderer(device, renderer)       basic.hpp:31
    RunBasicRenderer(device, renderer, rounds) basic.hpp:32

The renderer's CameraIndex / RenderFlags / PathLengthLimit /
PathTerminationProbability / FrameIndex are exposed as attributes, written
by the caller before Reset/Run exactly as application.cpp:104-107 does.
Everything runs in the HIP library; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native as N


class PathTracerError(RuntimeError):
    pass


def _check(rc, what):
    if rc != 0:
        raise PathTracerError(f"{what}: {N.hip_lib().ptGetLastError().decode()} (status {rc})")


def device_count() -> int:
    n = C.c_int(0)
    N.hip_lib().ptGetDeviceCount(C.byref(n))
    return n.value


class Device:
    """A HIP device + stream (replaces the reference's `vulkan` context)."""

    def __init__(self, hip_device: int = 0):
        L = N.hip_lib()
        self._h = L.ptCreateDevice(int(hip_device))
        if not self._h:
            raise PathTracerError(L.ptGetLastError().decode())
        self.index = hip_device

    @property
    def handle(self):
        return self._h

    def synchronize(self):
        _check(N.hip_lib().ptSynchronize(self._h), "ptSynchronize")

    def set_profiling(self, enable: bool, period: int = 1):
        """Kernel timing with HIP events; period > 1 times every period-th round only."""
        _check(N.hip_lib().ptSetProfiling(self._h, int(enable)), "ptSetProfiling")
        _check(N.hip_lib().ptSetProfilingPeriod(self._h, int(period)), "ptSetProfilingPeriod")

    def kernel_stats(self, kernel: int):
        n = C.c_uint64(0)
        ms = C.c_double(0)
        _check(N.hip_lib().ptGetKernelStats(self._h, kernel, C.byref(n), C.byref(ms)), "ptGetKernelStats")
        return int(n.value), float(ms.value)

    def kernel_rounds(self, kernel: int) -> int:
        """Rounds covered by the timed launches of `kernel` (a round batch
        covers several): total_ms / rounds is its time per round."""
        n = C.c_uint64(0)
        _check(N.hip_lib().ptGetKernelRounds(self._h, kernel, C.byref(n)), "ptGetKernelRounds")
        return int(n.value)

    def reset_kernel_stats(self):
        _check(N.hip_lib().ptResetKernelStats(self._h), "ptResetKernelStats")

    def check_fast_division(self, n: int, seed: int = 1) -> int:
        m = C.c_uint64(0)
        _check(N.hip_lib().ptCheckFastDivision(self._h, n, seed, C.byref(m)), "ptCheckFastDivision")
        return int(m.value)

    def check_fast_reciprocal(self) -> int:
        m = C.c_uint64(0)
        _check(N.hip_lib().ptCheckFastReciprocal(self._h, C.byref(m)), "ptCheckFastReciprocal")
        return int(m.value)

    def close(self):
        if self._h:
            N.hip_lib().ptDestroyDevice(self._h)
            self._h = None


class DeviceScene:
    """Device copy of a packed scene (CreateVulkanScene / UpdateVulkanScene)."""

    def __init__(self, device: Device):
        L = N.hip_lib()
        self.device = device
        self._h = L.ptCreateScene(device.handle)
        if not self._h:
            raise PathTracerError(L.ptGetLastError().decode())

    @property
    def handle(self):
        return self._h

    def set_stack_format(self, fmt: int):
        """PT_STACK_FORMAT_* (0 auto, 1 packed 32-bit words, 2 node indices); next update()."""
        _check(N.hip_lib().ptSetSceneStackFormat(self._h, int(fmt)), "ptSetSceneStackFormat")

    def set_hit_record_form(self, form: int):
        """PT_HIT_RECORD_* (0 auto, 1 face index); next update()."""
        _check(N.hip_lib().ptSetSceneHitRecordForm(self._h, int(form)), "ptSetSceneHitRecordForm")

    def update(self, scene, dirty_flags: int = 0xFFFFFFFF):
        packs = scene.packs() if hasattr(scene, "packs") else scene
        _check(N.hip_lib().ptUpdateScene(self.device.handle, self._h, C.byref(packs), dirty_flags), "ptUpdateScene")

    @property
    def stack_needed(self) -> int:
        """Traversal stack entries the uploaded scene can need (TLAS + BLAS depth)."""
        v = C.c_uint32(0)
        _check(N.hip_lib().ptSceneStackNeeded(self._h, C.byref(v)), "ptSceneStackNeeded")
        return int(v.value)

    @property
    def node_cache_pairs(self) -> int:
        """BLAS child pairs the extend kernel keeps in LDS (0: none; ptSceneNodeCache)."""
        v = C.c_uint32(0)
        _check(N.hip_lib().ptSceneNodeCache(self._h, C.byref(v)), "ptSceneNodeCache")
        return int(v.value)

    def trace_rays(self, origins: np.ndarray, packed_velocities: np.ndarray, durations: np.ndarray) -> np.ndarray:
        """Bit-exact Trace() of a ray batch (scene.glsl.inc:522-611)."""
        o = np.ascontiguousarray(origins, dtype=np.float32).reshape(-1, 3)
        v = np.ascontiguousarray(packed_velocities, dtype=np.uint32).reshape(-1)
        d = np.ascontiguousarray(durations, dtype=np.float32).reshape(-1)
        out = np.zeros(len(v), dtype=N.HIT_RECORD_DTYPE)
        _check(N.hip_lib().ptTraceRays(self.device.handle, self._h, len(v), N.fptr(o), N.u32ptr(v), N.fptr(d),
                                       out.ctypes.data), "ptTraceRays")
        return out

    def trace_rays_stats(self, origins: np.ndarray, packed_velocities: np.ndarray, durations: np.ndarray):
        """Traversal counters (ptExtendStats keys) and per-ray step counts of a
        ray batch (diagnostic, ptTraceRaysStats)."""
        o = np.ascontiguousarray(origins, dtype=np.float32).reshape(-1, 3)
        v = np.ascontiguousarray(packed_velocities, dtype=np.uint32).reshape(-1)
        d = np.ascontiguousarray(durations, dtype=np.float32).reshape(-1)
        out = (C.c_uint64 * 14)()
        steps = np.zeros(len(v), dtype=np.uint32)
        _check(N.hip_lib().ptTraceRaysStats(self.device.handle, self._h, len(v), N.fptr(o), N.u32ptr(v), N.fptr(d),
                                            out, steps.ctypes.data), "ptTraceRaysStats")
        keys = ("rays", "lane_steps", "wave_steps_x64", "internal_nodes", "blas_leaves", "faces", "pops",
                "tlas_leaves", "waves")
        stats = dict(zip(keys, (int(x) for x in out)))
        stats["simd_efficiency"] = stats["lane_steps"] / max(stats["wave_steps_x64"], 1)
        return stats, steps

    def close(self):
        if self._h:
            N.hip_lib().ptDestroyScene(self.device.handle, self._h)
            self._h = None


class ResolveParameters:
    """resolve_parameters (integrator.hpp:43-48) with the reference defaults."""

    def __init__(self, Brightness: float = 1.0, ToneMappingMode: int = N.TONE_MAPPING_CLAMP,
                 ToneMappingWhiteLevel: float = 1.0):
        self.Brightness = float(Brightness)
        self.ToneMappingMode = int(ToneMappingMode)
        self.ToneMappingWhiteLevel = float(ToneMappingWhiteLevel)

    def as_struct(self) -> N.pt_resolve_parameters:
        return N.pt_resolve_parameters(self.Brightness, self.ToneMappingMode, self.ToneMappingWhiteLevel)


class SampleBuffer:
    """rgba32f accumulator: CIE XYZ sums + sample count (integrator.cpp:15-87)."""

    def __init__(self, device: Device, width: int, height: int):
        L = N.hip_lib()
        self.device = device
        self.width, self.height = int(width), int(height)
        self._h = L.ptCreateSampleBuffer(device.handle, self.width, self.height)
        if not self._h:
            raise PathTracerError(L.ptGetLastError().decode())

    @property
    def handle(self):
        return self._h

    def read(self) -> np.ndarray:
        out = np.zeros((self.height, self.width, 4), dtype=np.float32)
        _check(N.hip_lib().ptReadSampleBuffer(self.device.handle, self._h, N.fptr(out)), "ptReadSampleBuffer")
        return out

    def write(self, rgba: np.ndarray):
        """Overwrite the accumulator (resume accumulation from a saved one)."""
        a = np.ascontiguousarray(rgba, dtype=np.float32).reshape(self.height, self.width, 4)
        _check(N.hip_lib().ptWriteSampleBuffer(self.device.handle, self._h, N.fptr(a)), "ptWriteSampleBuffer")

    def render(self, params: "ResolveParameters | None" = None, **kw):
        """RenderSampleBuffer (integrator.hpp:55-60): resolve on the device."""
        p = (params or ResolveParameters(**kw)).as_struct()
        _check(N.hip_lib().ptRenderSampleBuffer(self.device.handle, self._h, C.byref(p)), "ptRenderSampleBuffer")

    def read_resolved(self) -> np.ndarray:
        """OutColor of the last render(): (H, W, 4) float32, alpha 1."""
        out = np.zeros((self.height, self.width, 4), dtype=np.float32)
        _check(N.hip_lib().ptReadResolvedImage(self.device.handle, self._h, N.fptr(out)), "ptReadResolvedImage")
        return out

    def read_srgb8(self) -> np.ndarray:
        """The resolved image as B8G8R8A8_SRGB stores it: (H, W, 4) uint8, RGBA order."""
        out = np.zeros((self.height, self.width, 4), dtype=np.uint8)
        _check(N.hip_lib().ptReadResolvedImageSRGB8(self.device.handle, self._h,
                                                    out.ctypes.data_as(C.POINTER(C.c_uint8))),
               "ptReadResolvedImageSRGB8")
        return out

    def close(self):
        if self._h:
            N.hip_lib().ptDestroySampleBuffer(self.device.handle, self._h)
            self._h = None


class BasicRenderer:
    """basic_renderer (basic.hpp:6-26) running the HIP wavefront kernels."""

    _FIELDS = ("FrameIndex", "CameraIndex", "RenderFlags", "PathLengthLimit", "PathTerminationProbability")

    def __init__(self, device: Device, scene: DeviceScene, sample_buffer: SampleBuffer, rank: int = 0, nranks: int = 1,
                 streams: int = 1):
        """rank / nranks: the 16-row pixel bands owned (b % nranks == rank);
        streams: independent paths per owned pixel, stream k seeded at
        FrameIndex + (k << 24) (ptCreateBasicRendererStreams)."""
        L = N.hip_lib()
        self.device, self.scene, self.sample_buffer = device, scene, sample_buffer
        self.rank, self.nranks, self.streams = rank, nranks, streams
        self._h = L.ptCreateBasicRendererStreams(device.handle, scene.handle, sample_buffer.handle, rank, nranks,
                                                 streams)
        if not self._h:
            raise PathTracerError(L.ptGetLastError().decode())
        self._params = L.ptBasicRendererParams(self._h)

    def __getattr__(self, name):
        if name in BasicRenderer._FIELDS:
            return getattr(self._params.contents, name)
        raise AttributeError(name)

    def __setattr__(self, name, value):
        if name in BasicRenderer._FIELDS:
            setattr(self._params.contents, name, value)
        else:
            object.__setattr__(self, name, value)

    @property
    def handle(self):
        return self._h

    @property
    def slot_count(self) -> int:
        return int(N.hip_lib().ptBasicRendererSlotCount(self._h))

    def merge_streams(self):
        """The sample buffer's owned pixels := the sum of every stream's
        accumulator, stream 0 included, in stream order
        ((A0 + A1) + A2 ...; ptMergeBasicRendererStreams).  The streams are
        not cleared and keep accumulating, so a later merge writes the new
        totals (not deltas).  A no-op for one stream."""
        _check(N.hip_lib().ptMergeBasicRendererStreams(self.device.handle, self._h), "ptMergeBasicRendererStreams")

    def set_fused_rounds(self, mode: int):
        """0 never / 1 automatic / 2 whenever possible (ptSetBasicRendererFusedRounds)."""
        _check(N.hip_lib().ptSetBasicRendererFusedRounds(self._h, int(mode)), "ptSetBasicRendererFusedRounds")

    def set_round_batch(self, rounds: int):
        """Rounds per launch for consecutive Run(1) rounds (run_rounds,
        render_frame): 0 automatic (16 when every tile fits on the GPU at
        once), 1 never (one launch per round), R >= 2 always R."""
        _check(N.hip_lib().ptSetBasicRendererRoundBatch(self._h, int(rounds)), "ptSetBasicRendererRoundBatch")

    def set_split(self, groups: int):
        """Tile groups of consecutive rounds, each on its own HIP stream
        (ptSetBasicRendererSplit): 0 automatic, 1 off, 2..MAX_SPLIT that many.
        Results are identical for every value."""
        _check(N.hip_lib().ptSetBasicRendererSplit(self._h, int(groups)), "ptSetBasicRendererSplit")

    def split(self) -> dict:
        """{groups, timed_tiles, tiles}: the tile groups consecutive rounds use
        now, group 0's tiles (the launches kernel profiling times) and all
        tiles (ptGetBasicRendererSplit)."""
        g, t0, t = C.c_uint32(0), C.c_uint32(0), C.c_uint32(0)
        _check(N.hip_lib().ptGetBasicRendererSplit(self._h, C.byref(g), C.byref(t0), C.byref(t)),
               "ptGetBasicRendererSplit")
        return {"groups": int(g.value), "timed_tiles": int(t0.value), "tiles": int(t.value)}

    def set_class_lists(self, mode: int):
        """Class-pure shade inside tile groups (ptSetBasicRendererClassLists):
        0 automatic, 1 off.  Results are identical either way."""
        _check(N.hip_lib().ptSetBasicRendererClassLists(self._h, int(mode)), "ptSetBasicRendererClassLists")

    def class_lists(self) -> bool:
        """Whether consecutive rounds shade through per-class lists now."""
        u = C.c_uint32(0)
        _check(N.hip_lib().ptGetBasicRendererClassLists(self._h, C.byref(u)), "ptGetBasicRendererClassLists")
        return bool(u.value)

    def run_rounds(self, count: int):
        """count consecutive Run(1) calls (one new FrameIndex each), batched
        per set_round_batch (ptRunBasicRendererRounds)."""
        _check(N.hip_lib().ptRunBasicRendererRounds(self.device.handle, self._h, int(count)),
               "ptRunBasicRendererRounds")

    def set_openpbr(self, enable: bool):
        """Shade OpenPBR materials (ptSetBasicRendererOpenPBR); off by default,
        as in the reference, where an OpenPBR hit ends the path."""
        _check(N.hip_lib().ptSetBasicRendererOpenPBR(self._h, int(bool(enable))), "ptSetBasicRendererOpenPBR")

    def reset(self):
        _check(N.hip_lib().ptResetBasicRenderer(self.device.handle, self._h), "ptResetBasicRenderer")

    def run(self, rounds: int = 1):
        _check(N.hip_lib().ptRunBasicRenderer(self.device.handle, self._h, int(rounds)), "ptRunBasicRenderer")

    def render_frame(self, target_samples: int, max_rounds: int = 1 << 30):
        """Benchmark-mode frame (ptRenderFrame): Reset,
        Run(2), then Run(1) rounds until target_samples paths completed since
        the Reset.  Blocks; returns (rounds, samples)."""
        rounds, samples = C.c_uint32(0), C.c_uint64(0)
        _check(N.hip_lib().ptRenderFrame(self.device.handle, self._h, int(target_samples), int(max_rounds),
                                         C.byref(rounds), C.byref(samples)), "ptRenderFrame")
        return int(rounds.value), int(samples.value)

    def stats(self):
        """(rays traced, paths completed) since the last Reset (ptGetStats)."""
        rays, samples = C.c_uint64(0), C.c_uint64(0)
        _check(N.hip_lib().ptGetStats(self.device.handle, self._h, C.byref(rays), C.byref(samples)), "ptGetStats")
        return int(rays.value), int(samples.value)

    def extend_stats(self) -> dict:
        """Traversal counters of the current rays (diagnostic, ptExtendStats)."""
        out = (C.c_uint64 * 14)()
        _check(N.hip_lib().ptExtendStats(self.device.handle, self._h, out), "ptExtendStats")
        keys = ("rays", "lane_steps", "wave_steps_x64", "internal_nodes", "blas_leaves", "faces", "pops",
                "tlas_leaves", "waves", "blas_steps_distinct1", "blas_steps_distinct2", "blas_steps_distinct3_4",
                "blas_steps_distinct5_8", "blas_steps_distinct9_")
        d = dict(zip(keys, (int(x) for x in out)))
        d["simd_efficiency"] = d["lane_steps"] / max(d["wave_steps_x64"], 1)
        for k in ("lane_steps", "internal_nodes", "blas_leaves", "faces", "pops", "tlas_leaves"):
            d[k + "_per_ray"] = d[k] / max(d["rays"], 1)
        return d

    def _slot_count(self) -> int:
        sb = self.sample_buffer
        tiles_x, bands = (sb.width + 15) // 16, (sb.height + 15) // 16
        owned = (bands - self.rank + self.nranks - 1) // self.nranks if bands > self.rank else 0
        return owned * tiles_x * 256 * self.streams

    def extend_step_counts(self) -> np.ndarray:
        """Traversal steps of every current ray, per ray position (diagnostic)."""
        out = np.zeros(self._slot_count(), dtype=np.uint32)
        _check(N.hip_lib().ptExtendStepCounts(self.device.handle, self._h, out.ctypes.data), "ptExtendStepCounts")
        return out

    def read_state(self, stream: int = 0) -> np.ndarray:
        """Per-pixel state of one path stream, image order (owned pixels)."""
        sb = self.sample_buffer
        out = np.zeros(sb.width * sb.height, dtype=N.PIXEL_STATE_DTYPE)
        _check(N.hip_lib().ptReadBasicRendererStreamState(self.device.handle, self._h, int(stream), out.ctypes.data),
               "ptReadBasicRendererStreamState")
        return out.reshape(sb.height, sb.width)

    def write_state(self, state: np.ndarray, stream: int = 0):
        """Resume: restore every owned pixel's live path of one stream from a
        saved read_state() (ptWriteBasicRendererStreamState): the next ray and
        the path record; the trace record is not needed (the next run traces
        first).  With the sample buffer (SampleBuffer.write) and FrameIndex
        restored too, later runs equal the uninterrupted render bit for bit."""
        sb = self.sample_buffer
        a = np.ascontiguousarray(state, dtype=N.PIXEL_STATE_DTYPE).reshape(-1)
        if a.size != sb.width * sb.height:
            raise ValueError(f"state has {a.size} pixels, the sample buffer {sb.width * sb.height}")
        _check(N.hip_lib().ptWriteBasicRendererStreamState(self.device.handle, self._h, int(stream), a.ctypes.data),
               "ptWriteBasicRendererStreamState")

    def read_accumulator(self, stream: int = 0) -> np.ndarray:
        """One path stream's own accumulator (H, W, 4) (the sample buffer for one stream)."""
        sb = self.sample_buffer
        out = np.zeros((sb.height, sb.width, 4), dtype=np.float32)
        _check(N.hip_lib().ptReadBasicRendererStreamAccumulator(self.device.handle, self._h, int(stream), N.fptr(out)),
               "ptReadBasicRendererStreamAccumulator")
        return out

    def write_accumulator(self, rgba: np.ndarray, stream: int = 0):
        """Restore one path stream's own accumulator (resume of a multi-stream render)."""
        sb = self.sample_buffer
        a = np.ascontiguousarray(rgba, dtype=np.float32).reshape(sb.height, sb.width, 4)
        _check(N.hip_lib().ptWriteBasicRendererStreamAccumulator(self.device.handle, self._h, int(stream), N.fptr(a)),
               "ptWriteBasicRendererStreamAccumulator")

    def shade_info(self) -> dict:
        """The shade variant this renderer runs (diagnostic, ptGetBasicRendererShadeInfo):
        scene / kernel PT_SHADE_* masks, completion queue, grey path records."""
        info = N.pt_shade_info()
        _check(N.hip_lib().ptGetBasicRendererShadeInfo(self._h, C.byref(info)), "ptGetBasicRendererShadeInfo")
        return {"scene_mask": int(info.scene_mask), "kernel_mask": int(info.kernel_mask),
                "completion_queue": bool(info.completion_queue), "grey_records": bool(info.grey_records)}

    def close(self):
        if self._h:
            N.hip_lib().ptDestroyBasicRenderer(self.device.handle, self._h)
            self._h = None


class PreviewParameters:
    """preview_parameters (preview_render.hpp:22-33).  camera_to: the camera's
    4x4 world transform (column-major 16 floats or a (4,4) array, like
    packed_transform.To); From is not read by the preview."""

    def __init__(self, camera_to, RenderMode=0, Brightness=1.0, SelectedShapeIndex=0xFFFFFFFF,
                 RenderSizeX=640, RenderSizeY=360, MouseX=0xFFFFFFFF, MouseY=0xFFFFFFFF):
        m = np.asarray(camera_to, dtype=np.float32)
        self.camera_to = (m.T.reshape(-1) if m.shape == (4, 4) else m.reshape(-1)).copy()
        self.RenderMode, self.Brightness, self.SelectedShapeIndex = int(RenderMode), float(Brightness), int(SelectedShapeIndex)
        self.RenderSizeX, self.RenderSizeY, self.MouseX, self.MouseY = int(RenderSizeX), int(RenderSizeY), int(MouseX), int(MouseY)

    def as_struct(self) -> N.pt_preview_parameters:
        p = N.pt_preview_parameters()
        p.CameraTransform.To[:] = [float(x) for x in self.camera_to]
        p.RenderMode, p.Brightness, p.SelectedShapeIndex = self.RenderMode, self.Brightness, self.SelectedShapeIndex
        p.RenderSizeX, p.RenderSizeY, p.MouseX, p.MouseY = self.RenderSizeX, self.RenderSizeY, self.MouseX, self.MouseY
        return p


class PreviewRenderContext:
    """preview_render_context (preview_render.hpp:15-20): primary-ray preview,
    AOVs and pick queries over a DeviceScene."""

    def __init__(self, device: Device, scene: DeviceScene):
        L = N.hip_lib()
        self.device, self.scene = device, scene
        self._h = L.ptCreatePreviewRenderContext(device.handle, scene.handle)
        if not self._h:
            raise PathTracerError(L.ptGetLastError().decode())
        self._size = (0, 0)

    def render(self, params: PreviewParameters):
        _check(N.hip_lib().ptRenderPreview(self.device.handle, self._h, C.byref(params.as_struct())), "ptRenderPreview")
        self._size = (params.RenderSizeY, params.RenderSizeX)

    def query(self) -> int:
        """RetrievePreviewQueryResult: shape index under the mouse (0xFFFFFFFF = none)."""
        v = C.c_uint32(0)
        _check(N.hip_lib().ptRetrievePreviewQueryResult(self.device.handle, self._h, C.byref(v)),
               "ptRetrievePreviewQueryResult")
        return int(v.value)

    def image(self) -> np.ndarray:
        out = np.zeros(self._size + (4,), dtype=np.float32)
        _check(N.hip_lib().ptReadPreviewImage(self.device.handle, self._h, N.fptr(out)), "ptReadPreviewImage")
        return out

    def aovs(self) -> np.ndarray:
        out = np.zeros(self._size, dtype=N.PREVIEW_AOV_DTYPE)
        _check(N.hip_lib().ptReadPreviewAOVs(self.device.handle, self._h, out.ctypes.data), "ptReadPreviewAOVs")
        return out

    def close(self):
        if self._h:
            N.hip_lib().ptDestroyPreviewRenderContext(self.device.handle, self._h)
            self._h = None


class Comm:
    """RCCL communicator (one process per GPU) for the frame-end reduce."""

    def __init__(self, device: Device, nranks: int, rank: int, unique_id: bytes):
        L = N.hip_lib()
        buf = (C.c_uint8 * 128)(*unique_id)
        self.device = device
        self._h = L.ptCommCreate(device.handle, nranks, rank, buf)
        if not self._h:
            raise PathTracerError(L.ptGetLastError().decode())

    def set_timeout(self, seconds: float):
        """Deadline of a device-stream wait while this communicator is live
        (ptCommSetTimeout; default 600 s).  Past it the communicators are
        aborted and the waiting call raises (PT_ERROR_TIMEOUT)."""
        _check(N.hip_lib().ptCommSetTimeout(self._h, float(seconds)), "ptCommSetTimeout")

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * 128)()
        _check(N.hip_lib().ptCommGetUniqueId(buf), "ptCommGetUniqueId")
        return bytes(buf)

    def reduce_sample_buffer(self, sample_buffer: SampleBuffer, root: int = 0):
        _check(N.hip_lib().ptCommReduceSampleBuffer(self.device.handle, self._h, sample_buffer.handle, root),
               "ptCommReduceSampleBuffer")

    def reduce_sample_buffer_into(self, sample_buffer: SampleBuffer, total: SampleBuffer | None, root: int = 0):
        """Sample sharding: `total` on `root` = sum over ranks of their own
        accumulators (ptCommReduceSampleBufferInto); `total` may be None
        on the other ranks."""
        _check(N.hip_lib().ptCommReduceSampleBufferInto(self.device.handle, self._h, sample_buffer.handle,
                                                         total.handle if total is not None else None, root),
               "ptCommReduceSampleBufferInto")

    def gather_sample_buffer(self, sample_buffer: SampleBuffer, root: int = 0):
        """Each rank's own bands, point-to-point to `root` (1/N of the reduce's traffic)."""
        _check(N.hip_lib().ptCommGatherSampleBuffer(self.device.handle, self._h, sample_buffer.handle, root),
               "ptCommGatherSampleBuffer")

    def close(self):
        if self._h:
            N.hip_lib().ptCommDestroy(self._h)
            self._h = None


# Reference-named free functions ------------------------------------------------

def CreateSampleBuffer(device: Device, width: int, height: int) -> SampleBuffer:
    return SampleBuffer(device, width, height)


def CreateBasicRenderer(device: Device, scene: DeviceScene, sample_buffer: SampleBuffer) -> BasicRenderer:
    return BasicRenderer(device, scene, sample_buffer)


def ResetBasicRenderer(device: Device, renderer: BasicRenderer):
    renderer.reset()


def RunBasicRenderer(device: Device, renderer: BasicRenderer, rounds: int):
    renderer.run(rounds)


def DestroyBasicRenderer(device: Device, renderer: BasicRenderer):
    renderer.close()


def DestroySampleBuffer(device: Device, sample_buffer: SampleBuffer):
    sample_buffer.close()


def RenderSampleBuffer(device: Device, sample_buffer: SampleBuffer, parameters: ResolveParameters):
    sample_buffer.render(parameters)


def CreatePreviewRenderContext(device: Device, scene: DeviceScene) -> PreviewRenderContext:
    return PreviewRenderContext(device, scene)


def RenderPreview(device: Device, context: PreviewRenderContext, parameters: PreviewParameters):
    context.render(parameters)


def RetrievePreviewQueryResult(device: Device, context: PreviewRenderContext) -> int:
    return context.query()
