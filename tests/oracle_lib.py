"""ctypes wrapper of the CPU oracle (oracle/liboracle.so) — test infrastructure.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
ORACLE_DIR = ROOT / "oracle"
ORACLE_LIB = ORACLE_DIR / "liboracle.so"

_lib = None


def build_oracle():
    subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)


def lib():
    global _lib
    if _lib is None:
        if not ORACLE_LIB.exists():
            build_oracle()
        L = C.CDLL(str(ORACLE_LIB))
        vp, u32, f32, fptr = C.c_void_p, C.c_uint32, C.c_float, C.POINTER(C.c_float)
        L.oracle_create.restype = vp
        L.oracle_create.argtypes = [vp, u32, u32, u32, u32, C.c_int]
        L.oracle_destroy.argtypes = [vp]
        L.oracle_params.restype = vp
        L.oracle_params.argtypes = [vp]
        L.oracle_set_openpbr.argtypes = [vp, C.c_int]
        L.oracle_set_threads.argtypes = [vp, C.c_int]
        L.oracle_set_slab_division.argtypes = [C.c_int]
        L.oracle_slab_division.restype = C.c_int
        L.oracle_intersect_bounding_box.restype = f32
        L.oracle_intersect_bounding_box.argtypes = [fptr, fptr, f32, fptr, fptr]
        L.oracle_reset.argtypes = [vp]
        L.oracle_run.argtypes = [vp, u32]
        L.oracle_read_accum.argtypes = [vp, fptr]
        L.oracle_read_state.argtypes = [vp, vp]
        L.oracle_counters.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.oracle_trace_rays.argtypes = [vp, u32, fptr, C.POINTER(C.c_uint32), fptr, vp]
        for n in ("exp", "log", "sin", "cos", "asin"):
            f = getattr(L, f"oracle_fp_{n}")
            f.restype = f32
            f.argtypes = [f32]
        L.oracle_fp_atan2.restype = f32
        L.oracle_fp_atan2.argtypes = [f32, f32]
        L.oracle_pcg.restype = u32
        L.oracle_pcg.argtypes = [C.POINTER(C.c_uint32)]
        L.oracle_pack_unit_vector.restype = u32
        L.oracle_pack_unit_vector.argtypes = [fptr]
        L.oracle_unpack_unit_vector.argtypes = [u32, fptr]
        L.oracle_unpack_snorm16.restype = f32
        L.oracle_unpack_snorm16.argtypes = [u32]
        L.oracle_sample_observer.argtypes = [f32, fptr]
        L.oracle_resolve.argtypes = [fptr, u32, vp, fptr, C.POINTER(C.c_uint8)]
        L.oracle_preview.argtypes = [vp, vp, fptr, vp, C.POINTER(C.c_uint32)]
        _lib = L
    return _lib


class slab_division:
    """Context manager: the oracle's slab-test division convention inside the
    block ("ieee": correctly rounded (Min-O)/V, the default and the HIP
    kernels' convention; "rcp": RN((Min-O)*RN(1/V)), measurement only)."""

    def __init__(self, mode):
        assert mode in ("ieee", "rcp")
        self.mode = mode

    def __enter__(self):
        self.prev = lib().oracle_slab_division()
        lib().oracle_set_slab_division(1 if self.mode == "ieee" else 0)
        return self

    def __exit__(self, *exc):
        lib().oracle_set_slab_division(self.prev)


def intersect_bounding_box(origin, velocity, reach, mn, mx):
    """The oracle's slab test (common.glsl.inc:153-185) in the current convention."""
    a = [np.ascontiguousarray(x, dtype=np.float32) for x in (origin, velocity, mn, mx)]
    p = [x.ctypes.data_as(C.POINTER(C.c_float)) for x in a]
    return float(lib().oracle_intersect_bounding_box(p[0], p[1], float(reach), p[2], p[3]))


def default_threads():
    import os
    try:
        allowed = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        allowed = os.cpu_count() or 1
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(allowed, omp) if omp > 0 else allowed)


class OracleRenderer:
    """Per-pixel CPU restatement of basic_trace + basic_scatter."""

    def __init__(self, packs, width, height, rank=0, nranks=1, threads=0):
        """threads: 0 = the job's CPU share (OMP_NUM_THREADS when set, as on
        the GPU box, else this process's affinity CPUs), not every host CPU."""
        from path_tracer_amd import _native as N  # noqa: F401  (packs struct type)
        if threads <= 0:
            threads = default_threads()
        self._h = lib().oracle_create(C.addressof(packs), width, height, rank, nranks, threads)
        if not self._h:
            raise RuntimeError("oracle_create failed")
        self.width, self.height = width, height
        P = _params_struct()
        self._params = C.cast(lib().oracle_params(self._h), C.POINTER(P))

    def __getattr__(self, name):
        if name in ("FrameIndex", "CameraIndex", "RenderFlags", "PathLengthLimit", "PathTerminationProbability"):
            return getattr(self._params.contents, name)
        raise AttributeError(name)

    def __setattr__(self, name, value):
        if name in ("FrameIndex", "CameraIndex", "RenderFlags", "PathLengthLimit", "PathTerminationProbability"):
            setattr(self._params.contents, name, value)
        else:
            object.__setattr__(self, name, value)

    def set_openpbr(self, enable):
        """OpenPBR shading on/off (ptSetBasicRendererOpenPBR's counterpart)."""
        lib().oracle_set_openpbr(self._h, int(bool(enable)))

    def set_threads(self, threads):
        """Worker threads of the following rounds (CPU baseline scaling)."""
        lib().oracle_set_threads(self._h, int(threads))

    def reset(self):
        lib().oracle_reset(self._h)

    def run(self, rounds=1):
        lib().oracle_run(self._h, rounds)

    def accum(self) -> np.ndarray:
        out = np.zeros((self.height, self.width, 4), dtype=np.float32)
        lib().oracle_read_accum(self._h, out.ctypes.data_as(C.POINTER(C.c_float)))
        return out

    def state(self) -> np.ndarray:
        from path_tracer_amd import _native as N
        out = np.zeros(self.width * self.height, dtype=N.PIXEL_STATE_DTYPE)
        lib().oracle_read_state(self._h, out.ctypes.data)
        return out.reshape(self.height, self.width)

    def counters(self):
        r, s = C.c_uint64(0), C.c_uint64(0)
        lib().oracle_counters(self._h, C.byref(r), C.byref(s))
        return int(r.value), int(s.value)

    def close(self):
        if self._h:
            lib().oracle_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _params_struct():
    from path_tracer_amd import _native as N
    return N.pt_basic_renderer_params


def trace_rays(packs, origins, packed_velocities, durations):
    from path_tracer_amd import _native as N
    o = np.ascontiguousarray(origins, dtype=np.float32).reshape(-1, 3)
    v = np.ascontiguousarray(packed_velocities, dtype=np.uint32).reshape(-1)
    d = np.ascontiguousarray(durations, dtype=np.float32).reshape(-1)
    out = np.zeros(len(v), dtype=N.HIT_RECORD_DTYPE)
    lib().oracle_trace_rays(C.addressof(packs), len(v), o.ctypes.data_as(C.POINTER(C.c_float)),
                            v.ctypes.data_as(C.POINTER(C.c_uint32)), d.ctypes.data_as(C.POINTER(C.c_float)),
                            out.ctypes.data)
    return out


def pack_unit_vectors(v: np.ndarray) -> np.ndarray:
    v = np.ascontiguousarray(v, dtype=np.float32).reshape(-1, 3)
    out = np.zeros(len(v), dtype=np.uint32)
    for i in range(len(v)):
        out[i] = lib().oracle_pack_unit_vector(v[i].ctypes.data_as(C.POINTER(C.c_float)))
    return out


def resolve(accum: np.ndarray, brightness=1.0, mode=0, white=1.0):
    """RenderSampleBuffer restated on the CPU: (OutColor float32, sRGB8 uint8)."""
    from path_tracer_amd import _native as N
    a = np.ascontiguousarray(accum, dtype=np.float32)
    n = a.size // 4
    p = N.pt_resolve_parameters(brightness, mode, white)
    out = np.zeros(a.shape[:-1] + (4,), dtype=np.float32)
    out8 = np.zeros(a.shape[:-1] + (4,), dtype=np.uint8)
    lib().oracle_resolve(a.ctypes.data_as(C.POINTER(C.c_float)), n, C.addressof(p),
                         out.ctypes.data_as(C.POINTER(C.c_float)), out8.ctypes.data_as(C.POINTER(C.c_uint8)))
    return out, out8


def preview(packs, params):
    """RenderPreview restated on the CPU: (OutColor (H,W,4), AOVs (H,W), query)."""
    from path_tracer_amd import _native as N
    p = params.as_struct()
    H, W = params.RenderSizeY, params.RenderSizeX
    img = np.zeros((H, W, 4), dtype=np.float32)
    aov = np.zeros((H, W), dtype=N.PREVIEW_AOV_DTYPE)
    q = C.c_uint32(0xFFFFFFFF)
    lib().oracle_preview(C.addressof(packs), C.addressof(p), img.ctypes.data_as(C.POINTER(C.c_float)),
                         aov.ctypes.data, C.byref(q))
    return img, aov, int(q.value)
