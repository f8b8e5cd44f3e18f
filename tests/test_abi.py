"""The C-ABI libraries load and export every entry point their headers declare,
and the product path fails loudly without a GPU (no CPU fallback)."""
from __future__ import annotations

import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
INCLUDE = ROOT / "include"
PKG = ROOT / "path-tracer_amd"


def declared_functions(header: Path, prefix: str):
    text = header.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"//[^\n]*", "", text)
    names = re.findall(r"\b(" + prefix + r"[A-Z]\w*)\s*\(", text)
    return sorted(set(names))


@pytest.mark.parametrize("header,lib,prefix", [
    ("pt_api.h", "libpathtracer.so", "pt"),
    ("pt_scene.h", "libptscene.so", "pts"),
])
def test_library_exports_every_declared_symbol(header, lib, prefix):
    names = declared_functions(INCLUDE / header, prefix)
    if prefix == "pt":
        names = [n for n in names if not n.startswith("pts")]
    assert len(names) >= 10
    L = C.CDLL(str(PKG / lib))
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, f"{lib} lacks {missing}"


def test_python_bindings_cover_headers(pt):
    N = pt._native
    api = set(declared_functions(INCLUDE / "pt_api.h", "pt")) - set(declared_functions(INCLUDE / "pt_scene.h", "pts"))
    assert api <= set(N.HIP_API), api - set(N.HIP_API)
    assert set(declared_functions(INCLUDE / "pt_scene.h", "pts")) <= set(N.SCENE_API)


def test_struct_layouts(pt):
    N = pt._native
    assert N.HIT_RECORD_DTYPE.itemsize == 24
    assert N.PIXEL_STATE_DTYPE.itemsize == 96
    assert C.sizeof(N.pt_basic_renderer_params) == 20
    assert N.SHAPE_DTYPE.itemsize == 144 and N.CAMERA_DTYPE.itemsize == 160


def test_product_path_fails_loudly_without_gpu(pt):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    assert pt.device_count() == 0
    with pytest.raises(pt.PathTracerError):
        pt.Device(0)


def test_missing_extension_raises(pt, monkeypatch):
    N = pt._native
    monkeypatch.setattr(N, "_hip_lib", None)
    monkeypatch.setattr(N, "HIP_LIB_PATH", PKG / "does-not-exist.so")
    with pytest.raises(N.NativeLibraryMissing):
        N.hip_lib()


def test_null_arguments_rejected(pt):
    """Calls with NULL handles return an error status instead of crashing."""
    L = pt._native.hip_lib()
    assert L.ptSynchronize(None) != 0
    assert L.ptRunBasicRenderer(None, None, 1) != 0
    assert L.ptResetBasicRenderer(None, None) != 0
    assert L.ptCreateSampleBuffer(None, 4, 4) is None
    assert len(L.ptGetLastError()) > 0
    L.ptDestroyBasicRenderer(None, None)
    L.ptDestroySampleBuffer(None, None)
    L.ptDestroyScene(None, None)
    L.ptDestroyDevice(None)
    assert L.ptWriteBasicRendererState(None, None, None) != 0
    assert L.ptGetBasicRendererShadeInfo(None, None) != 0
    assert L.ptReadBasicRendererStreamAccumulator(None, None, 0, None) != 0
    assert L.ptSetBasicRendererSplit(None, 2) != 0
    assert L.ptGetBasicRendererSplit(None, None, None, None) != 0
    assert L.ptSetBasicRendererClassLists(None, 0) != 0
    assert L.ptGetBasicRendererClassLists(None, None) != 0
    out = np.zeros(1, dtype=pt._native.HIT_RECORD_DTYPE)
    assert L.ptTraceRays(None, None, 1, None, None, None, out.ctypes.data) != 0
