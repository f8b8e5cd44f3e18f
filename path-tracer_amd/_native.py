"""ctypes bindings of the C ABI (include/pt_api.h, include/pt_scene.h).

The libraries are built in-tree by path-tracer_amd/build.py.  There is no
fallback: if libpathtracer.so cannot be loaded, every device entry point
raises, so a GPU run can never silently take a CPU path.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG = Path(__file__).resolve().parent
SCENE_LIB_PATH = PKG / "libptscene.so"
HIP_LIB_PATH = PKG / "libpathtracer.so"


class NativeLibraryMissing(RuntimeError):
    pass


# --- structs (include/pt_packed.h, include/pt_api.h) ---------------------------

class pt_scene_packs(C.Structure):
    _fields_ = [
        ("globals", C.c_void_p),
        ("textures", C.c_void_p), ("texture_count", C.c_uint32),
        ("material_data", C.c_void_p), ("material_word_count", C.c_uint32),
        ("shapes", C.c_void_p), ("shape_count", C.c_uint32),
        ("shape_nodes", C.c_void_p), ("shape_node_count", C.c_uint32),
        ("mesh_faces", C.c_void_p), ("mesh_face_count", C.c_uint32),
        ("mesh_vertices", C.c_void_p), ("mesh_vertex_count", C.c_uint32),
        ("mesh_nodes", C.c_void_p), ("mesh_node_count", C.c_uint32),
        ("cameras", C.c_void_p), ("camera_count", C.c_uint32),
        ("atlas", C.c_void_p),
        ("atlas_width", C.c_uint32), ("atlas_height", C.c_uint32), ("atlas_layer_count", C.c_uint32),
    ]


class pt_shade_info(C.Structure):
    """pt_shade_info (include/pt_api.h): the shade variant a renderer runs."""
    _fields_ = [("scene_mask", C.c_uint32), ("kernel_mask", C.c_uint32), ("completion_queue", C.c_uint32),
                ("grey_records", C.c_uint32)]


SHADE_DIFFUSE, SHADE_METAL, SHADE_TRANSLUCENT, SHADE_SCATTER = 1, 2, 4, 8
SHADE_OPENPBR, SHADE_PRIMS, SHADE_SKY, SHADE_TEXWRAP = 16, 32, 64, 128


class pt_basic_renderer_params(C.Structure):
    _fields_ = [
        ("FrameIndex", C.c_uint32),
        ("CameraIndex", C.c_uint32),
        ("RenderFlags", C.c_uint32),
        ("PathLengthLimit", C.c_uint32),
        ("PathTerminationProbability", C.c_float),
    ]


class pts_load_model_options(C.Structure):
    """load_model_options (src/scene/scene.hpp:383-391) + openpbr_as_diffuse."""
    _fields_ = [
        ("name", C.c_char_p), ("directory_path", C.c_char_p),
        ("vertex_transform", C.c_float * 16), ("normal_transform", C.c_float * 16),
        ("texcoord_transform", C.c_float * 9), ("openpbr_as_diffuse", C.c_int),
    ]


class pt_resolve_parameters(C.Structure):
    """resolve_parameters (src/integrator/integrator.hpp:43-48)."""
    _fields_ = [
        ("Brightness", C.c_float),
        ("ToneMappingMode", C.c_uint32),
        ("ToneMappingWhiteLevel", C.c_float),
    ]


class pt_packed_transform(C.Structure):
    _fields_ = [("To", C.c_float * 16), ("From", C.c_float * 16)]


class pt_preview_parameters(C.Structure):
    """preview_parameters (src/application/preview_render.hpp:22-33)."""
    _fields_ = [
        ("CameraTransform", pt_packed_transform),
        ("RenderMode", C.c_uint32),
        ("Brightness", C.c_float),
        ("SelectedShapeIndex", C.c_uint32),
        ("RenderSizeX", C.c_uint32), ("RenderSizeY", C.c_uint32),
        ("MouseX", C.c_uint32), ("MouseY", C.c_uint32),
    ]


class pts_config_info(C.Structure):
    _fields_ = [
        ("width", C.c_uint32), ("height", C.c_uint32), ("spp", C.c_uint32), ("camera_count", C.c_uint32),
        ("render_flags", C.c_uint32), ("termination_probability", C.c_float),
        ("mesh_face_count", C.c_uint32), ("shape_count", C.c_uint32),
    ]


HIT_RECORD_DTYPE = np.dtype([
    ("time", "<f4"), ("shape_material", "<u4"), ("packed_normal", "<u4"),
    ("packed_tangent", "<u4"), ("u", "<f4"), ("v", "<f4"),
])
assert HIT_RECORD_DTYPE.itemsize == 24

PIXEL_STATE_DTYPE = np.dtype([
    ("origin", "<f4", (3,)), ("packed_velocity", "<u4"),
    ("hit", HIT_RECORD_DTYPE),
    ("lambda0", "<f4"), ("throughput", "<f4", (4,)), ("probability", "<f4", (4,)),
    ("sample", "<f4", (3,)), ("active01", "<u4"), ("active23", "<u4"),
])
assert PIXEL_STATE_DTYPE.itemsize == 96

PREVIEW_AOV_DTYPE = np.dtype([
    ("time", "<f4"), ("shape_index", "<u4"), ("material_index", "<u4"), ("primitive_index", "<u4"),
    ("mesh_complexity", "<u4"), ("scene_complexity", "<u4"), ("normal", "<f4", (3,)), ("u", "<f4"), ("v", "<f4"),
    ("reserved", "<u4"),
])
assert PREVIEW_AOV_DTYPE.itemsize == 48

# Packed scene layouts (include/pt_packed.h) as numpy dtypes, for tests.
SHAPE_NODE_DTYPE = np.dtype([("Minimum", "<f4", (3,)), ("ChildNodeIndices", "<u4"),
                             ("Maximum", "<f4", (3,)), ("ShapeIndex", "<u4")])
MESH_NODE_DTYPE = np.dtype([("Minimum", "<f4", (3,)), ("FaceBeginOrNodeIndex", "<u4"),
                            ("Maximum", "<f4", (3,)), ("FaceEndIndex", "<u4")])
MESH_FACE_DTYPE = np.dtype([("Position0", "<f4", (3,)), ("VertexIndex0", "<u4"),
                            ("Position1", "<f4", (3,)), ("VertexIndex1", "<u4"),
                            ("Position2", "<f4", (3,)), ("VertexIndex2", "<u4")])
MESH_VERTEX_DTYPE = np.dtype([("PackedNormal", "<u4"), ("PackedUV", "<u4")])
TRANSFORM_DTYPE = np.dtype([("To", "<f4", (16,)), ("From", "<f4", (16,))])
SHAPE_DTYPE = np.dtype([("Type", "<i4"), ("MaterialIndex", "<u4"), ("MeshRootNodeIndex", "<u4"),
                        ("Pad0", "<u4"), ("Transform", TRANSFORM_DTYPE)])
CAMERA_DTYPE = np.dtype([("Model", "<u4"), ("FocalLength", "<f4"), ("ApertureRadius", "<f4"),
                         ("SensorDistance", "<f4"), ("SensorSize", "<f4", (2,)), ("Pad0", "<u4", (2,)),
                         ("Transform", TRANSFORM_DTYPE)])
TEXTURE_DTYPE = np.dtype([("AtlasPlacementMinimum", "<f4", (2,)), ("AtlasPlacementMaximum", "<f4", (2,)),
                          ("AtlasImageIndex", "<u4"), ("Type", "<u4"), ("Flags", "<u4"), ("Unused0", "<u4")])
GLOBALS_DTYPE = np.dtype([("SkyboxMeanDirection", "<f4", (3,)), ("SkyboxConcentration", "<f4"),
                          ("SkyboxSamplingProbability", "<f4"), ("SkyboxBrightness", "<f4"),
                          ("SkyboxTextureIndex", "<u4"), ("ShapeCount", "<u4"), ("SceneScatterRate", "<f4"),
                          ("Pad0", "<u4", (3,))])
assert SHAPE_NODE_DTYPE.itemsize == 32 and MESH_NODE_DTYPE.itemsize == 32 and MESH_FACE_DTYPE.itemsize == 48
assert SHAPE_DTYPE.itemsize == 144 and CAMERA_DTYPE.itemsize == 160 and GLOBALS_DTYPE.itemsize == 48
assert TEXTURE_DTYPE.itemsize == 32

KERNEL_RAYGEN, KERNEL_EXTEND, KERNEL_SHADE, KERNEL_RESOLVE = 0, 1, 2, 3
TONE_MAPPING_CLAMP, TONE_MAPPING_REINHARD, TONE_MAPPING_HABLE, TONE_MAPPING_ACES = 0, 1, 2, 3
(PREVIEW_RENDER_MODE_BASE_COLOR, PREVIEW_RENDER_MODE_BASE_COLOR_SHADED, PREVIEW_RENDER_MODE_NORMAL,
 PREVIEW_RENDER_MODE_MATERIAL_INDEX, PREVIEW_RENDER_MODE_PRIMITIVE_INDEX, PREVIEW_RENDER_MODE_MESH_COMPLEXITY,
 PREVIEW_RENDER_MODE_SCENE_COMPLEXITY) = range(7)
KERNEL_PREVIEW = 4
KERNEL_ROUND = 5     # fused extend + shade (partitions that fit the GPU at once)
KERNEL_ROUNDS = 6    # a round batch: several rounds of every tile in one launch (PT_KERNEL_ROUNDS)
MAX_SPLIT = 4        # PT_MAX_SPLIT: tile groups of ptSetBasicRendererSplit

_vp = C.c_void_p
_u32 = C.c_uint32
_f32 = C.c_float
_i32 = C.c_int
_fptr = C.POINTER(C.c_float)
_u32ptr = C.POINTER(C.c_uint32)

# name: (restype, argtypes)
SCENE_API = {
    "ptsGetLastError": (C.c_char_p, []),
    "ptsCreateScene": (_vp, []),
    "ptsCreateEmptyScene": (_vp, []),
    "ptsCreateConfigScene": (_vp, [_i32, C.POINTER(pts_config_info)]),
    "ptsDestroyScene": (None, [_vp]),
    "ptsSceneRoot": (_vp, [_vp]),
    "ptsCreateEntity": (_vp, [_vp, _i32, _vp]),
    "ptsSetEntityTransform": (None, [_vp, _vp, _fptr, _fptr, _fptr]),
    "ptsSetEntityActive": (None, [_vp, _vp, _i32]),
    "ptsSetEntityMaterial": (None, [_vp, _vp, _vp]),
    "ptsSetEntityMesh": (None, [_vp, _vp, _vp]),
    "ptsEntityPackedShapeIndex": (_u32, [_vp]),
    "ptsSetCameraPinhole": (None, [_vp, _vp, _f32, _f32]),
    "ptsSetCameraThinLens": (None, [_vp, _vp, _f32, _f32, _f32, _f32, _f32]),
    "ptsSetCamera360": (None, [_vp, _vp]),
    "ptsFindCamera": (_vp, [_vp, _u32]),
    "ptsSetCameraTransform": (None, [_vp, _vp, _fptr, _fptr]),
    "ptsSetRootParameters": (None, [_vp, _f32, _f32, _f32, _vp]),
    "ptsCreateMaterial": (_vp, [_vp, _i32, C.c_char_p]),
    "ptsSetMaterialParameter": (_i32, [_vp, _vp, C.c_char_p, _fptr, _i32]),
    "ptsSetMaterialTexture": (_i32, [_vp, _vp, C.c_char_p, _vp]),
    "ptsMaterialPackedIndex": (_u32, [_vp]),
    "ptsCreateCheckerTexture": (_vp, [_vp, C.c_char_p, _i32, _fptr, _fptr]),
    "ptsCreateTexture": (_vp, [_vp, C.c_char_p, _i32, _u32, _u32, _fptr, _i32]),
    "ptsCreateMesh": (_vp, [_vp, C.c_char_p, _u32, _fptr, _fptr, _fptr, _u32, _u32ptr]),
    "ptsMeshDepth": (_u32, [_vp]),
    "ptsMeshNodeCount": (_u32, [_vp]),
    "ptsMeshFaces": (None, [_vp, _u32ptr]),
    "ptsDefaultLoadModelOptions": (None, [C.POINTER(pts_load_model_options)]),
    "ptsLoadTexture": (_vp, [_vp, C.c_char_p, _i32, C.c_char_p]),
    "ptsLoadImageRGBA8": (_i32, [C.c_char_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), _vp]),
    "ptsLoadModelAsPrefab": (_vp, [_vp, C.c_char_p, C.POINTER(pts_load_model_options)]),
    "ptsInstantiatePrefab": (_vp, [_vp, _vp, _vp]),
    "ptsLoadScene": (_vp, [C.c_char_p]),
    "ptsSaveScene": (_i32, [_vp, C.c_char_p]),
    "ptsSceneTextureCount": (_u32, [_vp]),
    "ptsSceneMaterialCount": (_u32, [_vp]),
    "ptsSceneMeshCount": (_u32, [_vp]),
    "ptsScenePrefabCount": (_u32, [_vp]),
    "ptsPrefabMeshCount": (_u32, [_vp]),
    "ptsPrefabMesh": (_vp, [_vp, _u32, C.POINTER(_vp), _fptr]),
    "ptsMeshVertexCount": (_u32, [_vp]),
    "ptsMeshFaceCount": (_u32, [_vp]),
    "ptsMeshVertices": (None, [_vp, _fptr]),
    "ptsMaterialType": (_i32, [_vp]),
    "ptsPackSceneData": (_u32, [_vp]),
    "ptsGetScenePacks": (None, [_vp, C.POINTER(pt_scene_packs)]),
    "ptsMarkDirty": (None, [_vp, _u32]),
    "ptsGetParametricSpectrumCoefficients": (_i32, [_fptr, _fptr]),
    "ptsBuildSpectrumTable": (_i32, [_i32]),
    "ptsSaveSpectrumTable": (_i32, [C.c_char_p]),
    "ptsLoadSpectrumTable": (_i32, [C.c_char_p]),
    "ptsSetSpectrumTablePath": (None, [C.c_char_p]),
}

HIP_API = {
    "ptGetLastError": (C.c_char_p, []),
    "ptGetDeviceCount": (_i32, [C.POINTER(_i32)]),
    "ptCreateDevice": (_vp, [_i32]),
    "ptDestroyDevice": (None, [_vp]),
    "ptSynchronize": (_i32, [_vp]),
    "ptCreateScene": (_vp, [_vp]),
    "ptUpdateScene": (_i32, [_vp, _vp, C.POINTER(pt_scene_packs), _u32]),
    "ptSetSceneStackFormat": (_i32, [_vp, _u32]),
    "ptSetSceneHitRecordForm": (_i32, [_vp, _u32]),
    "ptDestroyScene": (None, [_vp, _vp]),
    "ptCreateSampleBuffer": (_vp, [_vp, _u32, _u32]),
    "ptDestroySampleBuffer": (None, [_vp, _vp]),
    "ptReadSampleBuffer": (_i32, [_vp, _vp, _fptr]),
    "ptWriteSampleBuffer": (_i32, [_vp, _vp, _fptr]),
    "ptRenderSampleBuffer": (_i32, [_vp, _vp, C.POINTER(pt_resolve_parameters)]),
    "ptReadResolvedImage": (_i32, [_vp, _vp, _fptr]),
    "ptReadResolvedImageSRGB8": (_i32, [_vp, _vp, C.POINTER(C.c_uint8)]),
    "ptCreateBasicRenderer": (_vp, [_vp, _vp, _vp]),
    "ptCreateBasicRendererPartitioned": (_vp, [_vp, _vp, _vp, _u32, _u32]),
    "ptCreateBasicRendererStreams": (_vp, [_vp, _vp, _vp, _u32, _u32, _u32]),
    "ptMergeBasicRendererStreams": (_i32, [_vp, _vp]),
    "ptBasicRendererStreams": (_u32, [_vp]),
    "ptReadBasicRendererStreamState": (_i32, [_vp, _vp, _u32, _vp]),
    "ptWriteBasicRendererState": (_i32, [_vp, _vp, _vp]),
    "ptWriteBasicRendererStreamState": (_i32, [_vp, _vp, _u32, _vp]),
    "ptReadBasicRendererStreamAccumulator": (_i32, [_vp, _vp, _u32, _fptr]),
    "ptWriteBasicRendererStreamAccumulator": (_i32, [_vp, _vp, _u32, _fptr]),
    "ptGetBasicRendererShadeInfo": (_i32, [_vp, C.POINTER(pt_shade_info)]),
    "ptDestroyBasicRenderer": (None, [_vp, _vp]),
    "ptBasicRendererParams": (C.POINTER(pt_basic_renderer_params), [_vp]),
    "ptResetBasicRenderer": (_i32, [_vp, _vp]),
    "ptRunBasicRenderer": (_i32, [_vp, _vp, _u32]),
    "ptBasicRendererSlotCount": (_u32, [_vp]),
    "ptSetBasicRendererFusedRounds": (_i32, [_vp, _i32]),
    "ptRunBasicRendererRounds": (_i32, [_vp, _vp, _u32]),
    "ptSetBasicRendererRoundBatch": (_i32, [_vp, _u32]),
    "ptSetBasicRendererSplit": (_i32, [_vp, _u32]),
    "ptSetBasicRendererClassLists": (_i32, [_vp, _u32]),
    "ptGetBasicRendererClassLists": (_i32, [_vp, _u32ptr]),
    "ptGetBasicRendererSplit": (_i32, [_vp, _u32ptr, _u32ptr, _u32ptr]),
    "ptSetBasicRendererOpenPBR": (_i32, [_vp, _i32]),
    "ptGetStats": (_i32, [_vp, _vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "ptTraceRaysStats": (_i32, [_vp, _vp, _u32, _fptr, _u32ptr, _fptr, C.POINTER(C.c_uint64), _vp]),
    "ptRenderFrame": (_i32, [_vp, _vp, C.c_uint64, C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)]),
    "ptReadBasicRendererState": (_i32, [_vp, _vp, _vp]),
    "ptTraceRays": (_i32, [_vp, _vp, _u32, _fptr, _u32ptr, _fptr, _vp]),
    "ptCreatePreviewRenderContext": (_vp, [_vp, _vp]),
    "ptDestroyPreviewRenderContext": (None, [_vp, _vp]),
    "ptRenderPreview": (_i32, [_vp, _vp, C.POINTER(pt_preview_parameters)]),
    "ptRetrievePreviewQueryResult": (_i32, [_vp, _vp, C.POINTER(C.c_uint32)]),
    "ptReadPreviewImage": (_i32, [_vp, _vp, _fptr]),
    "ptReadPreviewAOVs": (_i32, [_vp, _vp, _vp]),
    "ptCheckFastDivision": (_i32, [_vp, C.c_uint64, _u32, C.POINTER(C.c_uint64)]),
    "ptCheckFastReciprocal": (_i32, [_vp, C.POINTER(C.c_uint64)]),
    "ptExtendStats": (_i32, [_vp, _vp, C.POINTER(C.c_uint64)]),
    "ptExtendStepCounts": (_i32, [_vp, _vp, _vp]),
    "ptSetProfilingPeriod": (_i32, [_vp, C.c_uint32]),
    "ptSceneStackNeeded": (_i32, [_vp, C.POINTER(C.c_uint32)]),
    "ptSceneNodeCache": (_i32, [_vp, C.POINTER(C.c_uint32)]),
    "ptSetProfiling": (_i32, [_vp, _i32]),
    "ptGetKernelStats": (_i32, [_vp, _i32, C.POINTER(C.c_uint64), C.POINTER(C.c_double)]),
    "ptGetKernelRounds": (_i32, [_vp, _i32, C.POINTER(C.c_uint64)]),
    "ptResetKernelStats": (_i32, [_vp]),
    "ptCommGetUniqueId": (_i32, [C.POINTER(C.c_uint8)]),
    "ptCommCreate": (_vp, [_vp, _i32, _i32, C.POINTER(C.c_uint8)]),
    "ptCommDestroy": (None, [_vp]),
    "ptCommSetTimeout": (_i32, [_vp, C.c_double]),
    "ptCommReduceSampleBuffer": (_i32, [_vp, _vp, _vp, _i32]),
    "ptCommGatherSampleBuffer": (_i32, [_vp, _vp, _vp, _i32]),
    "ptCommReduceSampleBufferInto": (_i32, [_vp, _vp, _vp, _vp, _i32]),
}

_scene_lib = None
_hip_lib = None


def _bind(lib, table, required=True):
    """Set every entry point's ctypes signature.  required=False (a
    PT_HIP_LIB experiment build of an older tree, A/B timing only) skips the
    entry points that build lacks; calling one then raises AttributeError.
    The in-tree library must export all of them (tests/test_abi.py)."""
    for name, (res, args) in table.items():
        if not required and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def scene_lib():
    """libptscene.so (host only)."""
    global _scene_lib
    if _scene_lib is None:
        if not SCENE_LIB_PATH.exists():
            raise NativeLibraryMissing(f"{SCENE_LIB_PATH} not built (run __graft_entry__.build())")
        lib = C.CDLL(str(SCENE_LIB_PATH))
        _scene_lib = _bind(lib, SCENE_API)
        table = os.environ.get("PT_SPECTRUM_TABLE")
        if table and Path(table).exists():
            _scene_lib.ptsLoadSpectrumTable(table.encode())
    return _scene_lib


def hip_lib():
    """libpathtracer.so (HIP kernels for gfx950).  Raises if absent."""
    global _hip_lib
    if _hip_lib is None:
        # PT_HIP_LIB: an alternative build of the same library (compiler-flag
        # experiments, tools/build_variant.py); the default is the in-tree one.
        path = Path(os.environ.get("PT_HIP_LIB", str(HIP_LIB_PATH)))
        if not path.exists():
            raise NativeLibraryMissing(f"{path} not built (run __graft_entry__.build())")
        lib = C.CDLL(str(path))
        _hip_lib = _bind(lib, HIP_API, required="PT_HIP_LIB" not in os.environ)
    return _hip_lib


def fptr(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(_fptr)


def u32ptr(a: np.ndarray):
    assert a.dtype == np.uint32 and a.flags.c_contiguous
    return a.ctypes.data_as(_u32ptr)
