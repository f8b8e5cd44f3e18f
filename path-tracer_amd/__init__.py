"""MI355X-native wavefront path tracer (drop-in for the integrator of
samukallio/path-tracer): host scene API + HIP/gfx950 kernels behind a C ABI.

Import as `path_tracer_amd` via the loader in tests/conftest.py or bench.py
(the directory name contains a hyphen).
"""
from . import _native
from .scene import (Scene, load_image_rgba8, spectrum_coefficients, build_spectrum_table, load_spectrum_table, mesh_depth,
                    mesh_node_count, ENTITY_CONTAINER, ENTITY_CAMERA, ENTITY_MESH_INSTANCE, ENTITY_PLANE,
                    ENTITY_SPHERE, ENTITY_CUBE, MATERIAL_BASIC_DIFFUSE, MATERIAL_BASIC_METAL,
                    MATERIAL_BASIC_TRANSLUCENT, MATERIAL_OPENPBR, TEXTURE_RAW, TEXTURE_REFLECTANCE_WITH_ALPHA,
                    TEXTURE_RADIANCE, SCENE_DIRTY_ALL, SCENE_DIRTY_GLOBALS, SCENE_DIRTY_TEXTURES,
                    SCENE_DIRTY_MATERIALS, SCENE_DIRTY_SHAPES, SCENE_DIRTY_MESHES, SCENE_DIRTY_CAMERAS,
                    SCENE_DIRTY_SKYBOX_TEXTURE, RENDER_FLAG_ACCUMULATE, RENDER_FLAG_SAMPLE_JITTER)
from .integrator import (Device, DeviceScene, SampleBuffer, BasicRenderer, Comm, PathTracerError, ResolveParameters,
                         device_count, CreateSampleBuffer, CreateBasicRenderer, ResetBasicRenderer, RunBasicRenderer,
                         DestroyBasicRenderer, DestroySampleBuffer, RenderSampleBuffer, PreviewParameters,
                         PreviewRenderContext, CreatePreviewRenderContext, RenderPreview, RetrievePreviewQueryResult)
from ._native import (PREVIEW_RENDER_MODE_BASE_COLOR, PREVIEW_RENDER_MODE_BASE_COLOR_SHADED, PREVIEW_RENDER_MODE_NORMAL,
                      PREVIEW_RENDER_MODE_MATERIAL_INDEX, PREVIEW_RENDER_MODE_PRIMITIVE_INDEX,
                      PREVIEW_RENDER_MODE_MESH_COMPLEXITY, PREVIEW_RENDER_MODE_SCENE_COMPLEXITY)
from ._native import TONE_MAPPING_CLAMP, TONE_MAPPING_REINHARD, TONE_MAPPING_HABLE, TONE_MAPPING_ACES, MAX_SPLIT
from ._native import (SHADE_DIFFUSE, SHADE_METAL, SHADE_TRANSLUCENT, SHADE_SCATTER, SHADE_OPENPBR, SHADE_PRIMS,
                      SHADE_SKY, SHADE_TEXWRAP)
from .image import write_png, write_ppm, write_pfm, read_png
from .layout import band_rows, owned_pixels

__all__ = [n for n in dir() if not n.startswith("_")]
