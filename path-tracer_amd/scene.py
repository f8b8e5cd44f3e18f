"""Host scene API (mirror of the reference's src/scene/scene.hpp:410-442).

Thin Python handles over libptscene.so: CreateScene / CreateEntity /
CreateMaterial / CreateCheckerTexture / mesh creation and PackSceneData,
keeping the reference's names and field meanings.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

from . import _native as N

ENTITY_CONTAINER, ENTITY_CAMERA, ENTITY_MESH_INSTANCE, ENTITY_PLANE, ENTITY_SPHERE, ENTITY_CUBE = 1, 2, 3, 4, 5, 6
MATERIAL_BASIC_DIFFUSE, MATERIAL_BASIC_METAL, MATERIAL_BASIC_TRANSLUCENT, MATERIAL_OPENPBR = 0, 1, 2, 3
TEXTURE_RAW, TEXTURE_REFLECTANCE_WITH_ALPHA, TEXTURE_RADIANCE = 0, 1, 2
# SCENE_DIRTY_* (scene.hpp:323-333)
(SCENE_DIRTY_GLOBALS, SCENE_DIRTY_TEXTURES, SCENE_DIRTY_MATERIALS, SCENE_DIRTY_SHAPES, SCENE_DIRTY_MESHES,
 SCENE_DIRTY_CAMERAS, SCENE_DIRTY_SKYBOX_TEXTURE) = (1 << i for i in range(7))
SCENE_DIRTY_ALL = 0xFFFFFFFF
RENDER_FLAG_ACCUMULATE, RENDER_FLAG_SAMPLE_JITTER = 1, 2


def _f3(v):
    return (C.c_float * 3)(*[float(x) for x in v]) if v is not None else None


class Scene:
    """A host scene (scene.hpp:335-362) and its packed buffers."""

    def __init__(self, handle, info=None):
        if not handle:
            raise RuntimeError(N.scene_lib().ptsGetLastError().decode())
        self._h = handle
        self.info = info
        self._keep = []

    # -- construction --------------------------------------------------------
    @classmethod
    def create(cls):
        """CreateScene (scene.cpp:912-943): checker plane + camera at (0,0,1)."""
        return cls(N.scene_lib().ptsCreateScene())

    @classmethod
    def empty(cls):
        return cls(N.scene_lib().ptsCreateEmptyScene())

    @classmethod
    def config(cls, config_id: int):
        """Benchmark scene C1..C5 (BASELINE.json configs), already packed."""
        info = N.pts_config_info()
        h = N.scene_lib().ptsCreateConfigScene(int(config_id), C.byref(info))
        return cls(h, info)

    @classmethod
    def load(cls, path):
        """LoadScene (serializer.cpp:511-524): the scene JSON at `path` plus the
        .texture / .mesh / spectrum.dat files beside it."""
        return cls(N.scene_lib().ptsLoadScene(str(path).encode()))

    def save(self, path):
        """SaveScene (serializer.cpp:526-529)."""
        if N.scene_lib().ptsSaveScene(self._h, str(path).encode()) != 0:
            raise RuntimeError(N.scene_lib().ptsGetLastError().decode())

    def counts(self):
        """(textures, materials, meshes, prefabs) held by the scene."""
        L = N.scene_lib()
        return (L.ptsSceneTextureCount(self._h), L.ptsSceneMaterialCount(self._h), L.ptsSceneMeshCount(self._h),
                L.ptsScenePrefabCount(self._h))

    def close(self):
        if self._h:
            N.scene_lib().ptsDestroyScene(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    @property
    def root(self):
        return N.scene_lib().ptsSceneRoot(self._h)

    def create_entity(self, entity_type: int, parent=None, position=None, rotation=None, scale=None, material=None):
        L = N.scene_lib()
        e = L.ptsCreateEntity(self._h, int(entity_type), parent)
        if not e:
            raise RuntimeError(L.ptsGetLastError().decode())
        if position is not None or rotation is not None or scale is not None:
            L.ptsSetEntityTransform(self._h, e, _f3(position), _f3(rotation), _f3(scale))
        if material is not None:
            L.ptsSetEntityMaterial(self._h, e, material)
        return e

    def set_transform(self, entity, position=None, rotation=None, scale=None):
        N.scene_lib().ptsSetEntityTransform(self._h, entity, _f3(position), _f3(rotation), _f3(scale))

    def set_material(self, entity, material):
        N.scene_lib().ptsSetEntityMaterial(self._h, entity, material)

    def shape_index(self, entity) -> int:
        """Packed shape index of an entity after pack() (entity::PackedShapeIndex)."""
        return int(N.scene_lib().ptsEntityPackedShapeIndex(entity))

    def set_mesh(self, entity, mesh):
        N.scene_lib().ptsSetEntityMesh(self._h, entity, mesh)

    def set_camera_pinhole(self, camera, fov_degrees=90.0, aperture_mm=0.0):
        N.scene_lib().ptsSetCameraPinhole(self._h, camera, fov_degrees, aperture_mm)

    def set_camera_thin_lens(self, camera, sensor_mm=(32.0, 18.0), focal_mm=20.0, aperture_mm=10.0, focus=1.0):
        N.scene_lib().ptsSetCameraThinLens(self._h, camera, sensor_mm[0], sensor_mm[1], focal_mm, aperture_mm, focus)

    def set_camera_360(self, camera):
        N.scene_lib().ptsSetCamera360(self._h, camera)

    def find_camera(self, packed_index: int = 0):
        """The camera entity the last pack() placed at `packed_index`."""
        L = N.scene_lib()
        c = L.ptsFindCamera(self._h, int(packed_index))
        if not c:
            raise KeyError(L.ptsGetLastError().decode())
        return c

    def move_camera(self, camera, position=None, rotation=None):
        """A camera move as the editor's fly controls make it
        (application.cpp:52-66): only SCENE_DIRTY_CAMERAS is set, so the next
        pack() re-packs the cameras alone."""
        N.scene_lib().ptsSetCameraTransform(self._h, camera, _f3(position), _f3(rotation))

    def set_root(self, scatter_rate=0.0, skybox_brightness=1.0, skybox_sampling_probability=0.0, skybox=None):
        N.scene_lib().ptsSetRootParameters(self._h, scatter_rate, skybox_brightness, skybox_sampling_probability, skybox)

    def create_material(self, material_type: int, name: str = "Material", **params):
        L = N.scene_lib()
        m = L.ptsCreateMaterial(self._h, int(material_type), name.encode())
        for k, v in params.items():
            self.set_material_parameter(m, k, v)
        return m

    def set_material_parameter(self, material, name, value):
        L = N.scene_lib()
        if name.endswith("Texture"):
            rc = L.ptsSetMaterialTexture(self._h, material, name.encode(), value)
        else:
            vals = np.atleast_1d(np.asarray(value, dtype=np.float32))
            rc = L.ptsSetMaterialParameter(self._h, material, name.encode(), N.fptr(vals), len(vals))
        if rc != 0:
            raise ValueError(L.ptsGetLastError().decode())

    def create_checker_texture(self, name, texture_type, color_a, color_b):
        a = (C.c_float * 4)(*color_a)
        b = (C.c_float * 4)(*color_b)
        return N.scene_lib().ptsCreateCheckerTexture(self._h, name.encode(), int(texture_type), a, b)

    def create_texture(self, name, texture_type, rgba: np.ndarray, nearest=False):
        rgba = np.ascontiguousarray(rgba, dtype=np.float32)
        h, w = rgba.shape[:2]
        return N.scene_lib().ptsCreateTexture(self._h, name.encode(), int(texture_type), w, h, N.fptr(rgba), int(nearest))

    def create_mesh(self, positions, indices, normals=None, uvs=None, name="Mesh"):
        pos = np.ascontiguousarray(positions, dtype=np.float32).reshape(-1, 3)
        idx = np.ascontiguousarray(indices, dtype=np.uint32).reshape(-1, 3)
        nrm = None if normals is None else np.ascontiguousarray(normals, dtype=np.float32).reshape(-1, 3)
        uv = None if uvs is None else np.ascontiguousarray(uvs, dtype=np.float32).reshape(-1, 2)
        L = N.scene_lib()
        m = L.ptsCreateMesh(self._h, name.encode(), len(pos), N.fptr(pos), N.fptr(nrm) if nrm is not None else None,
                            N.fptr(uv) if uv is not None else None, len(idx), N.u32ptr(idx))
        if not m:
            raise ValueError(L.ptsGetLastError().decode())
        return m

    # -- ingestion (scene.cpp:294-313, 601-903) ---------------------------------
    def load_texture(self, path, texture_type=TEXTURE_RAW, name=None):
        """LoadTexture: JPEG, PNG, BMP, GIF, PSD, PNM, TGA or Radiance .hdr, stbi_loadf semantics."""
        L = N.scene_lib()
        t = L.ptsLoadTexture(self._h, str(path).encode(), int(texture_type), name.encode() if name else None)
        if not t:
            raise OSError(L.ptsGetLastError().decode())
        return t

    def load_model_as_prefab(self, path, name=None, directory=None, vertex_transform=None, normal_transform=None,
                             texcoord_transform=None, openpbr_as_diffuse=False):
        """LoadModelAsPrefab (Wavefront OBJ + MTL).  Transforms are 4x4 / 3x3
        arrays (column vectors, like glm); directory defaults to the OBJ's."""
        L = N.scene_lib()
        o = N.pts_load_model_options()
        L.ptsDefaultLoadModelOptions(C.byref(o))
        o.name = name.encode() if name else None
        o.directory_path = str(directory if directory is not None else Path(path).parent).encode()
        for field, m, n in (("vertex_transform", vertex_transform, 4), ("normal_transform", normal_transform, 4),
                            ("texcoord_transform", texcoord_transform, 3)):
            if m is not None:
                a = np.asarray(m, dtype=np.float32).reshape(n, n).T.reshape(-1)   # column-major
                getattr(o, field)[:] = [float(x) for x in a]
        o.openpbr_as_diffuse = int(bool(openpbr_as_diffuse))
        p = L.ptsLoadModelAsPrefab(self._h, str(path).encode(), C.byref(o))
        if not p:
            raise OSError(L.ptsGetLastError().decode())
        return p

    def instantiate_prefab(self, prefab, parent=None):
        """CreateEntity(Scene, Prefab, Parent): deep copy into the scene."""
        return N.scene_lib().ptsInstantiatePrefab(self._h, prefab, parent)

    @staticmethod
    def prefab_meshes(prefab):
        """[(vertices (n, 8): position/normal/uv, faces (m, 3), material type, instance position)]."""
        L = N.scene_lib()
        out = []
        for i in range(L.ptsPrefabMeshCount(prefab)):
            mat = C.c_void_p()
            pos = np.zeros(3, dtype=np.float32)
            m = L.ptsPrefabMesh(prefab, i, C.byref(mat), N.fptr(pos))
            nv, nf = L.ptsMeshVertexCount(m), L.ptsMeshFaceCount(m)
            v = np.zeros((nv, 8), dtype=np.float32)
            f = np.zeros((nf, 3), dtype=np.uint32)
            if nv:
                L.ptsMeshVertices(m, N.fptr(v))
            if nf:
                L.ptsMeshFaces(m, N.u32ptr(f))
            out.append((v, f, L.ptsMaterialType(mat) if mat.value else None, pos))
        return out

    # -- packing -------------------------------------------------------------
    def pack(self) -> int:
        """PackSceneData (scene.cpp:1115-1621); returns the dirty flags it packed."""
        return int(N.scene_lib().ptsPackSceneData(self._h))

    def mark_dirty(self, flags=SCENE_DIRTY_ALL):
        N.scene_lib().ptsMarkDirty(self._h, flags)

    def packs(self) -> N.pt_scene_packs:
        p = N.pt_scene_packs()
        N.scene_lib().ptsGetScenePacks(self._h, C.byref(p))
        return p

    def arrays(self):
        """numpy copies of every packed buffer (for tests and fixtures)."""
        p = self.packs()

        def view(ptr, count, dtype):
            if count == 0 or not ptr:
                return np.zeros(0, dtype=dtype)
            buf = (C.c_char * (count * np.dtype(dtype).itemsize)).from_address(ptr)
            return np.frombuffer(buf, dtype=dtype).copy()

        return {
            "globals": view(p.globals, 1, N.GLOBALS_DTYPE),
            "textures": view(p.textures, p.texture_count, N.TEXTURE_DTYPE),
            "materials": view(p.material_data, p.material_word_count, np.uint32),
            "shapes": view(p.shapes, p.shape_count, N.SHAPE_DTYPE),
            "shape_nodes": view(p.shape_nodes, p.shape_node_count, N.SHAPE_NODE_DTYPE),
            "mesh_faces": view(p.mesh_faces, p.mesh_face_count, N.MESH_FACE_DTYPE),
            "mesh_vertices": view(p.mesh_vertices, p.mesh_vertex_count, N.MESH_VERTEX_DTYPE),
            "mesh_nodes": view(p.mesh_nodes, p.mesh_node_count, N.MESH_NODE_DTYPE),
            "cameras": view(p.cameras, p.camera_count, N.CAMERA_DTYPE),
        }


def mesh_depth(mesh) -> int:
    return int(N.scene_lib().ptsMeshDepth(mesh))


def mesh_node_count(mesh) -> int:
    return int(N.scene_lib().ptsMeshNodeCount(mesh))


def load_image_rgba8(path) -> np.ndarray:
    """The 8-bit RGBA samples LoadTexture linearises (ptsLoadImageRGBA8), H x W x 4."""
    L = N.scene_lib()
    w, h = C.c_uint32(0), C.c_uint32(0)
    if L.ptsLoadImageRGBA8(str(path).encode(), C.byref(w), C.byref(h), None) != 0:
        raise ValueError(L.ptsGetLastError().decode())
    out = np.zeros((h.value, w.value, 4), dtype=np.uint8)
    L.ptsLoadImageRGBA8(str(path).encode(), None, None, out.ctypes.data)
    return out


def spectrum_coefficients(rgb) -> np.ndarray:
    """GetParametricSpectrumCoefficients (spectrum.cpp:439-479)."""
    c = np.asarray(rgb, dtype=np.float32)
    out = np.zeros(3, dtype=np.float32)
    N.scene_lib().ptsGetParametricSpectrumCoefficients(N.fptr(c), N.fptr(out))
    return out


def build_spectrum_table(path: str | None = None, threads: int = 0):
    L = N.scene_lib()
    L.ptsBuildSpectrumTable(threads)
    if path:
        if L.ptsSaveSpectrumTable(str(path).encode()) != 0:
            raise OSError(f"cannot write {path}")


def load_spectrum_table(path) -> bool:
    return N.scene_lib().ptsLoadSpectrumTable(str(path).encode()) == 0
