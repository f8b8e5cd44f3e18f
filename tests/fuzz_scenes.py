"""Random scenes for the fuzz parity tests (tests/test_gpu_fuzz.py).

Each seed builds a scene through the host scene API (the reference's
CreateEntity / CreateMaterial / CreateMesh surface, scene.hpp:410-442) that
mixes what the fixed configs C1-C5 keep apart: several mesh instances under
one TLAS (BLAS enter/leave many times per ray), entity hierarchies with
rotated and non-uniformly scaled parents, every basic material type with and
without textures, nested translucent shapes (the active-shape priority
stack, basic_scatter.glsl:203-282), dispersive and scattering media, an HDR
sky sampled by the vMF lobe or not, and every camera model.  Also returns
renderer settings (RenderFlags, PathTerminationProbability) drawn from the
same seed.
"""
from __future__ import annotations

import numpy as np


def blob_mesh(rng, n_lat, n_lon, noise):
    """A closed lat-long sphere with a radially perturbed surface: positions,
    triangle indices, per-vertex normals (of the unperturbed sphere, so the
    shading normals disagree with the faces a little) and UVs."""
    th = np.linspace(0.0, np.pi, n_lat + 1)
    ph = np.linspace(0.0, 2 * np.pi, n_lon, endpoint=False)
    T, P = np.meshgrid(th, ph, indexing="ij")
    n = np.stack([np.sin(T) * np.cos(P), np.sin(T) * np.sin(P), np.cos(T)], -1).reshape(-1, 3)
    r = 1.0 + noise * rng.uniform(-1.0, 1.0, size=(len(n), 1))
    pos = n * r
    uv = np.stack([(P / (2 * np.pi)).reshape(-1), (T / np.pi).reshape(-1)], -1)
    idx = []
    for i in range(n_lat):
        for j in range(n_lon):
            a, b = i * n_lon + j, i * n_lon + (j + 1) % n_lon
            c, d = a + n_lon, b + n_lon
            if i > 0:
                idx.append((a, b, c))
            if i < n_lat - 1:
                idx.append((b, d, c))
    return pos.astype(np.float32), np.array(idx, np.uint32), n.astype(np.float32), uv.astype(np.float32)


def soup_mesh(rng, count, extent):
    """Unconnected random triangles (sizes over two decades) in a box: a
    deep, overlapping BVH with many near-ties between boxes."""
    centers = rng.uniform(-extent, extent, size=(count, 1, 3))
    size = 10.0 ** rng.uniform(-1.5, -0.3, size=(count, 1, 1))
    pos = (centers + size * rng.normal(size=(count, 3, 3))).reshape(-1, 3)
    idx = np.arange(3 * count, dtype=np.uint32).reshape(-1, 3)
    nrm = rng.normal(size=(3 * count, 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    uv = rng.uniform(-1.0, 2.0, size=(3 * count, 2))
    return pos.astype(np.float32), idx, nrm.astype(np.float32), uv.astype(np.float32)


def random_texture(rng, w, h):
    return rng.uniform(0.0, 1.0, size=(h, w, 4)).astype(np.float32)


def random_sky(rng, w=64, h=32):
    """A lat-long RGB radiance image with a bright sun lobe."""
    y, x = np.mgrid[0:h, 0:w]
    th = (y + 0.5) / h * np.pi
    ph = (x + 0.5) / w * 2 * np.pi
    d = np.stack([np.sin(th) * np.cos(ph), np.sin(th) * np.sin(ph), np.cos(th)], -1)
    s = rng.normal(size=3)
    s /= np.linalg.norm(s)
    sun = 40.0 * np.exp(60.0 * (d @ s - 1.0))
    base = rng.uniform(0.2, 1.0, size=3)
    img = np.zeros((h, w, 4), np.float32)
    img[..., :3] = base * (0.3 + 0.7 * np.clip(d[..., 2:3], 0, 1)) + sun[..., None]
    img[..., 3] = 1.0
    return img


def build(pt, seed):
    """(scene, settings) for one seed; settings = dict(flags, termination, camera)."""
    rng = np.random.default_rng(1000 + seed)
    s = pt.Scene.empty()

    # --- materials -------------------------------------------------------
    mats = []
    checker = s.create_checker_texture("Checker", pt.TEXTURE_REFLECTANCE_WITH_ALPHA,
                                       (0.9, 0.9, 0.9, 1.0), (0.2, 0.3, 0.7, 1.0))
    tex = s.create_texture("Noise", pt.TEXTURE_REFLECTANCE_WITH_ALPHA, random_texture(rng, 16, 8),
                           nearest=bool(rng.integers(2)))
    for k in range(int(rng.integers(4, 8))):
        kind = int(rng.integers(3))
        if kind == 0:
            m = s.create_material(pt.MATERIAL_BASIC_DIFFUSE, f"Diffuse{k}", BaseColor=rng.uniform(0.1, 0.95, 3))
            t = int(rng.integers(3))
            if t:
                s.set_material_parameter(m, "BaseTexture", checker if t == 1 else tex)
        elif kind == 1:
            m = s.create_material(pt.MATERIAL_BASIC_METAL, f"Metal{k}", BaseColor=rng.uniform(0.3, 1.0, 3),
                                  SpecularColor=rng.uniform(0.3, 1.0, 3),
                                  Roughness=float(rng.choice([0.0, rng.uniform(0.02, 0.6)])),
                                  RoughnessAnisotropy=float(rng.choice([0.0, rng.uniform(0.0, 0.9)])))
            if rng.integers(4) == 0:
                s.set_material_parameter(m, "RoughnessTexture", tex)
        else:
            m = s.create_material(pt.MATERIAL_BASIC_TRANSLUCENT, f"Glass{k}",
                                  IOR=float(rng.uniform(1.2, 2.0)),
                                  AbbeNumber=float(rng.choice([20.0, 40.0, 80.0])),
                                  Roughness=float(rng.choice([0.0, rng.uniform(0.05, 0.4)])),
                                  TransmissionColor=rng.uniform(0.5, 1.0, 3),
                                  TransmissionDepth=float(rng.choice([0.0, rng.uniform(0.2, 2.0)])))
            if rng.integers(3) == 0:
                s.set_material_parameter(m, "ScatteringColor", rng.uniform(0.2, 0.9, 3))
                s.set_material_parameter(m, "ScatteringAnisotropy", float(rng.uniform(-0.6, 0.8)))
        mats.append(m)
    if rng.integers(3) == 0:   # an OpenPBR surface: its hits end the path (scene.glsl.inc:685-693)
        mats.append(s.create_material(pt.MATERIAL_OPENPBR, "OpenPBR", BaseColor=(0.7, 0.7, 0.7)))

    def mat():
        return mats[int(rng.integers(len(mats)))]

    def rot():
        return tuple(rng.uniform(-np.pi, np.pi, 3))

    # --- shapes ----------------------------------------------------------
    meshes = [s.create_mesh(*blob_mesh(rng, int(rng.integers(4, 12)), int(rng.integers(6, 16)), 0.15),
                            name="Blob"),
              s.create_mesh(*soup_mesh(rng, int(rng.integers(40, 200)), 1.0), name="Soup")]
    s.create_entity(pt.ENTITY_PLANE, position=(0.0, 0.0, float(rng.uniform(-1.5, -0.5))),
                    rotation=tuple(rng.uniform(-0.2, 0.2, 3)), material=mat())
    parents = [None]
    for _ in range(int(rng.integers(1, 4))):
        parents.append(s.create_entity(pt.ENTITY_CONTAINER, parent=parents[int(rng.integers(len(parents)))],
                                       position=tuple(rng.uniform(-1, 1, 3)), rotation=rot(),
                                       scale=tuple(rng.uniform(0.6, 1.4, 3))))
    for _ in range(int(rng.integers(4, 14))):
        kind = int(rng.choice([pt.ENTITY_SPHERE, pt.ENTITY_CUBE, pt.ENTITY_MESH_INSTANCE, pt.ENTITY_MESH_INSTANCE]))
        uniform = rng.integers(2) == 0
        sc = np.full(3, rng.uniform(0.2, 0.9)) if uniform else rng.uniform(0.15, 1.0, 3)
        e = s.create_entity(kind, parent=parents[int(rng.integers(len(parents)))],
                            position=tuple(rng.uniform(-3.0, 3.0, 3) * (1.0, 1.0, 0.6) + (0.0, 0.0, 0.6)),
                            rotation=rot(), scale=tuple(sc), material=mat())
        if kind == pt.ENTITY_MESH_INSTANCE:
            s.set_mesh(e, meshes[int(rng.integers(len(meshes)))])
        if rng.integers(5) == 0:   # a nested shape inside this one (shared centre, smaller)
            s.create_entity(pt.ENTITY_SPHERE, parent=e, scale=(0.5, 0.5, 0.5), material=mat())

    # --- sky, globals, camera ---------------------------------------------
    sky = None
    if rng.integers(2):
        sky = s.create_texture("Sky", pt.TEXTURE_RADIANCE, random_sky(rng))
    s.set_root(scatter_rate=float(rng.choice([0.0, 0.0, rng.uniform(0.01, 0.08)])),
               skybox_brightness=float(rng.uniform(0.5, 2.0)),
               skybox_sampling_probability=float(rng.choice([0.0, 0.5])) if sky is not None else 0.0,
               skybox=sky)
    cam = s.create_entity(pt.ENTITY_CAMERA, position=(float(rng.uniform(-1, 1)), float(rng.uniform(-7, -5)),
                                                      float(rng.uniform(0.5, 2.0))),
                          rotation=(float(rng.uniform(1.3, 1.7)), 0.0, float(rng.uniform(-0.3, 0.3))))
    model = int(rng.integers(3))
    if model == 0:
        s.set_camera_pinhole(cam, fov_degrees=float(rng.uniform(40, 100)),
                             aperture_mm=float(rng.choice([0.0, rng.uniform(0.5, 5.0)])))
    elif model == 1:
        s.set_camera_thin_lens(cam, sensor_mm=(32.0, 16.0), focal_mm=float(rng.uniform(20, 60)),
                               aperture_mm=float(rng.uniform(2, 20)), focus=float(rng.uniform(2, 8)))
    else:
        s.set_camera_360(cam)
    s.pack()
    settings = {"flags": int(rng.choice([3, 3, 1, 2, 0])),
                "termination": float(rng.choice([0.0, 0.0, 0.15])),
                "camera": 0}
    return s, settings
