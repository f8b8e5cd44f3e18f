/*
 * pt_scene.h — C ABI of the host scene library (libptscene.so).
 *
 * Wraps the restatement of the reference's src/scene object / material /
 * camera API (src/scene/scene.hpp:410-442) and of PackSceneData
 * (src/scene/scene.cpp:1115-1621), which produce the flattened buffers the
 * integrator consumes (pt_scene_packs, include/pt_packed.h).  The entity,
 * material and camera fields keep the reference's names and meaning:
 *
 *   ptsCreateScene            scene.hpp:432  CreateScene (checker plane + camera)
 *   ptsCreateEntity           scene.hpp:413  CreateEntity(Scene, Type, Parent)
 *   ptsCreateMaterial         scene.hpp:418  CreateMaterial(Scene, Type, Name)
 *   ptsCreateCheckerTexture   scene.hpp:422  CreateCheckerTexture
 *   ptsCreateMesh             scene.cpp:790-866 (mesh + BuildMeshNode BVH)
 *   ptsPackSceneData          scene.hpp:436  PackSceneData (returns dirty flags)
 *   ptsGetParametricSpectrumCoefficients  spectrum.hpp:17
 *
 * Host only: no GPU is touched.  Material parameter names are the reference's
 * field names (basic_diffuse.hpp, basic_metal.hpp, basic_translucent.hpp).
 */
#ifndef PT_SCENE_H
#define PT_SCENE_H

#include <stdint.h>
#include "pt_packed.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pts_scene pts_scene;
typedef struct pts_entity pts_entity;
typedef struct pts_material pts_material;
typedef struct pts_texture pts_texture;
typedef struct pts_mesh pts_mesh;
typedef struct pts_prefab pts_prefab;

enum {   /* entity_type, scene.hpp:228-238 */
    PTS_ENTITY_ROOT = 0,
    PTS_ENTITY_CONTAINER = 1,
    PTS_ENTITY_CAMERA = 2,
    PTS_ENTITY_MESH_INSTANCE = 3,
    PTS_ENTITY_PLANE = 4,
    PTS_ENTITY_SPHERE = 5,
    PTS_ENTITY_CUBE = 6,
};

/* Benchmark configurations (BASELINE.json "configs"). */
enum {
    PTS_CONFIG_C1_SPHERE_PLANE = 1,   /* 256x256, 16 spp */
    PTS_CONFIG_C2_CORNELL_SKY  = 2,   /* 1024x1024, 256 spp */
    PTS_CONFIG_C3_ROOM         = 3,   /* 1920x1080, 1024 spp */
    PTS_CONFIG_C4_ROOM_4K      = 4,   /* 3840x2160, 4096 spp, 8 GPUs */
    PTS_CONFIG_C5_LENS_360     = 5,   /* 2048x1024, 8192 spp */
};

typedef struct pts_config_info {
    uint32_t width, height;
    uint32_t spp;
    uint32_t camera_count;
    uint32_t render_flags;
    float    termination_probability;
    uint32_t mesh_face_count;
    uint32_t shape_count;
} pts_config_info;

/* load_model_options (scene.hpp:383-391). */
typedef struct pts_load_model_options {
    const char* name;                     /* NULL: file stem */
    const char* directory_path;           /* NULL: "." (textures and .mtl are looked up here) */
    float vertex_transform[16];           /* mat4, column-major */
    float normal_transform[16];
    float texcoord_transform[9];          /* mat3, column-major */
    int   openpbr_as_diffuse;             /* extension: BasicDiffuse instead of OpenPBR (K9) */
} pts_load_model_options;

const char* ptsGetLastError(void);

pts_scene*  ptsCreateScene(void);
pts_scene*  ptsCreateEmptyScene(void);
pts_scene*  ptsCreateConfigScene(int config, pts_config_info* info);
void        ptsDestroyScene(pts_scene* scene);

pts_entity* ptsSceneRoot(pts_scene* scene);
pts_entity* ptsCreateEntity(pts_scene* scene, int type, pts_entity* parent);
void        ptsSetEntityTransform(pts_scene* scene, pts_entity* e, const float position[3], const float rotation[3],
                                  const float scale[3]);
void        ptsSetEntityActive(pts_scene* scene, pts_entity* e, int active);
void        ptsSetEntityMaterial(pts_scene* scene, pts_entity* e, pts_material* m);
void        ptsSetEntityMesh(pts_scene* scene, pts_entity* e, pts_mesh* mesh);
uint32_t    ptsEntityPackedShapeIndex(pts_entity* e);
void        ptsSetCameraPinhole(pts_scene* scene, pts_entity* camera, float fov_degrees, float aperture_mm);
void        ptsSetCameraThinLens(pts_scene* scene, pts_entity* camera, float sensor_w_mm, float sensor_h_mm,
                                 float focal_length_mm, float aperture_mm, float focus_distance);
void        ptsSetCamera360(pts_scene* scene, pts_entity* camera);
/* The camera entity packed at `packed_index` by the last PackSceneData (NULL
 * if none), and a camera move as the editor's fly controls make it
 * (application.cpp:52-66): position / rotation (may be NULL) and only
 * SCENE_DIRTY_CAMERAS set. */
pts_entity* ptsFindCamera(pts_scene* scene, uint32_t packed_index);
void        ptsSetCameraTransform(pts_scene* scene, pts_entity* camera, const float position[3], const float rotation[3]);
/* root_entity fields (scene.hpp:254-262). */
void        ptsSetRootParameters(pts_scene* scene, float scatter_rate, float skybox_brightness,
                                 float skybox_sampling_probability, pts_texture* skybox);

pts_material* ptsCreateMaterial(pts_scene* scene, int type, const char* name);
/* name: BaseColor, SpecularColor, Roughness, RoughnessAnisotropy, IOR, AbbeNumber,
 * TransmissionColor, TransmissionDepth, ScatteringColor, ScatteringAnisotropy. */
int ptsSetMaterialParameter(pts_scene* scene, pts_material* m, const char* name, const float* values, int count);
/* name: BaseTexture, SpecularTexture, RoughnessTexture, RoughnessAnisotropyTexture. */
int ptsSetMaterialTexture(pts_scene* scene, pts_material* m, const char* name, pts_texture* t);
uint32_t ptsMaterialPackedIndex(pts_material* m);

pts_texture* ptsCreateCheckerTexture(pts_scene* scene, const char* name, int type, const float a[4], const float b[4]);
pts_texture* ptsCreateTexture(pts_scene* scene, const char* name, int type, uint32_t width, uint32_t height,
                              const float* rgba, int nearest_filtering);

/* positions/normals: 3 floats per vertex, uvs: 2 (normals/uvs may be NULL),
 * indices: 3 per face.  Builds the binned-SAH BVH (scene.cpp:435-599). */
pts_mesh* ptsCreateMesh(pts_scene* scene, const char* name, uint32_t vertex_count, const float* positions,
                        const float* normals, const float* uvs, uint32_t face_count, const uint32_t* indices);
uint32_t  ptsMeshDepth(pts_mesh* mesh);
uint32_t  ptsMeshNodeCount(pts_mesh* mesh);
/* Face vertex indices in BVH order (3 per face). */
void      ptsMeshFaces(pts_mesh* mesh, uint32_t* indices);

/* Scene ingestion: LoadTexture (scene.cpp:294-313; PNG / Radiance HDR with
 * stbi_loadf semantics), LoadModelAsPrefab (scene.cpp:601-903; Wavefront
 * OBJ + MTL), CreateEntity(Scene, Prefab, Parent) (scene.cpp:251-254). */
void        ptsDefaultLoadModelOptions(pts_load_model_options* options);
pts_texture* ptsLoadTexture(pts_scene* scene, const char* path, int type, const char* name);
/* The 8-bit RGBA samples LoadTexture linearises (JPEG / PNG / BMP / TGA;
 * stb_image's stbi_load(..., 4) semantics), for tests: returns 0 and the size
 * in *width, *height; `rgba` (may be NULL for a size query) receives
 * width*height*4 bytes. */
int ptsLoadImageRGBA8(const char* path, uint32_t* width, uint32_t* height, uint8_t* rgba);
pts_prefab* ptsLoadModelAsPrefab(pts_scene* scene, const char* path, const pts_load_model_options* options);
pts_entity* ptsInstantiatePrefab(pts_scene* scene, pts_prefab* prefab, pts_entity* parent);
uint32_t    ptsPrefabMeshCount(pts_prefab* prefab);
pts_mesh*   ptsPrefabMesh(pts_prefab* prefab, uint32_t index, pts_material** material, float position[3]);
uint32_t    ptsMeshVertexCount(pts_mesh* mesh);
uint32_t    ptsMeshFaceCount(pts_mesh* mesh);
/* vertices: 8 floats each (position, normal, uv). */
void        ptsMeshVertices(pts_mesh* mesh, float* vertices);
int         ptsMaterialType(pts_material* material);

/* Scene files: LoadScene / SaveScene (serializer.cpp:511-529): <path> is the
 * scene JSON; textures (<name>.texture), meshes (<name>.mesh) and the
 * spectrum table (spectrum.dat) sit beside it.  Load returns NULL on error. */
pts_scene*  ptsLoadScene(const char* path);
int         ptsSaveScene(pts_scene* scene, const char* path);
uint32_t    ptsSceneTextureCount(pts_scene* scene);
uint32_t    ptsSceneMaterialCount(pts_scene* scene);
uint32_t    ptsSceneMeshCount(pts_scene* scene);
uint32_t    ptsScenePrefabCount(pts_scene* scene);

uint32_t ptsPackSceneData(pts_scene* scene);
void     ptsGetScenePacks(pts_scene* scene, pt_scene_packs* out);
void     ptsMarkDirty(pts_scene* scene, uint32_t flags);

/* Spectral upsampling table (src/core/spectrum.cpp). */
int  ptsGetParametricSpectrumCoefficients(const float rgb[3], float beta[3]);
int  ptsBuildSpectrumTable(int threads);
int  ptsSaveSpectrumTable(const char* path);
int  ptsLoadSpectrumTable(const char* path);
void ptsSetSpectrumTablePath(const char* path);

#ifdef __cplusplus
}
#endif

#endif /* PT_SCENE_H */
