/*
 * pt_packed.h — byte layouts of the flattened scene buffers that feed the
 * integrator.  These are exactly the std430 structs the reference packs in
 * PackSceneData (src/scene/scene.hpp:80-173, device mirror
 * src/scene/scene.glsl.inc:30-99), so a scene packed by the reference's
 * src/scene code can be handed to ptUpdateScene() unchanged.
 *
 * Matrices are column-major float[16] (glm::mat4 memory order).
 */
#ifndef PT_PACKED_H
#define PT_PACKED_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PT_SHAPE_INDEX_NONE   0xFFFFFFFFu
#define PT_TEXTURE_INDEX_NONE 0xFFFFFFFFu

enum {
    PT_SHAPE_TYPE_MESH_INSTANCE = 0,
    PT_SHAPE_TYPE_PLANE         = 1,
    PT_SHAPE_TYPE_SPHERE        = 2,
    PT_SHAPE_TYPE_CUBE          = 3,
};

enum {
    PT_TEXTURE_TYPE_RAW                    = 0,
    PT_TEXTURE_TYPE_REFLECTANCE_WITH_ALPHA = 1,
    PT_TEXTURE_TYPE_RADIANCE               = 2,
};

#define PT_TEXTURE_FLAG_FILTER_NEAREST 1u

enum {
    PT_MATERIAL_TYPE_BASIC_DIFFUSE     = 0,
    PT_MATERIAL_TYPE_BASIC_METAL       = 1,
    PT_MATERIAL_TYPE_BASIC_TRANSLUCENT = 2,
    PT_MATERIAL_TYPE_OPENPBR           = 3,
};

enum {
    PT_CAMERA_MODEL_PINHOLE   = 0,
    PT_CAMERA_MODEL_THIN_LENS = 1,
    PT_CAMERA_MODEL_360       = 2,
};

/* scene_dirty_flag, src/scene/scene.hpp:323-333 */
enum {
    PT_SCENE_DIRTY_GLOBALS        = 1u << 0,
    PT_SCENE_DIRTY_TEXTURES       = 1u << 1,
    PT_SCENE_DIRTY_MATERIALS      = 1u << 2,
    PT_SCENE_DIRTY_SHAPES         = 1u << 3,
    PT_SCENE_DIRTY_MESHES         = 1u << 4,
    PT_SCENE_DIRTY_CAMERAS        = 1u << 5,
    PT_SCENE_DIRTY_SKYBOX_TEXTURE = 1u << 6,
    PT_SCENE_DIRTY_ALL            = 0xFFFFFFFFu,
};

/* Material attribute slots (src/scene/basic_*.glsl.inc, first lines). */
#define PT_MATERIAL_SLOT_WORDS 32
#define PT_BASIC_DIFFUSE_BASE_SPECTRUM            1
#define PT_BASIC_METAL_BASE_SPECTRUM              1
#define PT_BASIC_METAL_SPECULAR_SPECTRUM          5
#define PT_BASIC_METAL_ROUGHNESS                  9
#define PT_BASIC_METAL_ROUGHNESS_ANISOTROPY       11
#define PT_BASIC_TRANSLUCENT_IOR                  1
#define PT_BASIC_TRANSLUCENT_ABBE_NUMBER          2
#define PT_BASIC_TRANSLUCENT_ROUGHNESS            3
#define PT_BASIC_TRANSLUCENT_ROUGHNESS_ANISOTROPY 5
#define PT_BASIC_TRANSLUCENT_TRANSMISSION_SPECTRUM 7
#define PT_BASIC_TRANSLUCENT_TRANSMISSION_DEPTH   10
#define PT_BASIC_TRANSLUCENT_SCATTERING_SPECTRUM  11
#define PT_BASIC_TRANSLUCENT_SCATTERING_ANISOTROPY 14
/* OpenPBR (src/scene/openpbr.glsl.inc:1-27): 64 words, two slots. */
#define PT_OPENPBR_LAYER_BOUNCE_LIMIT                  1
#define PT_OPENPBR_BASE_WEIGHT                         2
#define PT_OPENPBR_BASE_SPECTRUM                       3
#define PT_OPENPBR_BASE_SPECTRUM_TEXTURE_INDEX         6
#define PT_OPENPBR_BASE_METALNESS                      7
#define PT_OPENPBR_BASE_DIFFUSE_ROUGHNESS              8
#define PT_OPENPBR_SPECULAR_WEIGHT                     9
#define PT_OPENPBR_SPECULAR_SPECTRUM                   10
#define PT_OPENPBR_SPECULAR_IOR                        13
#define PT_OPENPBR_SPECULAR_ROUGHNESS                  14
#define PT_OPENPBR_SPECULAR_ROUGHNESS_TEXTURE_INDEX    15
#define PT_OPENPBR_SPECULAR_ROUGHNESS_ANISOTROPY       16
#define PT_OPENPBR_TRANSMISSION_SPECTRUM               17
#define PT_OPENPBR_TRANSMISSION_WEIGHT                 20
#define PT_OPENPBR_TRANSMISSION_SCATTER_SPECTRUM       21
#define PT_OPENPBR_TRANSMISSION_SCATTER_ANISOTROPY     24
#define PT_OPENPBR_TRANSMISSION_DEPTH                  25
#define PT_OPENPBR_TRANSMISSION_DISPERSION_ABBE_NUMBER 26
#define PT_OPENPBR_EMISSION_SPECTRUM                   27
#define PT_OPENPBR_EMISSION_SPECTRUM_TEXTURE_INDEX     30
#define PT_OPENPBR_EMISSION_LUMINANCE                  31
#define PT_OPENPBR_COAT_WEIGHT                         32
#define PT_OPENPBR_COAT_COLOR_SPECTRUM                 33
#define PT_OPENPBR_COAT_IOR                            36
#define PT_OPENPBR_COAT_ROUGHNESS                      37
#define PT_OPENPBR_COAT_ROUGHNESS_ANISOTROPY           38
#define PT_OPENPBR_COAT_DARKENING                      39

typedef struct pt_packed_transform {   /* scene.hpp:82-86 */
    float To[16];
    float From[16];
} pt_packed_transform;

typedef struct pt_packed_texture {     /* scene.hpp:90-98 */
    float AtlasPlacementMinimum[2];
    float AtlasPlacementMaximum[2];
    uint32_t AtlasImageIndex;
    uint32_t Type;
    uint32_t Flags;
    uint32_t Unused0;
} pt_packed_texture;

typedef struct pt_packed_shape {       /* scene.hpp:102-108 */
    int32_t  Type;
    uint32_t MaterialIndex;
    uint32_t MeshRootNodeIndex;
    uint32_t Pad0;
    pt_packed_transform Transform;
} pt_packed_shape;

typedef struct pt_packed_shape_node {  /* scene.hpp:112-118 */
    float    Minimum[3];
    uint32_t ChildNodeIndices;         /* A | B << 16; 0 = leaf */
    float    Maximum[3];
    uint32_t ShapeIndex;
} pt_packed_shape_node;

typedef struct pt_packed_mesh_face {   /* scene.hpp:122-130 */
    float    Position0[3];
    uint32_t VertexIndex0;
    float    Position1[3];
    uint32_t VertexIndex1;
    float    Position2[3];
    uint32_t VertexIndex2;
} pt_packed_mesh_face;

typedef struct pt_packed_mesh_vertex { /* scene.hpp:134-138 */
    uint32_t PackedNormal;             /* octahedral snorm16x2 */
    uint32_t PackedUV;                 /* half2 */
} pt_packed_mesh_vertex;

typedef struct pt_packed_mesh_node {   /* scene.hpp:142-148 */
    float    Minimum[3];
    uint32_t FaceBeginOrNodeIndex;
    float    Maximum[3];
    uint32_t FaceEndIndex;             /* > 0 = leaf */
} pt_packed_mesh_node;

typedef struct pt_packed_scene_globals { /* scene.hpp:152-162 (std140 UBO) */
    float    SkyboxMeanDirection[3];
    float    SkyboxConcentration;
    float    SkyboxSamplingProbability;
    float    SkyboxBrightness;
    uint32_t SkyboxTextureIndex;
    uint32_t ShapeCount;
    float    SceneScatterRate;
    uint32_t Pad0[3];
} pt_packed_scene_globals;

typedef struct pt_packed_camera {      /* scene.hpp:166-174 */
    uint32_t Model;
    float    FocalLength;
    float    ApertureRadius;
    float    SensorDistance;
    float    SensorSize[2];
    uint32_t Pad0[2];
    pt_packed_transform Transform;
} pt_packed_camera;

/* All flattened scene data, as plain arrays.  Replaces the 11 descriptor
 * bindings of src/scene/scene.glsl.inc:121-179.  The texture atlas is
 * atlas_layer_count layers of atlas_width x atlas_height rgba32f texels
 * (the reference's 4096x4096 sampler2DArray, scene.cpp:1122-1227). */
typedef struct pt_scene_packs {
    const pt_packed_scene_globals* globals;
    const pt_packed_texture*       textures;       uint32_t texture_count;
    const uint32_t*                material_data;  uint32_t material_word_count;
    const pt_packed_shape*         shapes;         uint32_t shape_count;
    const pt_packed_shape_node*    shape_nodes;    uint32_t shape_node_count;
    const pt_packed_mesh_face*     mesh_faces;     uint32_t mesh_face_count;
    const pt_packed_mesh_vertex*   mesh_vertices;  uint32_t mesh_vertex_count;
    const pt_packed_mesh_node*     mesh_nodes;     uint32_t mesh_node_count;
    const pt_packed_camera*        cameras;        uint32_t camera_count;
    const float*                   atlas;
    uint32_t atlas_width, atlas_height, atlas_layer_count;
} pt_scene_packs;

#ifdef __cplusplus
}
static_assert(sizeof(pt_packed_transform) == 128, "packed_transform");
static_assert(sizeof(pt_packed_texture) == 32, "packed_texture");
static_assert(sizeof(pt_packed_shape) == 144, "packed_shape");
static_assert(sizeof(pt_packed_shape_node) == 32, "packed_shape_node");
static_assert(sizeof(pt_packed_mesh_face) == 48, "packed_mesh_face");
static_assert(sizeof(pt_packed_mesh_vertex) == 8, "packed_mesh_vertex");
static_assert(sizeof(pt_packed_mesh_node) == 32, "packed_mesh_node");
static_assert(sizeof(pt_packed_scene_globals) == 48, "packed_scene_globals");
static_assert(sizeof(pt_packed_camera) == 160, "packed_camera");
#endif

#endif /* PT_PACKED_H */
