// scene.hpp — host scene object / material / camera API.
//
// Restates the parts of the reference's src/scene/scene.hpp (:177-442) and
// the basic material headers (src/scene/basic_*.hpp) that produce the
// integrator's inputs: entities with transforms, the three compiled material
// types (+ OpenPBR as the reference's fallback slot), textures, meshes with
// their binned-SAH BVH, and PackSceneData() which flattens everything into the
// pt_packed_* arrays of include/pt_packed.h.  No Vulkan: the packs are handed
// to the HIP runtime through ptUpdateScene() (include/pt_api.h).
#pragma once

#include "hmath.hpp"
#include "spectrum.hpp"
#include "../../../include/pt_packed.h"

#include <string>
#include <vector>

namespace pth {

enum entity_type {
    ENTITY_TYPE_ROOT = 0,
    ENTITY_TYPE_CONTAINER = 1,
    ENTITY_TYPE_CAMERA = 2,
    ENTITY_TYPE_MESH_INSTANCE = 3,
    ENTITY_TYPE_PLANE = 4,
    ENTITY_TYPE_SPHERE = 5,
    ENTITY_TYPE_CUBE = 6,
};

struct transform {                    // src/core/common.hpp:47-53
    vec3 Position = vec3(0, 0, 0);
    vec3 Rotation = vec3(0, 0, 0);
    vec3 Scale = vec3(1, 1, 1);
};

struct bounds {                       // src/core/common.hpp:55-59
    vec3 Minimum = vec3(+INF);
    vec3 Maximum = vec3(-INF);
};

struct texture {                      // scene.hpp:177-186
    std::string Name = "New Texture";
    uint32_t Type = PT_TEXTURE_TYPE_RAW;
    bool EnableNearestFiltering = false;
    uint32_t Width = 0;
    uint32_t Height = 0;
    std::vector<vec4> Pixels;
    uint32_t PackedTextureIndex = 0;
};

struct material {                     // scene.hpp:188-196 + basic_*.hpp
    uint32_t Type = PT_MATERIAL_TYPE_BASIC_DIFFUSE;
    std::string Name = "New Material";
    uint32_t Flags = 0;               // scene.hpp:192-193: editor data, serialised, not packed
    float Opacity = 1.0f;
    uint32_t PackedMaterialIndex = 0;

    // basic_diffuse_material / basic_metal_material
    vec3 BaseColor = vec3(1, 1, 1);
    texture* BaseTexture = nullptr;
    vec3 SpecularColor = vec3(1, 1, 1);
    texture* SpecularTexture = nullptr;
    float Roughness = 0.3f;
    texture* RoughnessTexture = nullptr;
    float RoughnessAnisotropy = 0.0f;
    texture* RoughnessAnisotropyTexture = nullptr;
    // basic_translucent_material
    float IOR = 1.5f;
    float AbbeNumber = 20.0f;
    vec3 TransmissionColor = vec3(1, 1, 1);
    float TransmissionDepth = 0.0f;
    vec3 ScatteringColor = vec3(1, 1, 1);
    float ScatteringAnisotropy = 0.0f;
    // openpbr_material subset used by the packer (openpbr.hpp:3-43)
    float BaseWeight = 1.0f;
    float BaseMetalness = 0.0f;
    float BaseDiffuseRoughness = 0.0f;
    float SpecularWeight = 1.0f;
    float SpecularIOR = 1.5f;
    float TransmissionWeight = 0.0f;
    vec3 TransmissionScatter = vec3(0, 0, 0);
    float TransmissionScatterAnisotropy = 0.0f;
    float TransmissionDispersionScale = 0.0f;
    float TransmissionDispersionAbbeNumber = 20.0f;
    float CoatWeight = 0.0f;
    vec3 CoatColor = vec3(1, 1, 1);
    float CoatRoughness = 0.0f;
    float CoatRoughnessAnisotropy = 0.0f;
    float CoatIOR = 1.6f;
    float CoatDarkening = 1.0f;
    float EmissionLuminance = 0.0f;
    vec3 EmissionColor = vec3(0, 0, 0);
    texture* EmissionColorTexture = nullptr;
    int LayerBounceLimit = 16;
};

// Reference defaults differ per type (basic_metal.hpp:8, basic_translucent.hpp:7,
// openpbr.hpp:10 Roughness 0.3); OpenPBR's SpecularRoughness is Roughness here.

struct mesh_face { uint32_t VertexIndex[3]; };

struct mesh_vertex {                  // scene.hpp:203-208
    vec3 Position;
    vec3 Normal;
    vec2 UV;
};

struct mesh_node {                    // scene.hpp:210-216
    bounds Bounds;
    uint32_t FaceBeginIndex = 0;
    uint32_t FaceEndIndex = 0;
    uint32_t ChildNodeIndex = 0;
};

struct mesh {                         // scene.hpp:218-226
    std::string Name;
    std::vector<mesh_vertex> Vertices;
    std::vector<mesh_face> Faces;
    std::vector<mesh_node> Nodes;
    uint32_t Depth = 0;
    uint32_t PackedRootNodeIndex = 0;
};

struct entity {                       // scene.hpp:240-252 (+ subtype fields)
    std::string Name = "Entity";
    entity_type Type = ENTITY_TYPE_ROOT;
    bool Active = true;
    transform Transform;
    entity* Parent = nullptr;
    std::vector<entity*> Children;
    material* Material = nullptr;
    uint32_t PackedShapeIndex = PT_SHAPE_INDEX_NONE;

    // root_entity (scene.hpp:254-262)
    float ScatterRate = 0.0f;
    float SkyboxBrightness = 1.0f;
    float SkyboxSamplingProbability = 0.0f;
    texture* SkyboxTexture = nullptr;

    // camera_entity (scene.hpp:268-296)
    uint32_t CameraModel = PT_CAMERA_MODEL_PINHOLE;
    float PinholeFieldOfViewInDegrees = 90.0f;
    float PinholeApertureDiameterInMM = 0.0f;
    vec2 ThinLensSensorSizeInMM = vec2(32.0f, 18.0f);
    float ThinLensFocalLengthInMM = 20.0f;
    float ThinLensApertureDiameterInMM = 10.0f;
    float ThinLensFocusDistance = 1.0f;
    uint32_t PackedCameraIndex = 0;

    // mesh_entity
    mesh* Mesh = nullptr;
};

struct prefab {                       // scene.hpp:318-321
    entity* Entity = nullptr;
    std::vector<entity*> Owned;       // the prefab's own entity tree (not in the scene)
    ~prefab() { for (entity* E : Owned) delete E; }
};

struct load_model_options {           // scene.hpp:383-391
    std::string Name;                 // empty: file stem
    std::string DirectoryPath = ".";
    mat4 VertexTransform = mat4(1.0f);
    mat4 NormalTransform = mat4(1.0f);
    float TextureCoordinateTransform[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};   // mat3, column-major
    // Extension: create BasicDiffuse (Kd + map_Kd) instead of the reference's
    // OpenPBR materials, which its integrator does not shade.
    bool OpenPBRAsDiffuse = false;
};

struct scene {                        // scene.hpp:335-362
    entity Root;
    std::vector<entity*> Entities;    // ownership of every non-root entity
    std::vector<mesh*> Meshes;
    std::vector<material*> Materials;
    std::vector<texture*> Textures;
    std::vector<prefab*> Prefabs;
    parametric_spectrum_table* RGBSpectrumTable = nullptr;
    bool OwnsSpectrumTable = false;   // LoadScene read the scene's own spectrum.dat

    // Packed data (PackSceneData).
    uint32_t AtlasWidth = 4096, AtlasHeight = 4096;
    std::vector<std::vector<vec4>> Images;
    std::vector<pt_packed_texture> TexturePack;
    std::vector<pt_packed_shape> ShapePack;
    std::vector<pt_packed_shape_node> ShapeNodePack;
    std::vector<uint32_t> MaterialAttributePack;
    std::vector<pt_packed_mesh_face> MeshFacePack;
    std::vector<pt_packed_mesh_vertex> MeshVertexPack;
    std::vector<pt_packed_mesh_node> MeshNodePack;
    std::vector<pt_packed_camera> CameraPack;
    pt_packed_scene_globals Globals{};
    std::vector<float> AtlasFlat;     // Images concatenated (rgba32f)

    uint32_t DirtyFlags = PT_SCENE_DIRTY_ALL;

    ~scene();
};

scene* CreateEmptyScene();
// CreateScene (scene.cpp:912-943): checker-textured plane + camera at (0,0,1).
scene* CreateScene();
void DestroyScene(scene* Scene);

entity* CreateEntity(scene* Scene, entity_type Type, entity* Parent = nullptr);
material* CreateMaterial(scene* Scene, uint32_t Type, const char* Name);
texture* CreateCheckerTexture(scene* Scene, const char* Name, uint32_t Type, vec4 ColorA, vec4 ColorB);
texture* CreateTexture(scene* Scene, const char* Name, uint32_t Type, uint32_t Width, uint32_t Height,
                       const float* RGBA);

// Mesh from raw arrays, then the binned-SAH BVH of scene.cpp:851-866.
mesh* CreateMesh(scene* Scene, const char* Name, uint32_t VertexCount, const float* Positions,
                 const float* Normals, const float* UVs, uint32_t FaceCount, const uint32_t* Indices);
void BuildMeshBVH(mesh* Mesh);

// Scene ingestion (import.cpp).
texture* LoadTexture(scene* Scene, const char* Path, uint32_t Type, const char* Name, std::string* Error);
prefab* LoadModelAsPrefab(scene* Scene, const char* Path, const load_model_options* Options, std::string* Error);
entity* CreateEntity(scene* Scene, const entity* Source, entity* Parent);
entity* CreateEntity(scene* Scene, const prefab* Prefab, entity* Parent);

// Scene file format (serializer.cpp; reference serializer.cpp:511-529).
scene* LoadScene(const char* Path, std::string* Error);
bool SaveScene(const char* Path, scene* Scene, std::string* Error);

uint32_t PackSceneData(scene* Scene);
void GetScenePacks(scene* Scene, pt_scene_packs* Out);

}  // namespace pth
