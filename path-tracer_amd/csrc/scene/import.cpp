// import.cpp — scene ingestion: LoadTexture (scene.cpp:294-313),
// LoadModelAsPrefab (scene.cpp:601-903) and prefab instancing
// (CreateEntity(Scene, Prefab, Parent), scene.cpp:205-254).
#include "scene.hpp"
#include "image.hpp"
#include "obj.hpp"

#include <unordered_map>
#include <unordered_set>

namespace pth {

namespace {

std::string FileName(const std::string& p)
{
    size_t s = p.find_last_of('/');
    return s == std::string::npos ? p : p.substr(s + 1);
}

std::string Stem(const std::string& p)
{
    std::string f = FileName(p);
    if (f == "." || f == "..") return f;
    size_t d = f.find_last_of('.');
    return (d == std::string::npos || d == 0) ? f : f.substr(0, d);
}

struct vertex_key {
    mesh_vertex v;
    bool operator==(const vertex_key& o) const   // scene.cpp:30-33: exact component equality
    {
        return v.Position.x == o.v.Position.x && v.Position.y == o.v.Position.y && v.Position.z == o.v.Position.z &&
               v.Normal.x == o.v.Normal.x && v.Normal.y == o.v.Normal.y && v.Normal.z == o.v.Normal.z &&
               v.UV.x == o.v.UV.x && v.UV.y == o.v.UV.y;
    }
};

struct vertex_hash {
    size_t operator()(const vertex_key& k) const
    {
        // any hash consistent with the equality; the reference's (scene.cpp:16-27)
        // only affects bucket placement, never the assigned indices
        auto h = [](float f) { return std::hash<float>()(f == 0.0f ? 0.0f : f); };
        size_t x = h(k.v.Position.x);
        for (float f : {k.v.Position.y, k.v.Position.z, k.v.Normal.x, k.v.Normal.y, k.v.Normal.z, k.v.UV.x, k.v.UV.y})
            x = x * 1000003u ^ h(f);
        return x;
    }
};

// glm mat3 * vec3 (left to right per row)
vec3 Mul3(const float m[9], vec3 v)
{
    return vec3(m[0] * v.x + m[3] * v.y + m[6] * v.z, m[1] * v.x + m[4] * v.y + m[7] * v.z,
                m[2] * v.x + m[5] * v.y + m[8] * v.z);
}

}  // namespace

texture* LoadTexture(scene* Scene, const char* Path, uint32_t Type, const char* Name, std::string* Error)
{
    int W = 0, H = 0;
    std::vector<vec4> Pixels;
    std::string Err;
    if (!LoadImageFloat(Path, W, H, Pixels, Err)) {
        if (Error) *Error = Err;
        return nullptr;
    }
    texture* T = new texture;
    T->Name = Name ? Name : FileName(Path);
    T->Type = Type;
    T->Width = (uint32_t)W;
    T->Height = (uint32_t)H;
    T->Pixels = std::move(Pixels);
    Scene->Textures.push_back(T);
    Scene->DirtyFlags |= PT_SCENE_DIRTY_TEXTURES;
    return T;
}

prefab* LoadModelAsPrefab(scene* Scene, const char* Path, const load_model_options* OptionsIn, std::string* Error)
{
    load_model_options Defaults;
    const load_model_options& Options = OptionsIn ? *OptionsIn : Defaults;

    obj_data Obj;
    if (!LoadObj(Obj, Path, Options.DirectoryPath.c_str())) {
        if (Error) *Error = Obj.error;
        return nullptr;
    }
    const size_t nv = Obj.vertices.size() / 3, nn = Obj.normals.size() / 3, nt = Obj.texcoords.size() / 2;
    for (const obj_shape& S : Obj.shapes)       // the reference reads these arrays unchecked
        for (const obj_index& I : S.indices)
            if (I.vertex_index < 0 || (size_t)I.vertex_index >= nv || I.normal_index >= (int)nn ||
                I.texcoord_index >= (int)nt) {
                if (Error) *Error = "face index out of range in " + std::string(Path);
                return nullptr;
            }

    // Smooth vertex normals when the file has none (scene.cpp:617-666).
    if (Obj.normals.empty()) {
        std::vector<float>& N = Obj.normals;
        N.assign(Obj.vertices.size(), 0.0f);
        for (obj_shape& S : Obj.shapes) {
            size_t n = S.indices.size();
            for (size_t i = 0; i < n; i += 3) {
                vec3 P[3];
                for (int j = 0; j < 3; j++) {
                    int vi = S.indices[i + j].vertex_index;
                    P[j] = vec3(Obj.vertices[3 * vi], Obj.vertices[3 * vi + 1], Obj.vertices[3 * vi + 2]);
                }
                vec3 Normal = normalize(cross(P[1] - P[0], P[2] - P[0]));
                for (int j = 0; j < 3; j++) {
                    obj_index& I = S.indices[i + j];
                    I.normal_index = I.vertex_index;
                    N[3 * I.normal_index + 0] += Normal.x;
                    N[3 * I.normal_index + 1] += Normal.y;
                    N[3 * I.normal_index + 2] += Normal.z;
                }
            }
        }
        for (size_t i = 0; i < N.size(); i += 3) {
            float L = length(vec3(N[i], N[i + 1], N[i + 2]));
            if (L > EPSILON) {
                N[i] /= L; N[i + 1] /= L; N[i + 2] /= L;
            } else {
                N[i] = 0; N[i + 1] = 0; N[i + 2] = 1;
            }
        }
    }

    // Materials (scene.cpp:668-728): OpenPBR with Kd / Ke and their maps.
    std::unordered_map<std::string, texture*> TextureMap;
    std::vector<material*> Materials;
    for (const obj_material& FM : Obj.materials) {
        material* M;
        if (Options.OpenPBRAsDiffuse) {
            M = CreateMaterial(Scene, PT_MATERIAL_TYPE_BASIC_DIFFUSE, FM.name.c_str());
        } else {
            M = CreateMaterial(Scene, PT_MATERIAL_TYPE_OPENPBR, FM.name.c_str());
            M->Roughness = 1.0f;           // SpecularRoughness
            M->SpecularIOR = 0.0f;
            M->TransmissionWeight = 0.0f;
            M->EmissionColor = vec3(FM.emission[0], FM.emission[1], FM.emission[2]);
        }
        M->BaseColor = vec3(FM.diffuse[0], FM.diffuse[1], FM.diffuse[2]);
        struct slot { const std::string* name; uint32_t type; texture** dst; };
        slot Slots[2] = {{&FM.diffuse_texname, PT_TEXTURE_TYPE_REFLECTANCE_WITH_ALPHA, &M->BaseTexture},
                         {&FM.emissive_texname, PT_TEXTURE_TYPE_RADIANCE, &M->EmissionColorTexture}};
        for (const slot& S : Slots) {
            if (S.name->empty()) { *S.dst = nullptr; continue; }
            if (!TextureMap.count(*S.name)) {
                std::string P = Options.DirectoryPath + "/" + *S.name;
                TextureMap[*S.name] = LoadTexture(Scene, P.c_str(), S.type, S.name->c_str(), nullptr);
            }
            *S.dst = TextureMap[*S.name];
        }
        if (Options.OpenPBRAsDiffuse) M->EmissionColorTexture = nullptr;
        Materials.push_back(M);
    }

    std::string ModelName = Options.Name.empty() ? Stem(Path) : Options.Name;

    // Shape / material pairs (scene.cpp:742-776).  std::unordered_set<int>
    // iteration order is the standard library's, as in the reference build.
    std::vector<std::pair<size_t, int>> ShapeMaterialPairs;
    std::vector<vec3> Origins;
    for (size_t ShapeIndex = 0; ShapeIndex < Obj.shapes.size(); ShapeIndex++) {
        const obj_shape& Shape = Obj.shapes[ShapeIndex];
        size_t FaceCount = Shape.indices.size() / 3;
        if (FaceCount == 0) continue;
        vec3 Minimum(+INF), Maximum(-INF);
        for (size_t I = 0; I < 3 * FaceCount; I++) {
            int vi = Shape.indices[I].vertex_index;
            vec3 P(Obj.vertices[3 * vi], Obj.vertices[3 * vi + 1], Obj.vertices[3 * vi + 2]);
            Minimum = vmin(Minimum, P);
            Maximum = vmax(Maximum, P);
        }
        Origins.push_back(0.5f * (Minimum + Maximum));
        std::unordered_set<int> MaterialIndices;
        for (size_t I = 0; I < FaceCount; I++) MaterialIndices.insert(Shape.material_ids[I]);
        for (int MaterialIndex : MaterialIndices) ShapeMaterialPairs.push_back({ShapeIndex, MaterialIndex});
    }

    // Meshes (scene.cpp:778-849).  Origins is indexed by ShapeIndex here and
    // by mesh index below, exactly as the reference does; the two agree when
    // every shape has faces and a single material.
    std::vector<mesh*> Meshes;
    std::vector<material*> MeshMaterials;
    for (auto [ShapeIndex, MaterialIndex] : ShapeMaterialPairs) {
        const obj_shape& Shape = Obj.shapes[ShapeIndex];
        size_t ShapeFaceCount = Shape.indices.size() / 3;
        MeshMaterials.push_back(MaterialIndex >= 0 ? Materials[MaterialIndex] : nullptr);
        vec3 Origin = ShapeIndex < Origins.size() ? Origins[ShapeIndex] : vec3(0.0f);
        mesh* Mesh = new mesh;
        Mesh->Name = !Shape.name.empty() ? Shape.name : ModelName + " " + std::to_string(ShapeIndex);
        std::unordered_map<vertex_key, uint32_t, vertex_hash> VertexIndexMap;
        for (size_t I = 0; I < ShapeFaceCount; I++) {
            if (Shape.material_ids[I] != MaterialIndex) continue;
            mesh_face Face;
            for (size_t J = 0; J < 3; J++) {
                const obj_index& Index = Shape.indices[3 * I + J];
                mesh_vertex Vertex{};
                int vi = Index.vertex_index;
                vec4 P = Options.VertexTransform * vec4(Obj.vertices[3 * vi + 0] - Origin.x,
                                                         Obj.vertices[3 * vi + 1] - Origin.y,
                                                         Obj.vertices[3 * vi + 2] - Origin.z, 1.0f);
                Vertex.Position = vec3(P.x, P.y, P.z);
                if (Index.normal_index >= 0) {
                    int ni = Index.normal_index;
                    vec4 N = Options.NormalTransform *
                             vec4(Obj.normals[3 * ni + 0], Obj.normals[3 * ni + 1], Obj.normals[3 * ni + 2], 0.0f);
                    Vertex.Normal = vec3(N.x, N.y, N.z);
                }
                if (Index.texcoord_index >= 0) {
                    int ti = Index.texcoord_index;
                    vec3 T = Mul3(Options.TextureCoordinateTransform,
                                  vec3(Obj.texcoords[2 * ti + 0], Obj.texcoords[2 * ti + 1], 1.0f));
                    Vertex.UV = vec2(T.x, T.y);
                }
                vertex_key K{Vertex};
                auto It = VertexIndexMap.find(K);
                if (It == VertexIndexMap.end()) {
                    It = VertexIndexMap.emplace(K, (uint32_t)Mesh->Vertices.size()).first;
                    Mesh->Vertices.push_back(Vertex);
                }
                Face.VertexIndex[J] = It->second;
            }
            Mesh->Faces.push_back(Face);
        }
        Meshes.push_back(Mesh);
    }

    for (mesh* Mesh : Meshes) {                    // scene.cpp:851-866
        BuildMeshBVH(Mesh);
        Scene->Meshes.push_back(Mesh);
    }
    Scene->DirtyFlags |= PT_SCENE_DIRTY_MATERIALS | PT_SCENE_DIRTY_MESHES;

    // Prefab entity tree (scene.cpp:868-900).
    prefab* Prefab = new prefab;
    auto NewEntity = [&](entity_type Type) {
        entity* E = new entity;
        E->Type = Type;
        Prefab->Owned.push_back(E);
        return E;
    };
    if (Meshes.size() == 1) {
        entity* Instance = NewEntity(ENTITY_TYPE_MESH_INSTANCE);
        Instance->Name = Meshes[0]->Name;
        Instance->Mesh = Meshes[0];
        Instance->Material = MeshMaterials[0];
        Prefab->Entity = Instance;
    } else {
        entity* Container = NewEntity(ENTITY_TYPE_CONTAINER);
        Container->Name = ModelName;
        for (size_t I = 0; I < Meshes.size(); I++) {
            entity* Instance = NewEntity(ENTITY_TYPE_MESH_INSTANCE);
            Instance->Name = Meshes[I]->Name;
            Instance->Mesh = Meshes[I];
            Instance->Material = MeshMaterials[I];
            vec3 O = I < Origins.size() ? Origins[I] : vec3(0.0f);
            vec4 P = Options.VertexTransform * vec4(O, 1.0f);
            Instance->Transform.Position = vec3(P.x, P.y, P.z);
            Instance->Parent = Container;
            Container->Children.push_back(Instance);
        }
        Prefab->Entity = Container;
    }
    Scene->Prefabs.push_back(Prefab);
    return Prefab;
}

// CreateEntity(Scene, Source, Parent) (scene.cpp:205-249): deep copy.
entity* CreateEntity(scene* Scene, const entity* Source, entity* Parent)
{
    entity* E = new entity(*Source);
    E->Children.clear();
    if (!Parent) Parent = &Scene->Root;
    E->Parent = Parent;
    E->PackedShapeIndex = PT_SHAPE_INDEX_NONE;
    Parent->Children.push_back(E);
    Scene->Entities.push_back(E);
    for (const entity* Child : Source->Children) CreateEntity(Scene, Child, E);
    Scene->DirtyFlags |= PT_SCENE_DIRTY_SHAPES | PT_SCENE_DIRTY_CAMERAS;
    return E;
}

entity* CreateEntity(scene* Scene, const prefab* Prefab, entity* Parent)
{
    return CreateEntity(Scene, Prefab->Entity, Parent);
}

}  // namespace pth
