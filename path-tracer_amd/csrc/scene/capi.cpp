// capi.cpp — C ABI of libptscene.so (include/pt_scene.h) over the C++ scene
// restatement.  Handles are the C++ objects themselves.
#include "scene.hpp"
#include "configs.hpp"
#include "image.hpp"
#include "../../../include/pt_scene.h"

#include <cstring>
#include <exception>
#include <new>
#include <string>
#include <vector>

using namespace pth;

namespace {
thread_local std::string g_err;
scene* S(pts_scene* s) { return reinterpret_cast<scene*>(s); }
entity* E(pts_entity* e) { return reinterpret_cast<entity*>(e); }
material* M(pts_material* m) { return reinterpret_cast<material*>(m); }
texture* T(pts_texture* t) { return reinterpret_cast<texture*>(t); }
mesh* Me(pts_mesh* m) { return reinterpret_cast<mesh*>(m); }

// No exception crosses the C ABI: an entry point that parses files or
// allocates from caller-given sizes runs under Guard, which turns
// std::bad_alloc (or any other exception) into the error return.
template <class R, class F>
R Guard(R fail, const char* what, F&& f)
{
    try {
        return f();
    } catch (const std::bad_alloc&) {
        g_err = std::string(what) + ": out of memory";
    } catch (const std::exception& e) {
        g_err = std::string(what) + ": " + e.what();
    } catch (...) {
        g_err = std::string(what) + ": unknown exception";
    }
    return fail;
}
}  // namespace

extern "C" {

const char* ptsGetLastError(void) { return g_err.c_str(); }

pts_scene* ptsCreateScene(void) { return reinterpret_cast<pts_scene*>(CreateScene()); }
pts_scene* ptsCreateEmptyScene(void) { return reinterpret_cast<pts_scene*>(CreateEmptyScene()); }

pts_scene* ptsCreateConfigScene(int config, pts_config_info* info)
{
    config_info I{};
    scene* s = CreateConfigScene(config, &I);
    if (!s) { g_err = "unknown config " + std::to_string(config); return nullptr; }
    if (info) {
        info->width = I.width; info->height = I.height; info->spp = I.spp; info->camera_count = I.camera_count;
        info->render_flags = I.render_flags; info->termination_probability = I.termination_probability;
        info->mesh_face_count = I.mesh_face_count; info->shape_count = I.shape_count;
    }
    return reinterpret_cast<pts_scene*>(s);
}

void ptsDestroyScene(pts_scene* s) { if (s) DestroyScene(S(s)); }

pts_entity* ptsSceneRoot(pts_scene* s) { return reinterpret_cast<pts_entity*>(&S(s)->Root); }

pts_entity* ptsCreateEntity(pts_scene* s, int type, pts_entity* parent)
{
    if (type <= ENTITY_TYPE_ROOT || type > ENTITY_TYPE_CUBE) { g_err = "bad entity type"; return nullptr; }
    return reinterpret_cast<pts_entity*>(CreateEntity(S(s), (entity_type)type, parent ? E(parent) : nullptr));
}

void ptsSetEntityTransform(pts_scene* s, pts_entity* e, const float p[3], const float r[3], const float sc[3])
{
    if (p) E(e)->Transform.Position = vec3(p[0], p[1], p[2]);
    if (r) E(e)->Transform.Rotation = vec3(r[0], r[1], r[2]);
    if (sc) E(e)->Transform.Scale = vec3(sc[0], sc[1], sc[2]);
    S(s)->DirtyFlags |= PT_SCENE_DIRTY_SHAPES | PT_SCENE_DIRTY_CAMERAS;
}

void ptsSetEntityActive(pts_scene* s, pts_entity* e, int active)
{
    E(e)->Active = active != 0;
    S(s)->DirtyFlags |= PT_SCENE_DIRTY_SHAPES | PT_SCENE_DIRTY_CAMERAS;
}

void ptsSetEntityMaterial(pts_scene* s, pts_entity* e, pts_material* m)
{
    E(e)->Material = m ? M(m) : nullptr;
    S(s)->DirtyFlags |= PT_SCENE_DIRTY_SHAPES;
}

void ptsSetEntityMesh(pts_scene* s, pts_entity* e, pts_mesh* m)
{
    E(e)->Mesh = m ? Me(m) : nullptr;
    S(s)->DirtyFlags |= PT_SCENE_DIRTY_SHAPES;
}

uint32_t ptsEntityPackedShapeIndex(pts_entity* e) { return E(e)->PackedShapeIndex; }

void ptsSetCameraPinhole(pts_scene* s, pts_entity* c, float fov, float aperture)
{
    E(c)->CameraModel = PT_CAMERA_MODEL_PINHOLE;
    E(c)->PinholeFieldOfViewInDegrees = fov;
    E(c)->PinholeApertureDiameterInMM = aperture;
    S(s)->DirtyFlags |= PT_SCENE_DIRTY_CAMERAS;
}

void ptsSetCameraThinLens(pts_scene* s, pts_entity* c, float sw, float sh, float f, float a, float focus)
{
    E(c)->CameraModel = PT_CAMERA_MODEL_THIN_LENS;
    E(c)->ThinLensSensorSizeInMM = vec2(sw, sh);
    E(c)->ThinLensFocalLengthInMM = f;
    E(c)->ThinLensApertureDiameterInMM = a;
    E(c)->ThinLensFocusDistance = focus;
    S(s)->DirtyFlags |= PT_SCENE_DIRTY_CAMERAS;
}

void ptsSetCamera360(pts_scene* s, pts_entity* c)
{
    E(c)->CameraModel = PT_CAMERA_MODEL_360;
    S(s)->DirtyFlags |= PT_SCENE_DIRTY_CAMERAS;
}

void ptsSetRootParameters(pts_scene* s, float scatter, float brightness, float sampling, pts_texture* sky)
{
    entity& R = S(s)->Root;
    R.ScatterRate = scatter;
    R.SkyboxBrightness = brightness;
    R.SkyboxSamplingProbability = sampling;
    R.SkyboxTexture = sky ? T(sky) : nullptr;
    S(s)->DirtyFlags |= PT_SCENE_DIRTY_GLOBALS | PT_SCENE_DIRTY_SKYBOX_TEXTURE;
}

pts_material* ptsCreateMaterial(pts_scene* s, int type, const char* name)
{
    if (type < 0 || type > PT_MATERIAL_TYPE_OPENPBR) { g_err = "bad material type"; return nullptr; }
    return reinterpret_cast<pts_material*>(CreateMaterial(S(s), (uint32_t)type, name));
}

int ptsSetMaterialParameter(pts_scene* s, pts_material* mp, const char* name, const float* v, int n)
{
    material* m = M(mp);
    auto vec = [&](vec3& dst) { if (n != 3) return -1; dst = vec3(v[0], v[1], v[2]); return 0; };
    auto flt = [&](float& dst) { if (n != 1) return -1; dst = v[0]; return 0; };
    std::string k = name ? name : "";
    int rc;
    if (k == "BaseColor") rc = vec(m->BaseColor);
    else if (k == "SpecularColor") rc = vec(m->SpecularColor);
    else if (k == "TransmissionColor") rc = vec(m->TransmissionColor);
    else if (k == "ScatteringColor") rc = vec(m->ScatteringColor);
    else if (k == "Roughness") rc = flt(m->Roughness);
    else if (k == "RoughnessAnisotropy") rc = flt(m->RoughnessAnisotropy);
    else if (k == "IOR") rc = flt(m->IOR);
    else if (k == "AbbeNumber") rc = flt(m->AbbeNumber);
    else if (k == "TransmissionDepth") rc = flt(m->TransmissionDepth);
    else if (k == "ScatteringAnisotropy") rc = flt(m->ScatteringAnisotropy);
    // OpenPBR (openpbr.hpp:5-37); its SpecularRoughness is "Roughness" above
    else if (k == "BaseWeight") rc = flt(m->BaseWeight);
    else if (k == "BaseMetalness") rc = flt(m->BaseMetalness);
    else if (k == "BaseDiffuseRoughness") rc = flt(m->BaseDiffuseRoughness);
    else if (k == "SpecularWeight") rc = flt(m->SpecularWeight);
    else if (k == "SpecularIOR") rc = flt(m->SpecularIOR);
    else if (k == "TransmissionWeight") rc = flt(m->TransmissionWeight);
    else if (k == "TransmissionScatter") rc = vec(m->TransmissionScatter);
    else if (k == "TransmissionScatterAnisotropy") rc = flt(m->TransmissionScatterAnisotropy);
    else if (k == "TransmissionDispersionScale") rc = flt(m->TransmissionDispersionScale);
    else if (k == "TransmissionDispersionAbbeNumber") rc = flt(m->TransmissionDispersionAbbeNumber);
    else if (k == "CoatWeight") rc = flt(m->CoatWeight);
    else if (k == "CoatColor") rc = vec(m->CoatColor);
    else if (k == "CoatRoughness") rc = flt(m->CoatRoughness);
    else if (k == "CoatRoughnessAnisotropy") rc = flt(m->CoatRoughnessAnisotropy);
    else if (k == "CoatIOR") rc = flt(m->CoatIOR);
    else if (k == "CoatDarkening") rc = flt(m->CoatDarkening);
    else if (k == "EmissionLuminance") rc = flt(m->EmissionLuminance);
    else if (k == "EmissionColor") rc = vec(m->EmissionColor);
    else if (k == "LayerBounceLimit") {
        rc = n == 1 && v[0] >= 0.0f && v[0] <= 1024.0f && v[0] == (float)(int)v[0] ? 0 : -1;
        if (rc == 0) m->LayerBounceLimit = (int)v[0];
    }
    else { g_err = "unknown material parameter " + k; return -1; }
    if (rc) { g_err = "wrong value count for " + k; return -1; }
    S(s)->DirtyFlags |= PT_SCENE_DIRTY_MATERIALS;
    return 0;
}

int ptsSetMaterialTexture(pts_scene* s, pts_material* mp, const char* name, pts_texture* t)
{
    material* m = M(mp);
    std::string k = name ? name : "";
    texture* tx = t ? T(t) : nullptr;
    if (k == "BaseTexture") m->BaseTexture = tx;
    else if (k == "SpecularTexture") m->SpecularTexture = tx;
    else if (k == "RoughnessTexture") m->RoughnessTexture = tx;
    else if (k == "RoughnessAnisotropyTexture") m->RoughnessAnisotropyTexture = tx;
    else if (k == "EmissionColorTexture") m->EmissionColorTexture = tx;
    else { g_err = "unknown material texture " + k; return -1; }
    S(s)->DirtyFlags |= PT_SCENE_DIRTY_MATERIALS;
    return 0;
}

uint32_t ptsMaterialPackedIndex(pts_material* m) { return M(m)->PackedMaterialIndex; }

pts_texture* ptsCreateCheckerTexture(pts_scene* s, const char* name, int type, const float a[4], const float b[4])
{
    return reinterpret_cast<pts_texture*>(
        CreateCheckerTexture(S(s), name ? name : "Checker", (uint32_t)type, vec4(a[0], a[1], a[2], a[3]), vec4(b[0], b[1], b[2], b[3])));
}

pts_texture* ptsCreateTexture(pts_scene* s, const char* name, int type, uint32_t w, uint32_t h, const float* rgba, int nearest)
{
    if (!rgba || w == 0 || h == 0) { g_err = "bad texture"; return nullptr; }
    return Guard<pts_texture*>(nullptr, "CreateTexture", [&] {
        texture* t = CreateTexture(S(s), name, (uint32_t)type, w, h, rgba);
        t->EnableNearestFiltering = nearest != 0;
        return reinterpret_cast<pts_texture*>(t);
    });
}

pts_mesh* ptsCreateMesh(pts_scene* s, const char* name, uint32_t nv, const float* pos, const float* nrm, const float* uv,
                        uint32_t nf, const uint32_t* idx)
{
    if (!pos || !idx || nv == 0 || nf == 0) { g_err = "bad mesh"; return nullptr; }
    for (uint32_t i = 0; i < 3 * nf; i++)
        if (idx[i] >= nv) { g_err = "mesh index out of range"; return nullptr; }
    return Guard<pts_mesh*>(nullptr, "CreateMesh", [&] {
        return reinterpret_cast<pts_mesh*>(CreateMesh(S(s), name, nv, pos, nrm, uv, nf, idx));
    });
}

uint32_t ptsMeshDepth(pts_mesh* m) { return Me(m)->Depth; }
uint32_t ptsMeshNodeCount(pts_mesh* m) { return (uint32_t)Me(m)->Nodes.size(); }
void ptsMeshFaces(pts_mesh* m, uint32_t* out)
{
    for (size_t f = 0; f < Me(m)->Faces.size(); f++)
        for (int j = 0; j < 3; j++) out[3 * f + j] = Me(m)->Faces[f].VertexIndex[j];
}

void ptsDefaultLoadModelOptions(pts_load_model_options* o)
{
    std::memset(o, 0, sizeof(*o));
    for (int i = 0; i < 4; i++) { o->vertex_transform[5 * i] = 1; o->normal_transform[5 * i] = 1; }
    for (int i = 0; i < 3; i++) o->texcoord_transform[4 * i] = 1;
}

int ptsLoadImageRGBA8(const char* path, uint32_t* w, uint32_t* h, uint8_t* rgba)
{
    return Guard(-1, "LoadImage", [&] {
        int W = 0, H = 0;
        std::vector<uint8_t> px;
        std::string err;
        if (!path || !LoadImageRGBA8(path, W, H, px, err)) { g_err = err.empty() ? "bad path" : err; return -1; }
        if (w) *w = (uint32_t)W;
        if (h) *h = (uint32_t)H;
        if (rgba) std::memcpy(rgba, px.data(), px.size());
        return 0;
    });
}

pts_texture* ptsLoadTexture(pts_scene* s, const char* path, int type, const char* name)
{
    return Guard<pts_texture*>(nullptr, "LoadTexture", [&] {
        std::string err;
        texture* t = LoadTexture(S(s), path, (uint32_t)type, name, &err);
        if (!t) g_err = "LoadTexture: " + err;
        return reinterpret_cast<pts_texture*>(t);
    });
}

pts_prefab* ptsLoadModelAsPrefab(pts_scene* s, const char* path, const pts_load_model_options* o)
{
    load_model_options opt;
    if (o) {
        if (o->name) opt.Name = o->name;
        if (o->directory_path) opt.DirectoryPath = o->directory_path;
        for (int c = 0; c < 4; c++)
            for (int r = 0; r < 4; r++) {
                opt.VertexTransform[c][r] = o->vertex_transform[4 * c + r];
                opt.NormalTransform[c][r] = o->normal_transform[4 * c + r];
            }
        for (int i = 0; i < 9; i++) opt.TextureCoordinateTransform[i] = o->texcoord_transform[i];
        opt.OpenPBRAsDiffuse = o->openpbr_as_diffuse != 0;
    }
    return Guard<pts_prefab*>(nullptr, "LoadModelAsPrefab", [&] {
        std::string err;
        prefab* p = LoadModelAsPrefab(S(s), path, &opt, &err);
        if (!p) g_err = "LoadModelAsPrefab: " + err;
        return reinterpret_cast<pts_prefab*>(p);
    });
}

pts_scene* ptsLoadScene(const char* path)
{
    if (!path) { g_err = "LoadScene: null path"; return nullptr; }
    return Guard<pts_scene*>(nullptr, "LoadScene", [&] {
        std::string err;
        scene* sc = LoadScene(path, &err);
        if (!sc) g_err = "LoadScene: " + err;
        return reinterpret_cast<pts_scene*>(sc);
    });
}

int ptsSaveScene(pts_scene* s, const char* path)
{
    if (!s || !path) { g_err = "SaveScene: null argument"; return -1; }
    return Guard(-1, "SaveScene", [&] {
        std::string err;
        if (!SaveScene(path, S(s), &err)) { g_err = "SaveScene: " + err; return -1; }
        return 0;
    });
}

uint32_t ptsSceneTextureCount(pts_scene* s) { return s ? (uint32_t)S(s)->Textures.size() : 0; }
uint32_t ptsSceneMaterialCount(pts_scene* s) { return s ? (uint32_t)S(s)->Materials.size() : 0; }
uint32_t ptsSceneMeshCount(pts_scene* s) { return s ? (uint32_t)S(s)->Meshes.size() : 0; }
uint32_t ptsScenePrefabCount(pts_scene* s) { return s ? (uint32_t)S(s)->Prefabs.size() : 0; }

pts_entity* ptsInstantiatePrefab(pts_scene* s, pts_prefab* p, pts_entity* parent)
{
    return reinterpret_cast<pts_entity*>(
        CreateEntity(S(s), reinterpret_cast<prefab*>(p), reinterpret_cast<entity*>(parent)));
}

static void CollectMeshes(entity* e, std::vector<entity*>& out)
{
    if (e->Type == ENTITY_TYPE_MESH_INSTANCE) out.push_back(e);
    for (entity* c : e->Children) CollectMeshes(c, out);
}

uint32_t ptsPrefabMeshCount(pts_prefab* p)
{
    std::vector<entity*> m;
    CollectMeshes(reinterpret_cast<prefab*>(p)->Entity, m);
    return (uint32_t)m.size();
}

pts_mesh* ptsPrefabMesh(pts_prefab* p, uint32_t index, pts_material** material, float position[3])
{
    std::vector<entity*> m;
    CollectMeshes(reinterpret_cast<prefab*>(p)->Entity, m);
    if (index >= m.size()) return nullptr;
    if (material) *material = reinterpret_cast<pts_material*>(m[index]->Material);
    if (position) {
        position[0] = m[index]->Transform.Position.x;
        position[1] = m[index]->Transform.Position.y;
        position[2] = m[index]->Transform.Position.z;
    }
    return reinterpret_cast<pts_mesh*>(m[index]->Mesh);
}

uint32_t ptsMeshVertexCount(pts_mesh* m) { return (uint32_t)Me(m)->Vertices.size(); }
uint32_t ptsMeshFaceCount(pts_mesh* m) { return (uint32_t)Me(m)->Faces.size(); }

void ptsMeshVertices(pts_mesh* m, float* out)
{
    for (size_t i = 0; i < Me(m)->Vertices.size(); i++) {
        const mesh_vertex& v = Me(m)->Vertices[i];
        float* o = out + 8 * i;
        o[0] = v.Position.x; o[1] = v.Position.y; o[2] = v.Position.z;
        o[3] = v.Normal.x; o[4] = v.Normal.y; o[5] = v.Normal.z;
        o[6] = v.UV.x; o[7] = v.UV.y;
    }
}

int ptsMaterialType(pts_material* m) { return m ? (int)reinterpret_cast<material*>(m)->Type : -1; }

static entity* FindCamera(entity* e, uint32_t index)
{
    if (e->Type == ENTITY_TYPE_CAMERA && e->PackedCameraIndex == index) return e;
    for (entity* c : e->Children)
        if (entity* f = FindCamera(c, index)) return f;
    return nullptr;
}

pts_entity* ptsFindCamera(pts_scene* s, uint32_t packed_index)
{
    entity* e = FindCamera(&S(s)->Root, packed_index);
    if (!e) g_err = "no camera with packed index " + std::to_string(packed_index);
    return reinterpret_cast<pts_entity*>(e);
}

void ptsSetCameraTransform(pts_scene* s, pts_entity* c, const float p[3], const float r[3])
{
    if (p) E(c)->Transform.Position = vec3(p[0], p[1], p[2]);
    if (r) E(c)->Transform.Rotation = vec3(r[0], r[1], r[2]);
    S(s)->DirtyFlags |= PT_SCENE_DIRTY_CAMERAS;
}

uint32_t ptsPackSceneData(pts_scene* s) { return PackSceneData(S(s)); }
void ptsGetScenePacks(pts_scene* s, pt_scene_packs* out) { GetScenePacks(S(s), out); }
void ptsMarkDirty(pts_scene* s, uint32_t flags) { S(s)->DirtyFlags |= flags; }

int ptsGetParametricSpectrumCoefficients(const float rgb[3], float beta[3])
{
    vec3 b = GetParametricSpectrumCoefficients(GetSharedSpectrumTable(), vec3(rgb[0], rgb[1], rgb[2]));
    beta[0] = b.x; beta[1] = b.y; beta[2] = b.z;
    return 0;
}

int ptsBuildSpectrumTable(int threads)
{
    BuildParametricSpectrumTableForSRGB(GetSharedSpectrumTable(), threads);
    return 0;
}

int ptsSaveSpectrumTable(const char* path)
{
    return SaveParametricSpectrumTable(GetSharedSpectrumTable(), path) ? 0 : -1;
}

int ptsLoadSpectrumTable(const char* path)
{
    return LoadParametricSpectrumTable(GetSharedSpectrumTable(), path) ? 0 : -1;
}

void ptsSetSpectrumTablePath(const char* path) { SetSpectrumTablePath(path ? path : ""); }

}  // extern "C"
