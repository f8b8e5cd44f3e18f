// configs.cpp — the benchmark scenes of BASELINE.json / SURVEY.md §8(d),
// built through the restated scene API exactly as the reference application
// would build them (CreateScene, CreateEntity, CreateMaterial, ...).
//
// The Viking Room OBJ and its texture are not available in this environment
// (SURVEY.md §8(c) "Assets"), so C3/C4/C5 use a deterministic synthetic room
// mesh of 3,976 triangles (two log walls, a plank floor, barrels, a chest, a
// table, a bed and a pot) with a procedural 1024x1024 texture; C2's HDR sky
// is procedural as well.  Every input is a pure function of this file.
#include "scene.hpp"
#include "configs.hpp"

#include <cmath>

namespace pth {

namespace {

uint32_t Hash(uint32_t x)   // PCG output hash for deterministic texture noise
{
    uint32_t s = x * 747796405u + 2891336453u;
    uint32_t w = ((s >> ((s >> 28u) + 4u)) ^ s) * 277803737u;
    return (w >> 22u) ^ w;
}
float Noise(uint32_t x, uint32_t y, uint32_t salt) { return (Hash(x * 73856093u ^ y * 19349663u ^ salt) & 0xFFFFFF) / 16777216.0f; }

struct mesh_builder {
    std::vector<float> P, N, UV;
    std::vector<uint32_t> I;

    uint32_t Vertex(vec3 p, vec3 n, vec2 uv)
    {
        P.insert(P.end(), {p.x, p.y, p.z});
        N.insert(N.end(), {n.x, n.y, n.z});
        UV.insert(UV.end(), {uv.x, uv.y});
        return (uint32_t)(P.size() / 3 - 1);
    }
    void Tri(uint32_t a, uint32_t b, uint32_t c) { I.insert(I.end(), {a, b, c}); }

    // Grid quad: origin + u*U + v*V, nu x nv cells, UVs in [uv0, uv1].
    void Grid(vec3 O, vec3 U, vec3 V, int nu, int nv, vec2 uv0, vec2 uv1, float bump = 0.0f, uint32_t salt = 0)
    {
        vec3 Nn = normalize(cross(U, V));
        uint32_t base = (uint32_t)(P.size() / 3);
        for (int j = 0; j <= nv; j++)
            for (int i = 0; i <= nu; i++) {
                float s = i / float(nu), t = j / float(nv);
                float h = 0.0f;
                if (bump != 0.0f && i > 0 && j > 0 && i < nu && j < nv) h = bump * (Noise(i, j, salt) - 0.5f);
                vec3 p = O + U * s + V * t + Nn * h;
                Vertex(p, Nn, vec2(uv0.x + (uv1.x - uv0.x) * s, uv0.y + (uv1.y - uv0.y) * t));
            }
        for (int j = 0; j < nv; j++)
            for (int i = 0; i < nu; i++) {
                uint32_t a = base + j * (nu + 1) + i, b = a + 1, c = a + (nu + 1), d = c + 1;
                Tri(a, b, d);
                Tri(a, d, c);
            }
    }

    // Axis-aligned box, each face split into n x n cells.
    void Box(vec3 c, vec3 h, int n, vec2 uv0, vec2 uv1)
    {
        vec3 X(h.x, 0, 0), Y(0, h.y, 0), Z(0, 0, h.z);
        Grid(c - X - Y - Z, Y * 2, X * 2, n, n, uv0, uv1);   // bottom (-z)
        Grid(c - X - Y + Z, X * 2, Y * 2, n, n, uv0, uv1);   // top (+z)
        Grid(c - X - Y - Z, X * 2, Z * 2, n, n, uv0, uv1);   // front (-y)
        Grid(c - X + Y - Z, Z * 2, X * 2, n, n, uv0, uv1);   // back (+y)
        Grid(c - X - Y - Z, Z * 2, Y * 2, n, n, uv0, uv1);   // left (-x)
        Grid(c + X - Y - Z, Y * 2, Z * 2, n, n, uv0, uv1);   // right (+x)
    }

    // Capped cylinder along +z (smooth side normals).
    void Cylinder(vec3 base, float r, float h, int seg, int rings, vec2 uv0, vec2 uv1)
    {
        uint32_t b0 = (uint32_t)(P.size() / 3);
        for (int j = 0; j <= rings; j++)
            for (int i = 0; i <= seg; i++) {
                float a = TAU * i / seg;
                float bulge = 1.0f + 0.12f * std::sin(PI * j / rings);   // barrel profile
                vec3 n(std::cos(a), std::sin(a), 0);
                vec3 p = base + vec3(n.x * r * bulge, n.y * r * bulge, h * j / rings);
                Vertex(p, n, vec2(uv0.x + (uv1.x - uv0.x) * i / seg, uv0.y + (uv1.y - uv0.y) * j / rings));
            }
        for (int j = 0; j < rings; j++)
            for (int i = 0; i < seg; i++) {
                uint32_t a = b0 + j * (seg + 1) + i, b = a + 1, c = a + (seg + 1), d = c + 1;
                Tri(a, b, d);
                Tri(a, d, c);
            }
        for (int cap = 0; cap < 2; cap++) {
            float z = cap ? h : 0.0f;
            vec3 n(0, 0, cap ? 1.0f : -1.0f);
            uint32_t center = Vertex(base + vec3(0, 0, z), n, vec2((uv0.x + uv1.x) / 2, (uv0.y + uv1.y) / 2));
            uint32_t ring0 = (uint32_t)(P.size() / 3);
            for (int i = 0; i <= seg; i++) {
                float a = TAU * i / seg;
                Vertex(base + vec3(std::cos(a) * r, std::sin(a) * r, z), n,
                       vec2(uv0.x + (uv1.x - uv0.x) * 0.5f * (1 + std::cos(a)), uv0.y + (uv1.y - uv0.y) * 0.5f * (1 + std::sin(a))));
            }
            for (int i = 0; i < seg; i++) {
                if (cap) Tri(center, ring0 + i, ring0 + i + 1);
                else Tri(center, ring0 + i + 1, ring0 + i);
            }
        }
    }

    // UV sphere (smooth normals).
    void Sphere(vec3 c, float r, int seg, int rings, vec2 uv0, vec2 uv1)
    {
        uint32_t b0 = (uint32_t)(P.size() / 3);
        for (int j = 0; j <= rings; j++)
            for (int i = 0; i <= seg; i++) {
                float th = PI * j / rings, ph = TAU * i / seg;
                vec3 n(std::sin(th) * std::cos(ph), std::sin(th) * std::sin(ph), -std::cos(th));
                Vertex(c + n * r, n, vec2(uv0.x + (uv1.x - uv0.x) * i / seg, uv0.y + (uv1.y - uv0.y) * j / rings));
            }
        for (int j = 0; j < rings; j++)
            for (int i = 0; i < seg; i++) {
                uint32_t a = b0 + j * (seg + 1) + i, b = a + 1, cc = a + (seg + 1), d = cc + 1;
                Tri(a, b, d);
                Tri(a, d, cc);
            }
    }
};

// Synthetic stand-in for the Viking Room: a room corner (walls at x = -1 and
// y = +1, floor z = 0, open towards -x/+y's opposite sides and the sky).
mesh* BuildRoomMesh(scene* Scene)
{
    mesh_builder B;
    B.Grid(vec3(-1, -1, 0), vec3(2, 0, 0), vec3(0, 2, 0), 20, 20, vec2(0.0f, 0.0f), vec2(0.5f, 0.5f), 0.004f, 1);     // floor
    B.Grid(vec3(-1, -1, 0), vec3(0, 2, 0), vec3(0, 0, 1.4f), 20, 14, vec2(0.5f, 0.0f), vec2(1.0f, 0.35f), 0.01f, 2);  // wall x=-1
    B.Grid(vec3(-1, 1, 0), vec3(0, 0, 1.4f), vec3(2, 0, 0), 14, 20, vec2(0.5f, 0.35f), vec2(1.0f, 0.7f), 0.01f, 3);   // wall y=+1
    B.Cylinder(vec3(-0.62f, 0.6f, 0), 0.18f, 0.45f, 32, 6, vec2(0.0f, 0.5f), vec2(0.25f, 0.75f));                     // barrels
    B.Cylinder(vec3(-0.22f, 0.78f, 0), 0.14f, 0.35f, 32, 6, vec2(0.0f, 0.5f), vec2(0.25f, 0.75f));
    B.Box(vec3(0.45f, 0.72f, 0.16f), vec3(0.28f, 0.16f, 0.16f), 4, vec2(0.25f, 0.5f), vec2(0.5f, 0.75f));            // chest
    B.Box(vec3(0.1f, -0.2f, 0.42f), vec3(0.3f, 0.2f, 0.025f), 1, vec2(0.25f, 0.75f), vec2(0.5f, 1.0f));              // table
    const float lx[2] = {-0.17f, 0.37f}, ly[2] = {-0.37f, -0.03f};
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 2; j++)
            B.Box(vec3(lx[i], ly[j], 0.2f), vec3(0.025f, 0.025f, 0.2f), 1, vec2(0.25f, 0.75f), vec2(0.5f, 1.0f));
    B.Grid(vec3(-0.95f, -0.6f, 0.28f), vec3(0.55f, 0, 0), vec3(0, 1.0f, 0), 16, 16, vec2(0.5f, 0.7f), vec2(1.0f, 1.0f), 0.06f, 4);  // bed
    B.Sphere(vec3(0.1f, -0.15f, 0.55f), 0.08f, 16, 12, vec2(0.0f, 0.75f), vec2(0.25f, 1.0f));                          // pot
    B.Box(vec3(-0.93f, 0.1f, 0.95f), vec3(0.07f, 0.45f, 0.02f), 1, vec2(0.25f, 0.75f), vec2(0.5f, 1.0f));             // shelf
    return CreateMesh(Scene, "SyntheticRoom", (uint32_t)(B.P.size() / 3), B.P.data(), B.N.data(), B.UV.data(),
                      (uint32_t)(B.I.size() / 3), B.I.data());
}

// Procedural stand-in for the room texture (sRGB-ish reflectances).
texture* BuildRoomTexture(scene* Scene)
{
    const uint32_t W = 1024, H = 1024;
    std::vector<float> px((size_t)W * H * 4);
    for (uint32_t y = 0; y < H; y++)
        for (uint32_t x = 0; x < W; x++) {
            float u = (x + 0.5f) / W, v = (y + 0.5f) / H;
            float n = Noise(x, y, 11) * 0.08f;
            float r, g, b;
            if (u < 0.5f && v < 0.5f) {            // floor planks
                int plank = (int)(v * 24);
                float t = 0.75f + 0.25f * Noise(plank, 0, 21);
                float grain = 0.04f * std::sin(u * 180.0f + plank);
                r = (0.45f + grain) * t + n; g = (0.30f + grain) * t + n * 0.7f; b = 0.17f * t + n * 0.5f;
            } else if (u >= 0.5f && v < 0.7f) {    // log walls
                float ring = std::fmod(v * 40.0f, 1.0f);
                float shade = 0.6f + 0.4f * std::sin(PI * ring);
                r = 0.52f * shade + n; g = 0.38f * shade + n * 0.6f; b = 0.24f * shade + n * 0.4f;
            } else if (u < 0.25f) {                // barrels and pot
                float band = (std::fmod(v * 16.0f, 1.0f) < 0.12f) ? 0.35f : 1.0f;
                r = 0.55f * band + n; g = 0.35f * band + n; b = 0.2f * band + n;
            } else if (u < 0.5f) {                 // chest / table / shelf
                r = 0.38f + n; g = 0.22f + n * 0.5f; b = 0.12f + n * 0.3f;
            } else {                               // bed cloth
                bool check = ((int)(u * 64) + (int)(v * 64)) & 1;
                r = check ? 0.70f : 0.55f; g = check ? 0.18f : 0.12f; b = check ? 0.15f : 0.10f;
                r += n; g += n * 0.5f; b += n * 0.5f;
            }
            float* p = &px[((size_t)y * W + x) * 4];
            p[0] = std::min(std::max(r, 0.0f), 1.0f);
            p[1] = std::min(std::max(g, 0.0f), 1.0f);
            p[2] = std::min(std::max(b, 0.0f), 1.0f);
            p[3] = 1.0f;
        }
    return CreateTexture(Scene, "SyntheticRoomTexture", PT_TEXTURE_TYPE_REFLECTANCE_WITH_ALPHA, W, H, px.data());
}

// Procedural HDR sky, 512x256 lat-long: horizon-to-zenith gradient, dim
// ground, and a sun lobe of peak intensity 50 around (0.3, 0.4, 0.866).
texture* BuildSkyTexture(scene* Scene)
{
    const uint32_t W = 512, H = 256;
    vec3 Sun = normalize(vec3(0.3f, 0.4f, 0.866f));
    std::vector<float> px((size_t)W * H * 4);
    for (uint32_t y = 0; y < H; y++) {
        float Theta = (0.5f - (y + 0.5f) / H) * PI;
        for (uint32_t x = 0; x < W; x++) {
            float Phi = ((x + 0.5f) / W - 0.5f) * TAU;
            vec3 D(std::cos(Theta) * std::cos(Phi), std::cos(Theta) * std::sin(Phi), std::sin(Theta));
            vec3 C;
            if (Theta > 0) {
                float t = std::sin(Theta);
                C = vec3(0.9f, 0.9f, 1.0f) * (1 - t) + vec3(0.25f, 0.45f, 0.95f) * t;
            } else {
                C = vec3(0.15f, 0.14f, 0.12f);
            }
            float c = dot(D, Sun);
            float lobe = 50.0f * std::exp(-(1.0f - c) / 0.0012f);
            C = C + vec3(1.0f, 0.95f, 0.85f) * lobe;
            float* p = &px[((size_t)y * W + x) * 4];
            p[0] = C.x; p[1] = C.y; p[2] = C.z; p[3] = 1.0f;
        }
    }
    return CreateTexture(Scene, "ProceduralSky", PT_TEXTURE_TYPE_RADIANCE, W, H, px.data());
}

material* Diffuse(scene* S, const char* name, vec3 c)
{
    material* m = CreateMaterial(S, PT_MATERIAL_TYPE_BASIC_DIFFUSE, name);
    m->BaseColor = c;
    return m;
}

entity* Shape(scene* S, entity_type t, vec3 pos, vec3 rot, vec3 scl, material* m)
{
    entity* e = CreateEntity(S, t);
    e->Transform.Position = pos;
    e->Transform.Rotation = rot;
    e->Transform.Scale = scl;
    e->Material = m;
    return e;
}

entity* FirstCamera(scene* S)
{
    for (entity* e : S->Root.Children)
        if (e->Type == ENTITY_TYPE_CAMERA) return e;
    return nullptr;
}

}  // namespace

scene* CreateConfigScene(int config, config_info* info)
{
    config_info I{};
    I.render_flags = PT_RENDER_FLAG_ACCUMULATE_ | PT_RENDER_FLAG_JITTER_;
    I.termination_probability = 0.0f;
    scene* S = nullptr;

    switch (config) {
        case 1: {   // C1: sphere + plane, 256x256 16 spp (SURVEY.md §8(d) "C1 inputs")
            S = CreateScene();
            Shape(S, ENTITY_TYPE_SPHERE, vec3(0, 0, 1), vec3(0, 0, 0), vec3(1, 1, 1), Diffuse(S, "Sphere", vec3(0.8f, 0.3f, 0.3f)));
            entity* cam = FirstCamera(S);
            cam->Transform.Position = vec3(0, -4, 1);
            cam->Transform.Rotation = vec3(PI / 2, 0, 0);
            cam->PinholeFieldOfViewInDegrees = 90.0f;
            I.width = 256; I.height = 256; I.spp = 16; I.camera_count = 1;
            break;
        }
        case 2: {   // C2: open Cornell-style box + three spheres + HDR sky
            S = CreateEmptyScene();
            material* white = Diffuse(S, "White", vec3(0.73f, 0.73f, 0.73f));
            material* red = Diffuse(S, "Red", vec3(0.65f, 0.05f, 0.05f));
            material* green = Diffuse(S, "Green", vec3(0.12f, 0.45f, 0.15f));
            Shape(S, ENTITY_TYPE_CUBE, vec3(0, 0, -0.1f), vec3(0, 0, 0), vec3(3.6f, 3.6f, 0.1f), white);      // floor
            Shape(S, ENTITY_TYPE_CUBE, vec3(0, 3.7f, 3.0f), vec3(0, 0, 0), vec3(3.6f, 0.1f, 3.1f), white);    // back
            Shape(S, ENTITY_TYPE_CUBE, vec3(-3.7f, 0, 3.0f), vec3(0, 0, 0), vec3(0.1f, 3.6f, 3.1f), red);     // left
            Shape(S, ENTITY_TYPE_CUBE, vec3(3.7f, 0, 3.0f), vec3(0, 0, 0), vec3(0.1f, 3.6f, 3.1f), green);    // right
            Shape(S, ENTITY_TYPE_CUBE, vec3(0, 1.8f, 6.1f), vec3(0, 0, 0), vec3(3.6f, 1.8f, 0.1f), white);    // half ceiling
            Shape(S, ENTITY_TYPE_SPHERE, vec3(-2.2f, 0.6f, 1), vec3(0, 0, 0), vec3(1, 1, 1), Diffuse(S, "Blue", vec3(0.2f, 0.3f, 0.8f)));
            material* metal = CreateMaterial(S, PT_MATERIAL_TYPE_BASIC_METAL, "Gold");
            metal->BaseColor = vec3(0.95f, 0.7f, 0.35f);
            metal->SpecularColor = vec3(1, 1, 1);
            metal->Roughness = 0.2f;
            Shape(S, ENTITY_TYPE_SPHERE, vec3(0, 1.6f, 1), vec3(0, 0, 0), vec3(1, 1, 1), metal);
            material* glass = CreateMaterial(S, PT_MATERIAL_TYPE_BASIC_TRANSLUCENT, "Glass");
            glass->IOR = 1.5f;
            glass->AbbeNumber = 20.0f;
            glass->Roughness = 0.0f;
            Shape(S, ENTITY_TYPE_SPHERE, vec3(2.2f, 0.2f, 1), vec3(0, 0, 0), vec3(1, 1, 1), glass);
            entity* cam = CreateEntity(S, ENTITY_TYPE_CAMERA);
            cam->Transform.Position = vec3(0, -10, 3);
            cam->Transform.Rotation = vec3(PI / 2, 0, 0);
            cam->PinholeFieldOfViewInDegrees = 60.0f;
            S->Root.SkyboxTexture = BuildSkyTexture(S);
            S->Root.SkyboxSamplingProbability = 0.5f;
            S->Root.SkyboxBrightness = 1.0f;
            I.width = 1024; I.height = 1024; I.spp = 256; I.camera_count = 1;
            break;
        }
        case 3:
        case 4: {   // C3 / C4: room mesh (Viking Room stand-in), constant sky
            S = CreateEmptyScene();
            material* m = CreateMaterial(S, PT_MATERIAL_TYPE_BASIC_DIFFUSE, "RoomMaterial");
            m->BaseTexture = BuildRoomTexture(S);
            entity* room = CreateEntity(S, ENTITY_TYPE_MESH_INSTANCE);
            room->Mesh = BuildRoomMesh(S);
            room->Material = m;
            entity* cam = CreateEntity(S, ENTITY_TYPE_CAMERA);
            cam->Transform.Position = vec3(0.75f, -0.75f, 0.75f);
            cam->Transform.Rotation = vec3(PI / 2 - 0.35f, 0, PI / 4);
            cam->PinholeFieldOfViewInDegrees = 60.0f;
            I.width = config == 3 ? 1920 : 3840;
            I.height = config == 3 ? 1080 : 2160;
            I.spp = config == 3 ? 1024 : 4096;
            I.camera_count = 1;
            I.mesh_face_count = (uint32_t)room->Mesh->Faces.size();
            break;
        }
        case 5: {   // C5: thin lens + 360 cameras, mixed primitives + mesh
            S = CreateScene();
            material* blue = Diffuse(S, "Diffuse", vec3(0.25f, 0.5f, 0.8f));
            Shape(S, ENTITY_TYPE_SPHERE, vec3(-2.5f, 2.0f, 1), vec3(0, 0, 0), vec3(1, 1, 1), blue);
            material* metal = CreateMaterial(S, PT_MATERIAL_TYPE_BASIC_METAL, "Metal");
            metal->BaseColor = vec3(0.9f, 0.9f, 0.9f);
            metal->Roughness = 0.1f;
            Shape(S, ENTITY_TYPE_SPHERE, vec3(-0.8f, 2.8f, 1), vec3(0, 0, 0), vec3(1, 1, 1), metal);
            material* glass = CreateMaterial(S, PT_MATERIAL_TYPE_BASIC_TRANSLUCENT, "Glass");
            glass->Roughness = 0.0f;
            Shape(S, ENTITY_TYPE_SPHERE, vec3(0.9f, 1.5f, 1), vec3(0, 0, 0), vec3(1, 1, 1), glass);
            material* amber = CreateMaterial(S, PT_MATERIAL_TYPE_BASIC_TRANSLUCENT, "Amber");
            amber->Roughness = 0.1f;
            amber->TransmissionColor = vec3(0.9f, 0.45f, 0.2f);
            amber->TransmissionDepth = 0.5f;
            amber->ScatteringColor = vec3(0.3f, 0.3f, 0.3f);
            amber->ScatteringAnisotropy = 0.3f;
            Shape(S, ENTITY_TYPE_SPHERE, vec3(2.6f, 2.6f, 1), vec3(0, 0, 0), vec3(1, 1, 1), amber);
            material* grey = Diffuse(S, "Grey", vec3(0.6f, 0.6f, 0.6f));
            Shape(S, ENTITY_TYPE_CUBE, vec3(-1.6f, 5.0f, 0.5f), vec3(0, 0, 0.5f), vec3(0.5f, 0.5f, 0.5f), grey);
            Shape(S, ENTITY_TYPE_CUBE, vec3(1.8f, 5.5f, 0.7f), vec3(0.2f, 0, -0.3f), vec3(0.7f, 0.7f, 0.7f), blue);
            material* rm = CreateMaterial(S, PT_MATERIAL_TYPE_BASIC_DIFFUSE, "RoomMaterial");
            rm->BaseTexture = BuildRoomTexture(S);
            entity* room = CreateEntity(S, ENTITY_TYPE_MESH_INSTANCE);
            room->Mesh = BuildRoomMesh(S);
            room->Material = rm;
            room->Transform.Position = vec3(0, 9, 0.001f);
            room->Transform.Scale = vec3(1.5f, 1.5f, 1.5f);
            entity* lens = FirstCamera(S);
            lens->CameraModel = PT_CAMERA_MODEL_THIN_LENS;
            lens->ThinLensSensorSizeInMM = vec2(32.0f, 16.0f);
            lens->ThinLensFocalLengthInMM = 50.0f;
            lens->ThinLensApertureDiameterInMM = 20.0f;
            lens->ThinLensFocusDistance = 3.0f;
            lens->Transform.Position = vec3(0, -2.5f, 1.2f);
            lens->Transform.Rotation = vec3(PI / 2 - 0.05f, 0, 0);
            entity* pano = CreateEntity(S, ENTITY_TYPE_CAMERA);
            pano->CameraModel = PT_CAMERA_MODEL_360;
            pano->Transform.Position = vec3(0, 0.5f, 1.6f);
            I.width = 2048; I.height = 1024; I.spp = 8192; I.camera_count = 2;
            I.mesh_face_count = (uint32_t)room->Mesh->Faces.size();
            break;
        }
        default:
            return nullptr;
    }
    S->DirtyFlags = PT_SCENE_DIRTY_ALL;
    PackSceneData(S);
    I.shape_count = (uint32_t)S->ShapePack.size();
    if (info) *info = I;
    return S;
}

}  // namespace pth
