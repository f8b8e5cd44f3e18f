// scene.cpp — restatement of the reference's scene construction and
// PackSceneData (src/scene/scene.cpp:161-1621), without Vulkan.
#include "scene.hpp"

#include <algorithm>
#include <cassert>
#include <cstring>
#include <array>
#include <cstdlib>
#include <functional>
#include <thread>
#include <vector>

namespace pth {

namespace {

void Grow(bounds& B, vec3 P)                  // scene.cpp:41-45
{
    B.Minimum = vmin(B.Minimum, P);
    B.Maximum = vmax(B.Maximum, P);
}

void Grow(bounds& B, bounds const& O)         // scene.cpp:47-51
{
    B.Minimum = vmin(B.Minimum, O.Minimum);
    B.Maximum = vmax(B.Maximum, O.Maximum);
}

float HalfArea(bounds const& Box)             // scene.cpp:59-63
{
    vec3 E = Box.Maximum - Box.Minimum;
    return E.x * E.y + E.y * E.z + E.z * E.x;
}

uint32_t F2U(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

uint32_t GetPackedTextureIndex(texture* T) { return T ? T->PackedTextureIndex : PT_TEXTURE_INDEX_NONE; }
uint32_t GetPackedMaterialIndex(material* M) { return M ? M->PackedMaterialIndex : 0; }

void PackTransform(const mat4& M, pt_packed_transform* Out)   // scene.hpp:403-406
{
    mat4 I = inverse(M);
    for (int c = 0; c < 4; c++)
        for (int r = 0; r < 4; r++) {
            Out->To[c * 4 + r] = M[c][r];
            Out->From[c * 4 + r] = I[c][r];
        }
}

// ForEachEntityWithTransform (scene.cpp:127-159): children first, then the
// entity itself, with Transform = Outer * T * R * S.
void ForEachEntityWithTransform(entity* Entity, const mat4& Outer,
                                const std::function<void(entity*, const mat4&)>& F)
{
    if (!Entity->Active) return;
    mat4 Transform = Outer * MakeTransformMatrix(Entity->Transform.Position, Entity->Transform.Rotation,
                                                 Entity->Transform.Scale);
    for (entity* Inner : Entity->Children) ForEachEntityWithTransform(Inner, Transform, F);
    F(Entity, Transform);
}

// BuildMeshNode (scene.cpp:435-599): 32-bin centroid SAH per axis.
//
// The build is split into SplitMeshNode (one node's bounds, binned SAH and
// partition: the reference's function body up to its recursion) and two
// drivers: BuildMeshNode, the reference's sequential recursion, and
// BuildMeshSubtree, which runs the two children of the top nodes on separate
// threads and the bounds / centroid-range / binning passes of large nodes
// over chunks of the face range.  Both give the reference's nodes and face
// order bit for bit: chunk results merge in chunk order, and Grow, gmin/gmax
// and std::min/max keep the earlier of equal values exactly as the sequential
// fold does (so even the signs of zero bounds agree); bin counts are integer
// sums; the SAH sweep and the partition loop are the reference's, run by one
// thread per node; and the node array is assembled in the reference's
// allocation order (a node's two children, then the left child's
// descendants, then the right child's).

struct bvh_ctx {
    const std::vector<mesh_vertex>* V;
    std::vector<mesh_face>* F;
};

inline float FaceCentroid(const bvh_ctx& C, uint32_t FaceIndex, int Axis)   // GetMeshFaceCentroid, scene.cpp:424-433
{
    float Centroid = 0.0f;
    for (uint32_t I = 0; I < 3; I++) Centroid += (*C.V)[(*C.F)[FaceIndex].VertexIndex[I]].Position[Axis];
    return Centroid / 3.0f;
}

constexpr uint32_t BVH_BINS = 32;
struct bvh_bin { bounds Bounds; uint32_t FaceCount = 0; };

// Runs body(chunk, begin, end) over `parts` contiguous chunks of [b, e)
// (chunk 0 on the calling thread).
template <class Body>
void ForChunks(uint32_t b, uint32_t e, unsigned parts, Body body)
{
    if (parts <= 1) { body(0u, b, e); return; }
    std::vector<std::thread> pool;
    uint64_t n = e - b;
    for (unsigned c = 1; c < parts; c++) {
        uint32_t cb = (uint32_t)(b + n * c / parts), ce = (uint32_t)(b + n * (c + 1) / parts);
        try {
            pool.emplace_back(body, c, cb, ce);
        } catch (...) {   // no thread available: this chunk on the calling thread (same result)
            body(c, cb, ce);
        }
    }
    body(0u, b, (uint32_t)(b + n / parts));
    for (auto& t : pool) t.join();
}

constexpr uint32_t BVH_PARALLEL_PASS_FACES = 1u << 16;   // below this a node's passes stay on one thread

// One node of BuildMeshNode: bounds, split choice, partition.  Returns the
// split index, or 0 when the node stays a leaf.
uint32_t SplitMeshNode(const bvh_ctx& C, mesh_node& Node, unsigned threads)
{
    const uint32_t B0 = Node.FaceBeginIndex, E0 = Node.FaceEndIndex;
    uint32_t FaceCount = E0 - B0;
    unsigned parts = FaceCount >= BVH_PARALLEL_PASS_FACES ? std::max(1u, threads) : 1u;

    {
        std::vector<bounds> part(parts);
        ForChunks(B0, E0, parts, [&](unsigned c, uint32_t b, uint32_t e) {
            bounds Bd;
            for (uint32_t Index = b; Index < e; Index++)
                for (int J = 0; J < 3; J++) Grow(Bd, (*C.V)[(*C.F)[Index].VertexIndex[J]].Position);
            part[c] = Bd;
        });
        Node.Bounds = {};
        for (auto& Bd : part) Grow(Node.Bounds, Bd);
    }

    int SplitAxis = 0;
    float SplitPosition = 0;
    float SplitCost = +INF;

    for (int Axis = 0; Axis < 3; Axis++) {
        std::vector<float> pmin(parts, +INF), pmax(parts, -INF);
        ForChunks(B0, E0, parts, [&](unsigned c, uint32_t b, uint32_t e) {
            float Mn = +INF, Mx = -INF;
            for (uint32_t FaceIndex = b; FaceIndex < e; FaceIndex++) {
                float Centroid = FaceCentroid(C, FaceIndex, Axis);
                Mn = std::min(Mn, Centroid);
                Mx = std::max(Mx, Centroid);
            }
            pmin[c] = Mn;
            pmax[c] = Mx;
        });
        float Minimum = +INF, Maximum = -INF;
        for (unsigned c = 0; c < parts; c++) { Minimum = std::min(Minimum, pmin[c]); Maximum = std::max(Maximum, pmax[c]); }
        if (Minimum == Maximum) continue;

        float BinIndexPerUnit = float(BVH_BINS) / (Maximum - Minimum);
        std::vector<std::array<bvh_bin, BVH_BINS>> pbins(parts);
        ForChunks(B0, E0, parts, [&](unsigned c, uint32_t b, uint32_t e) {
            auto& Bins = pbins[c];
            for (uint32_t I = b; I < e; I++) {
                float Centroid = FaceCentroid(C, I, Axis);
                uint32_t BinIndexUnclamped = static_cast<uint32_t>(BinIndexPerUnit * (Centroid - Minimum));
                bvh_bin& Bin = Bins[std::min(BinIndexUnclamped, BVH_BINS - 1)];
                for (int J = 0; J < 3; J++) Grow(Bin.Bounds, (*C.V)[(*C.F)[I].VertexIndex[J]].Position);
                Bin.FaceCount++;
            }
        });
        std::array<bvh_bin, BVH_BINS> Bins;
        for (unsigned c = 0; c < parts; c++)
            for (uint32_t k = 0; k < BVH_BINS; k++) {
                Grow(Bins[k].Bounds, pbins[c][k].Bounds);
                Bins[k].FaceCount += pbins[c][k].FaceCount;
            }

        struct split { float LeftArea = 0; uint32_t LeftCount = 0; float RightArea = 0; uint32_t RightCount = 0; };
        split Splits[BVH_BINS - 1];
        bounds LeftBounds, RightBounds;
        uint32_t LeftCountSum = 0, RightCountSum = 0;
        for (uint32_t I = 0; I < BVH_BINS - 1; I++) {
            uint32_t J = BVH_BINS - 2 - I;
            bvh_bin const& LeftBin = Bins[I];
            if (LeftBin.FaceCount > 0) { LeftCountSum += LeftBin.FaceCount; Grow(LeftBounds, LeftBin.Bounds); }
            Splits[I].LeftCount = LeftCountSum;
            Splits[I].LeftArea = HalfArea(LeftBounds);
            bvh_bin const& RightBin = Bins[J + 1];
            if (RightBin.FaceCount > 0) { RightCountSum += RightBin.FaceCount; Grow(RightBounds, RightBin.Bounds); }
            Splits[J].RightCount = RightCountSum;
            Splits[J].RightArea = HalfArea(RightBounds);
        }

        float Interval = (Maximum - Minimum) / float(BVH_BINS);
        float Position = Minimum + Interval;
        for (uint32_t I = 0; I < BVH_BINS - 1; I++) {
            split const& Split = Splits[I];
            float Cost = Split.LeftCount * Split.LeftArea + Split.RightCount * Split.RightArea;
            if (Cost < SplitCost) { SplitCost = Cost; SplitAxis = Axis; SplitPosition = Position; }
            Position += Interval;
        }
    }

    float NoSplitCost = FaceCount * HalfArea(Node.Bounds);
    if (SplitCost >= NoSplitCost) return 0;

    // Partition (scene.cpp:556-573); the element where the two indices meet
    // is not examined and ends up on the right.
    uint32_t SplitIndex = B0;
    uint32_t SwapIndex = E0 - 1;
    while (SplitIndex < SwapIndex) {
        float Centroid = FaceCentroid(C, SplitIndex, SplitAxis);
        if (Centroid < SplitPosition) SplitIndex++;
        else { std::swap((*C.F)[SplitIndex], (*C.F)[SwapIndex]); SwapIndex--; }
    }
    if (SplitIndex == B0 || SplitIndex == E0) return 0;
    return SplitIndex;
}

// The reference's recursion over Nodes (children pushed adjacently, then
// the left subtree, then the right one).
void BuildMeshNode(const bvh_ctx& C, std::vector<mesh_node>& Nodes, uint32_t& MaxDepth, uint32_t NodeIndex,
                   uint32_t Depth)
{
    uint32_t SplitIndex = SplitMeshNode(C, Nodes[NodeIndex], 1);
    if (!SplitIndex) return;
    uint32_t LeftNodeIndex = static_cast<uint32_t>(Nodes.size());
    uint32_t RightNodeIndex = LeftNodeIndex + 1;
    Nodes[NodeIndex].ChildNodeIndex = LeftNodeIndex;
    mesh_node Left, Right;
    Left.FaceBeginIndex = Nodes[NodeIndex].FaceBeginIndex; Left.FaceEndIndex = SplitIndex;
    Right.FaceBeginIndex = SplitIndex; Right.FaceEndIndex = Nodes[NodeIndex].FaceEndIndex;
    Nodes.push_back(Left);
    Nodes.push_back(Right);
    MaxDepth = std::max(MaxDepth, Depth + 1);
    BuildMeshNode(C, Nodes, MaxDepth, LeftNodeIndex, Depth + 1);
    BuildMeshNode(C, Nodes, MaxDepth, RightNodeIndex, Depth + 1);
}

// Subtree of `Root` as [Root] + its descendants in the reference's order,
// child indices local to the returned array.  With threads > 1 the two
// children are built concurrently (threads split between them); their
// arrays are then spliced: S(X) = [X, L, R] + S(L)[1:] + S(R)[1:].
std::vector<mesh_node> BuildMeshSubtree(const bvh_ctx& C, mesh_node Root, uint32_t Depth, uint32_t& MaxDepth,
                                        unsigned threads)
{
    std::vector<mesh_node> Out;
    if (threads <= 1 || Root.FaceEndIndex - Root.FaceBeginIndex < BVH_PARALLEL_PASS_FACES / 4) {
        Out.reserve(2 * (size_t)(Root.FaceEndIndex - Root.FaceBeginIndex));
        Out.push_back(Root);
        BuildMeshNode(C, Out, MaxDepth, 0, Depth);
        return Out;
    }
    uint32_t SplitIndex = SplitMeshNode(C, Root, threads);
    if (!SplitIndex) { Out.push_back(Root); return Out; }
    mesh_node Left, Right;
    Left.FaceBeginIndex = Root.FaceBeginIndex; Left.FaceEndIndex = SplitIndex;
    Right.FaceBeginIndex = SplitIndex; Right.FaceEndIndex = Root.FaceEndIndex;
    MaxDepth = std::max(MaxDepth, Depth + 1);
    uint32_t DL = 0, DR = 0;
    std::vector<mesh_node> SL, SR;
    unsigned tl = threads / 2, tr = threads - tl;
    std::thread worker;
    try {
        worker = std::thread([&] { SL = BuildMeshSubtree(C, Left, Depth + 1, DL, tl); });
    } catch (...) {   // no thread available: build the left subtree here first (same result)
        SL = BuildMeshSubtree(C, Left, Depth + 1, DL, 1);
    }
    SR = BuildMeshSubtree(C, Right, Depth + 1, DR, tr);
    if (worker.joinable()) worker.join();
    MaxDepth = std::max(MaxDepth, std::max(DL, DR));
    const uint32_t offL = 2, offR = 2 + (uint32_t)(SL.size() - 1);
    Out.reserve(1 + SL.size() + SR.size());
    Root.ChildNodeIndex = 1;
    Out.push_back(Root);
    Out.push_back(SL[0]);
    Out.push_back(SR[0]);
    if (Out[1].ChildNodeIndex) Out[1].ChildNodeIndex += offL;
    if (Out[2].ChildNodeIndex) Out[2].ChildNodeIndex += offR;
    for (size_t i = 1; i < SL.size(); i++) {
        Out.push_back(SL[i]);
        if (Out.back().ChildNodeIndex) Out.back().ChildNodeIndex += offL;
    }
    for (size_t i = 1; i < SR.size(); i++) {
        Out.push_back(SR[i]);
        if (Out.back().ChildNodeIndex) Out.back().ChildNodeIndex += offR;
    }
    return Out;
}

// ShapeBounds (scene.cpp:1031-1093)
bounds ShapeBounds(scene const* Scene, pt_packed_shape const& Object)
{
    vec4 Corners[8];
    switch (Object.Type) {
        case PT_SHAPE_TYPE_MESH_INSTANCE: {
            const pt_packed_mesh_node& R = Scene->MeshNodePack[Object.MeshRootNodeIndex];
            vec3 Mn(R.Minimum[0], R.Minimum[1], R.Minimum[2]);
            vec3 Mx(R.Maximum[0], R.Maximum[1], R.Maximum[2]);
            Corners[0] = {Mn.x, Mn.y, Mn.z, 1}; Corners[1] = {Mn.x, Mn.y, Mx.z, 1};
            Corners[2] = {Mn.x, Mx.y, Mn.z, 1}; Corners[3] = {Mn.x, Mx.y, Mx.z, 1};
            Corners[4] = {Mx.x, Mn.y, Mn.z, 1}; Corners[5] = {Mx.x, Mn.y, Mx.z, 1};
            Corners[6] = {Mx.x, Mx.y, Mn.z, 1}; Corners[7] = {Mx.x, Mx.y, Mx.z, 1};
            break;
        }
        case PT_SHAPE_TYPE_PLANE:
            Corners[0] = {-1e9f, -1e9f, -EPSILON, 1}; Corners[1] = {+1e9f, -1e9f, -EPSILON, 1};
            Corners[2] = {-1e9f, +1e9f, -EPSILON, 1}; Corners[3] = {+1e9f, +1e9f, -EPSILON, 1};
            Corners[4] = {-1e9f, -1e9f, +EPSILON, 1}; Corners[5] = {+1e9f, -1e9f, +EPSILON, 1};
            Corners[6] = {-1e9f, +1e9f, +EPSILON, 1}; Corners[7] = {+1e9f, +1e9f, +EPSILON, 1};
            break;
        default:
            Corners[0] = {-1, -1, -1, 1}; Corners[1] = {+1, -1, -1, 1};
            Corners[2] = {-1, +1, -1, 1}; Corners[3] = {+1, +1, -1, 1};
            Corners[4] = {-1, -1, +1, 1}; Corners[5] = {+1, -1, +1, 1};
            Corners[6] = {-1, +1, +1, 1}; Corners[7] = {+1, +1, +1, 1};
            break;
    }
    mat4 To;
    for (int c = 0; c < 4; c++)
        for (int r = 0; r < 4; r++) To[c][r] = Object.Transform.To[c * 4 + r];
    vec3 WorldMin(+INF), WorldMax(-INF);
    for (const vec4& Corner : Corners) {
        vec3 W = (To * Corner).xyz();
        WorldMin = vmin(WorldMin, W);
        WorldMax = vmax(WorldMax, W);
    }
    return {WorldMin, WorldMax};
}

// --- texture atlas: skyline bottom-left packer --------------------------------
// Restates stb_rect_pack's default heuristic (Skyline_BL_sortHeight,
// src/core/stb_rect_pack.h:258-600) as the reference configures it
// (scene.cpp:1143-1147: 4096x4096 target, 4096 nodes, so align = 1).
struct skyline_rect { int id, w, h, x, y; bool packed; };

void SkylinePack(int W, int H, std::vector<skyline_rect>& Rects)
{
    struct node { int x, y; };
    std::vector<node> Sky{{0, 0}};   // segment i spans [Sky[i].x, Sky[i+1].x or W)
    std::vector<int> order(Rects.size());
    for (size_t i = 0; i < order.size(); i++) order[i] = (int)i;
    // rect_height_compare: height desc, then width desc (ties: original order).
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
        if (Rects[a].h != Rects[b].h) return Rects[a].h > Rects[b].h;
        return Rects[a].w > Rects[b].w;
    });
    for (int idx : order) {
        skyline_rect& R = Rects[idx];
        R.packed = false;
        if (R.w == 0 || R.h == 0) { R.x = R.y = 0; R.packed = true; continue; }
        if (R.w > W || R.h > H) continue;
        int best_y = 1 << 30, best_i = -1;
        for (size_t i = 0; i < Sky.size(); i++) {
            int x0 = Sky[i].x;
            if (x0 + R.w > W) break;
            int min_y = 0;
            for (size_t k = i; k < Sky.size() && Sky[k].x < x0 + R.w; k++) min_y = std::max(min_y, Sky[k].y);
            if (min_y < best_y) { best_y = min_y; best_i = (int)i; }
        }
        if (best_i < 0 || best_y + R.h > H) continue;
        int x0 = Sky[best_i].x, x1 = x0 + R.w;
        // New skyline: segments before x0, [x0,x1) at best_y+h, remainder after x1
        // (x0 is always a segment start: candidates are segment starts).
        std::vector<node> NewSky;
        for (size_t k = 0; k < Sky.size(); k++) {
            int sx = Sky[k].x;
            int ex = (k + 1 < Sky.size()) ? Sky[k + 1].x : W;
            if (ex <= x0) { NewSky.push_back(Sky[k]); continue; }
            if (sx == x0) NewSky.push_back({x0, best_y + R.h});
            if (ex > x1) NewSky.push_back({std::max(sx, x1), Sky[k].y});
        }
        Sky = NewSky;
        R.x = x0;
        R.y = best_y;
        R.packed = true;
    }
}

}  // namespace

scene::~scene()
{
    for (entity* E : Entities) delete E;
    for (mesh* M : Meshes) delete M;
    for (material* M : Materials) delete M;
    for (texture* T : Textures) delete T;
    for (prefab* P : Prefabs) delete P;
    if (OwnsSpectrumTable) delete RGBSpectrumTable;
}

scene* CreateEmptyScene()
{
    scene* Scene = new scene;
    Scene->Root.Name = "Scene";
    Scene->Root.Type = ENTITY_TYPE_ROOT;
    Scene->RGBSpectrumTable = GetSharedSpectrumTable();
    // packed_scene_globals member defaults (scene.hpp:152-162)
    Scene->Globals = pt_packed_scene_globals{};
    Scene->Globals.SkyboxConcentration = 1.0f;
    Scene->Globals.SkyboxSamplingProbability = 0.0f;
    Scene->Globals.SkyboxBrightness = 1.0f;
    Scene->Globals.SkyboxTextureIndex = PT_TEXTURE_INDEX_NONE;
    Scene->DirtyFlags = PT_SCENE_DIRTY_ALL;
    return Scene;
}

scene* CreateScene()
{
    scene* Scene = CreateEmptyScene();
    material* PlaneMaterial = CreateMaterial(Scene, PT_MATERIAL_TYPE_BASIC_DIFFUSE, "Plane Material");
    PlaneMaterial->BaseTexture = CreateCheckerTexture(Scene, "Plane Texture", PT_TEXTURE_TYPE_REFLECTANCE_WITH_ALPHA,
                                                      vec4(1, 1, 1, 1), vec4(0.5f, 0.5f, 0.5f, 1));
    PlaneMaterial->BaseTexture->EnableNearestFiltering = true;
    entity* Plane = CreateEntity(Scene, ENTITY_TYPE_PLANE);
    Plane->Name = "Plane";
    Plane->Material = PlaneMaterial;
    entity* Camera = CreateEntity(Scene, ENTITY_TYPE_CAMERA);
    Camera->Name = "Camera";
    Camera->Transform.Position = vec3(0, 0, 1);
    Scene->DirtyFlags = PT_SCENE_DIRTY_ALL;
    return Scene;
}

void DestroyScene(scene* Scene) { delete Scene; }

entity* CreateEntity(scene* Scene, entity_type Type, entity* Parent)
{
    entity* E = new entity;
    E->Type = Type;
    if (!Parent) Parent = &Scene->Root;
    E->Parent = Parent;
    Parent->Children.push_back(E);
    Scene->Entities.push_back(E);
    Scene->DirtyFlags |= PT_SCENE_DIRTY_SHAPES | PT_SCENE_DIRTY_CAMERAS;
    return E;
}

material* CreateMaterial(scene* Scene, uint32_t Type, const char* Name)
{
    material* M = new material;
    M->Type = Type;
    M->Name = Name ? Name : "New Material";
    Scene->Materials.push_back(M);
    Scene->DirtyFlags |= PT_SCENE_DIRTY_MATERIALS;
    return M;
}

texture* CreateCheckerTexture(scene* Scene, const char* Name, uint32_t Type, vec4 ColorA, vec4 ColorB)
{
    texture* T = new texture;   // scene.cpp:270-292
    T->Name = Name;
    T->Type = Type;
    T->Width = 2;
    T->Height = 2;
    T->Pixels = {ColorA, ColorB, ColorB, ColorA};
    Scene->Textures.push_back(T);
    Scene->DirtyFlags |= PT_SCENE_DIRTY_TEXTURES;
    return T;
}

texture* CreateTexture(scene* Scene, const char* Name, uint32_t Type, uint32_t Width, uint32_t Height,
                       const float* RGBA)
{
    texture* T = new texture;
    T->Name = Name ? Name : "Texture";
    T->Type = Type;
    T->Width = Width;
    T->Height = Height;
    T->Pixels.resize((size_t)Width * Height);
    for (size_t i = 0; i < T->Pixels.size(); i++)
        T->Pixels[i] = vec4(RGBA[4 * i + 0], RGBA[4 * i + 1], RGBA[4 * i + 2], RGBA[4 * i + 3]);
    Scene->Textures.push_back(T);
    Scene->DirtyFlags |= PT_SCENE_DIRTY_TEXTURES;
    return T;
}

// Threads for a mesh build: PT_BVH_THREADS, else OMP_NUM_THREADS, else the
// hardware's; 1 runs the reference's sequential recursion.
unsigned BvhThreads()
{
    unsigned t = std::thread::hardware_concurrency();
    if (const char* e = std::getenv("OMP_NUM_THREADS")) t = (unsigned)std::max(1, atoi(e));
    if (const char* e = std::getenv("PT_BVH_THREADS")) t = (unsigned)std::max(1, atoi(e));
    return std::min(std::max(t, 1u), 64u);
}

void BuildMeshBVH(mesh* Mesh)   // scene.cpp:851-866
{
    mesh_node Root;
    Root.FaceBeginIndex = 0;
    Root.FaceEndIndex = static_cast<uint32_t>(Mesh->Faces.size());
    Root.ChildNodeIndex = 0;
    bvh_ctx C{&Mesh->Vertices, &Mesh->Faces};
    Mesh->Depth = 0;
    Mesh->Nodes = BuildMeshSubtree(C, Root, 0, Mesh->Depth, BvhThreads());
}

mesh* CreateMesh(scene* Scene, const char* Name, uint32_t VertexCount, const float* Positions,
                 const float* Normals, const float* UVs, uint32_t FaceCount, const uint32_t* Indices)
{
    mesh* M = new mesh;
    M->Name = Name ? Name : "Mesh";
    M->Vertices.resize(VertexCount);
    for (uint32_t i = 0; i < VertexCount; i++) {
        M->Vertices[i].Position = vec3(Positions[3 * i], Positions[3 * i + 1], Positions[3 * i + 2]);
        if (Normals) M->Vertices[i].Normal = vec3(Normals[3 * i], Normals[3 * i + 1], Normals[3 * i + 2]);
        if (UVs) M->Vertices[i].UV = vec2(UVs[2 * i], UVs[2 * i + 1]);
    }
    M->Faces.resize(FaceCount);
    for (uint32_t f = 0; f < FaceCount; f++)
        for (int j = 0; j < 3; j++) M->Faces[f].VertexIndex[j] = Indices[3 * f + j];
    BuildMeshBVH(M);
    Scene->Meshes.push_back(M);
    Scene->DirtyFlags |= PT_SCENE_DIRTY_MESHES;
    return M;
}

// --- material attribute packing (basic_*.hpp *_PackData) --------------------
static void PackMaterialData(scene* Scene, material* M, uint32_t* A)
{
    parametric_spectrum_table* T = Scene->RGBSpectrumTable;
    auto Spec = [&](vec3 C, uint32_t* Dst) {
        vec3 B = GetParametricSpectrumCoefficients(T, C);
        Dst[0] = F2U(B.x); Dst[1] = F2U(B.y); Dst[2] = F2U(B.z);
    };
    switch (M->Type) {
        case PT_MATERIAL_TYPE_BASIC_DIFFUSE:       // basic_diffuse.hpp:17-28
            Spec(M->BaseColor, &A[PT_BASIC_DIFFUSE_BASE_SPECTRUM]);
            A[PT_BASIC_DIFFUSE_BASE_SPECTRUM + 3] = GetPackedTextureIndex(M->BaseTexture);
            break;
        case PT_MATERIAL_TYPE_BASIC_METAL:         // basic_metal.hpp:26-52
            Spec(M->BaseColor, &A[PT_BASIC_METAL_BASE_SPECTRUM]);
            A[PT_BASIC_METAL_BASE_SPECTRUM + 3] = GetPackedTextureIndex(M->BaseTexture);
            Spec(M->SpecularColor, &A[PT_BASIC_METAL_SPECULAR_SPECTRUM]);
            A[PT_BASIC_METAL_SPECULAR_SPECTRUM + 3] = GetPackedTextureIndex(M->SpecularTexture);
            A[PT_BASIC_METAL_ROUGHNESS + 0] = F2U(M->Roughness);
            A[PT_BASIC_METAL_ROUGHNESS + 1] = GetPackedTextureIndex(M->RoughnessTexture);
            A[PT_BASIC_METAL_ROUGHNESS_ANISOTROPY + 0] = F2U(M->RoughnessAnisotropy);
            A[PT_BASIC_METAL_ROUGHNESS_ANISOTROPY + 1] = GetPackedTextureIndex(M->RoughnessAnisotropyTexture);
            break;
        case PT_MATERIAL_TYPE_BASIC_TRANSLUCENT:   // basic_translucent.hpp:26-61
            A[PT_BASIC_TRANSLUCENT_IOR] = F2U(M->IOR);
            A[PT_BASIC_TRANSLUCENT_ABBE_NUMBER] = F2U(M->AbbeNumber);
            A[PT_BASIC_TRANSLUCENT_ROUGHNESS + 0] = F2U(M->Roughness);
            A[PT_BASIC_TRANSLUCENT_ROUGHNESS + 1] = GetPackedTextureIndex(M->RoughnessTexture);
            A[PT_BASIC_TRANSLUCENT_ROUGHNESS_ANISOTROPY + 0] = F2U(M->RoughnessAnisotropy);
            A[PT_BASIC_TRANSLUCENT_ROUGHNESS_ANISOTROPY + 1] = GetPackedTextureIndex(M->RoughnessAnisotropyTexture);
            Spec(M->TransmissionColor, &A[PT_BASIC_TRANSLUCENT_TRANSMISSION_SPECTRUM]);
            A[PT_BASIC_TRANSLUCENT_TRANSMISSION_DEPTH] = F2U(M->TransmissionDepth);
            Spec(M->ScatteringColor, &A[PT_BASIC_TRANSLUCENT_SCATTERING_SPECTRUM]);
            A[PT_BASIC_TRANSLUCENT_SCATTERING_ANISOTROPY] = F2U(M->ScatteringAnisotropy);
            break;
        case PT_MATERIAL_TYPE_OPENPBR: {           // openpbr.hpp:52-134
            A[PT_OPENPBR_LAYER_BOUNCE_LIMIT] = static_cast<uint32_t>(M->LayerBounceLimit);
            A[PT_OPENPBR_BASE_WEIGHT] = F2U(M->BaseWeight);
            Spec(M->BaseColor, &A[PT_OPENPBR_BASE_SPECTRUM]);
            A[PT_OPENPBR_BASE_SPECTRUM_TEXTURE_INDEX] = GetPackedTextureIndex(M->BaseTexture);
            A[PT_OPENPBR_BASE_METALNESS] = F2U(M->BaseMetalness);
            A[PT_OPENPBR_BASE_DIFFUSE_ROUGHNESS] = F2U(M->BaseDiffuseRoughness);
            A[PT_OPENPBR_SPECULAR_WEIGHT] = F2U(M->SpecularWeight);
            Spec(M->SpecularColor, &A[PT_OPENPBR_SPECULAR_SPECTRUM]);
            A[PT_OPENPBR_SPECULAR_IOR] = F2U(M->SpecularIOR);
            A[PT_OPENPBR_SPECULAR_ROUGHNESS] = F2U(M->Roughness);
            A[PT_OPENPBR_SPECULAR_ROUGHNESS_TEXTURE_INDEX] = GetPackedTextureIndex(M->RoughnessTexture);
            A[PT_OPENPBR_SPECULAR_ROUGHNESS_ANISOTROPY] = F2U(M->RoughnessAnisotropy);
            Spec(M->TransmissionColor, &A[PT_OPENPBR_TRANSMISSION_SPECTRUM]);
            A[PT_OPENPBR_TRANSMISSION_WEIGHT] = F2U(M->TransmissionWeight);
            Spec(M->TransmissionScatter, &A[PT_OPENPBR_TRANSMISSION_SCATTER_SPECTRUM]);
            A[PT_OPENPBR_TRANSMISSION_SCATTER_ANISOTROPY] = F2U(M->TransmissionScatterAnisotropy);
            A[PT_OPENPBR_TRANSMISSION_DEPTH] = F2U(M->TransmissionDepth);
            A[PT_OPENPBR_TRANSMISSION_DISPERSION_ABBE_NUMBER] =
                F2U(M->TransmissionDispersionAbbeNumber / M->TransmissionDispersionScale);
            Spec(M->EmissionColor, &A[PT_OPENPBR_EMISSION_SPECTRUM]);
            A[PT_OPENPBR_EMISSION_SPECTRUM_TEXTURE_INDEX] = GetPackedTextureIndex(M->EmissionColorTexture);
            A[PT_OPENPBR_EMISSION_LUMINANCE] = F2U(M->EmissionLuminance);
            A[PT_OPENPBR_COAT_WEIGHT] = F2U(M->CoatWeight);
            Spec(M->CoatColor, &A[PT_OPENPBR_COAT_COLOR_SPECTRUM]);
            A[PT_OPENPBR_COAT_IOR] = F2U(M->CoatIOR);
            A[PT_OPENPBR_COAT_ROUGHNESS] = F2U(M->CoatRoughness);
            A[PT_OPENPBR_COAT_ROUGHNESS_ANISOTROPY] = F2U(M->CoatRoughnessAnisotropy);
            A[PT_OPENPBR_COAT_DARKENING] = F2U(M->CoatDarkening);
            break;
        }
    }
}

uint32_t PackSceneData(scene* Scene)
{
    uint32_t DirtyFlags = Scene->DirtyFlags;
    parametric_spectrum_table* Table = Scene->RGBSpectrumTable;

    // Textures -> atlas layers (scene.cpp:1120-1233).
    if (DirtyFlags & PT_SCENE_DIRTY_TEXTURES) {
        const uint32_t AW = Scene->AtlasWidth, AH = Scene->AtlasHeight;
        std::vector<skyline_rect> Rects;
        for (size_t i = 0; i < Scene->Textures.size(); i++)
            Rects.push_back({(int)i, (int)Scene->Textures[i]->Width, (int)Scene->Textures[i]->Height, 0, 0, false});
        Scene->TexturePack.clear();
        Scene->AtlasFlat.clear();
        uint32_t ImageIndex = 0;
        while (!Rects.empty()) {
            SkylinePack((int)AW, (int)AH, Rects);
            size_t LayerBase = Scene->AtlasFlat.size();
            Scene->AtlasFlat.resize(LayerBase + (size_t)AW * AH * 4, 0.0f);
            float* Pixels = Scene->AtlasFlat.data() + LayerBase;
            bool any = false;
            for (skyline_rect& Rect : Rects) {
                if (!Rect.packed) continue;
                any = true;
                texture* Tx = Scene->Textures[Rect.id];
                Tx->PackedTextureIndex = static_cast<uint32_t>(Scene->TexturePack.size());
                pt_packed_texture P{};
                P.Flags = 0;
                P.AtlasImageIndex = ImageIndex;
                P.Type = Tx->Type;
                P.AtlasPlacementMinimum[0] = (Rect.x + 0.5f) / float(AW);
                P.AtlasPlacementMinimum[1] = (Rect.y + Rect.h - 0.5f) / float(AH);
                P.AtlasPlacementMaximum[0] = (Rect.x + Rect.w - 0.5f) / float(AW);
                P.AtlasPlacementMaximum[1] = (Rect.y + 0.5f) / float(AH);
                for (uint32_t Y = 0; Y < Tx->Height; Y++) {
                    const vec4* Src = Tx->Pixels.data() + (size_t)Y * Tx->Width;
                    float* Dst = Pixels + (((size_t)(Rect.y + Y) * AW + Rect.x) * 4);
                    for (uint32_t X = 0; X < Tx->Width; X++, Src++, Dst += 4) {
                        vec4 V = *Src;
                        vec4 Out;
                        if (Tx->Type == PT_TEXTURE_TYPE_RAW) {
                            Out = V;
                        } else if (Tx->Type == PT_TEXTURE_TYPE_REFLECTANCE_WITH_ALPHA) {
                            vec3 B = GetParametricSpectrumCoefficients(Table, V.xyz());
                            Out = vec4(B, V.w);
                        } else {
                            float Intensity = 2 * std::max(std::max(V.x, V.y), V.z);
                            if (Intensity > 1e-6f) {
                                vec3 B = GetParametricSpectrumCoefficients(Table, V.xyz() / Intensity);
                                Out = vec4(B, Intensity);
                            } else {
                                Out = vec4(0, 0, 0, 0);
                            }
                        }
                        Dst[0] = Out.x; Dst[1] = Out.y; Dst[2] = Out.z; Dst[3] = Out.w;
                    }
                }
                if (Tx->EnableNearestFiltering) P.Flags |= PT_TEXTURE_FLAG_FILTER_NEAREST;
                Scene->TexturePack.push_back(P);
            }
            ImageIndex++;
            Rects.erase(std::remove_if(Rects.begin(), Rects.end(), [](const skyline_rect& R) { return R.packed; }),
                        Rects.end());
            if (!any) break;   // a texture larger than the atlas can never be placed
        }
        DirtyFlags |= PT_SCENE_DIRTY_MATERIALS;
    }

    // Materials (scene.cpp:1236-1263): fallback OpenPBR in slots 0-1.
    if (DirtyFlags & PT_SCENE_DIRTY_MATERIALS) {
        Scene->MaterialAttributePack.clear();
        {
            material Fallback;
            Fallback.Type = PT_MATERIAL_TYPE_OPENPBR;
            Scene->MaterialAttributePack.resize(64, 0u);
            Scene->MaterialAttributePack[0] = Fallback.Type;
            PackMaterialData(Scene, &Fallback, &Scene->MaterialAttributePack[0]);
        }
        for (material* M : Scene->Materials) {
            size_t Offset = Scene->MaterialAttributePack.size();
            size_t Size = M->Type == PT_MATERIAL_TYPE_OPENPBR ? 64 : 32;
            Scene->MaterialAttributePack.resize(Offset + Size, 0u);
            Scene->MaterialAttributePack[Offset] = M->Type;
            PackMaterialData(Scene, M, &Scene->MaterialAttributePack[Offset]);
            M->PackedMaterialIndex = static_cast<uint32_t>(Offset) / 32;
        }
        DirtyFlags |= PT_SCENE_DIRTY_SHAPES;
    }

    // Meshes (scene.cpp:1266-1343).
    if (DirtyFlags & PT_SCENE_DIRTY_MESHES) {
        Scene->MeshVertexPack.clear();
        Scene->MeshFacePack.clear();
        Scene->MeshNodePack.clear();
        for (mesh* Mesh : Scene->Meshes) {
            uint32_t VertexIndexBase = (uint32_t)Scene->MeshVertexPack.size();
            uint32_t FaceIndexBase = (uint32_t)Scene->MeshFacePack.size();
            uint32_t NodeIndexBase = (uint32_t)Scene->MeshNodePack.size();
            for (const mesh_vertex& V : Mesh->Vertices) {
                pt_packed_mesh_vertex P;
                P.PackedNormal = PackUnitVector(V.Normal);
                P.PackedUV = packHalf2x16(V.UV);
                Scene->MeshVertexPack.push_back(P);
            }
            for (const mesh_face& F : Mesh->Faces) {
                pt_packed_mesh_face P;
                for (int j = 0; j < 3; j++) {
                    // A mesh loaded from a reference-written scene file has no
                    // vertices (serializer.cpp): pack zero positions instead of
                    // reading out of bounds; ptUpdateScene then rejects the faces.
                    uint32_t Vi = F.VertexIndex[j];
                    vec3 Pos = Vi < Mesh->Vertices.size() ? Mesh->Vertices[Vi].Position : vec3(0.0f);
                    float* Dst = j == 0 ? P.Position0 : (j == 1 ? P.Position1 : P.Position2);
                    Dst[0] = Pos.x; Dst[1] = Pos.y; Dst[2] = Pos.z;
                }
                P.VertexIndex0 = VertexIndexBase + F.VertexIndex[0];
                P.VertexIndex1 = VertexIndexBase + F.VertexIndex[1];
                P.VertexIndex2 = VertexIndexBase + F.VertexIndex[2];
                Scene->MeshFacePack.push_back(P);
            }
            for (const mesh_node& N : Mesh->Nodes) {
                pt_packed_mesh_node P;
                P.Minimum[0] = N.Bounds.Minimum.x; P.Minimum[1] = N.Bounds.Minimum.y; P.Minimum[2] = N.Bounds.Minimum.z;
                P.Maximum[0] = N.Bounds.Maximum.x; P.Maximum[1] = N.Bounds.Maximum.y; P.Maximum[2] = N.Bounds.Maximum.z;
                if (N.ChildNodeIndex > 0) {
                    P.FaceBeginOrNodeIndex = NodeIndexBase + N.ChildNodeIndex;
                    P.FaceEndIndex = 0;
                } else {
                    P.FaceBeginOrNodeIndex = FaceIndexBase + N.FaceBeginIndex;
                    P.FaceEndIndex = FaceIndexBase + N.FaceEndIndex;
                }
                Scene->MeshNodePack.push_back(P);
            }
            Mesh->PackedRootNodeIndex = NodeIndexBase;
        }
        DirtyFlags |= PT_SCENE_DIRTY_SHAPES;
    }

    // Shapes + shape TLAS (scene.cpp:1346-1498).
    if (DirtyFlags & PT_SCENE_DIRTY_SHAPES) {
        Scene->ShapePack.clear();
        Scene->ShapeNodePack.resize(1);
        ForEachEntityWithTransform(&Scene->Root, mat4(1.0f), [Scene](entity* Entity, const mat4& Transform) {
            pt_packed_shape P{};
            P.MaterialIndex = 0;
            switch (Entity->Type) {
                case ENTITY_TYPE_MESH_INSTANCE:
                    if (!Entity->Mesh) return;
                    P.MaterialIndex = GetPackedMaterialIndex(Entity->Material);
                    P.MeshRootNodeIndex = Entity->Mesh->PackedRootNodeIndex;
                    P.Type = PT_SHAPE_TYPE_MESH_INSTANCE;
                    break;
                case ENTITY_TYPE_PLANE:
                    P.MaterialIndex = GetPackedMaterialIndex(Entity->Material);
                    P.Type = PT_SHAPE_TYPE_PLANE;
                    break;
                case ENTITY_TYPE_SPHERE:
                    P.MaterialIndex = GetPackedMaterialIndex(Entity->Material);
                    P.Type = PT_SHAPE_TYPE_SPHERE;
                    break;
                case ENTITY_TYPE_CUBE:
                    P.MaterialIndex = GetPackedMaterialIndex(Entity->Material);
                    P.Type = PT_SHAPE_TYPE_CUBE;
                    break;
                default:
                    return;
            }
            PackTransform(Transform, &P.Transform);
            Entity->PackedShapeIndex = static_cast<uint32_t>(Scene->ShapePack.size());
            Scene->ShapePack.push_back(P);
        });

        std::vector<uint16_t> Map;
        for (uint32_t ShapeIndex = 0; ShapeIndex < Scene->ShapePack.size(); ShapeIndex++) {
            bounds B = ShapeBounds(Scene, Scene->ShapePack[ShapeIndex]);
            Map.push_back(static_cast<uint16_t>(Scene->ShapeNodePack.size()));
            pt_packed_shape_node N;
            N.Minimum[0] = B.Minimum.x; N.Minimum[1] = B.Minimum.y; N.Minimum[2] = B.Minimum.z;
            N.ChildNodeIndices = 0;
            N.Maximum[0] = B.Maximum.x; N.Maximum[1] = B.Maximum.y; N.Maximum[2] = B.Maximum.z;
            N.ShapeIndex = ShapeIndex;
            Scene->ShapeNodePack.push_back(N);
        }

        auto NodeMin = [Scene](uint16_t i) { auto& n = Scene->ShapeNodePack[i]; return vec3(n.Minimum[0], n.Minimum[1], n.Minimum[2]); };
        auto NodeMax = [Scene](uint16_t i) { auto& n = Scene->ShapeNodePack[i]; return vec3(n.Maximum[0], n.Maximum[1], n.Maximum[2]); };

        // FindBestMatch (scene.cpp:1422-1446), including the Size.z*Size.z typo.
        auto FindBestMatch = [&](const std::vector<uint16_t>& M, uint16_t IndexA) -> uint16_t {
            vec3 MinA = NodeMin(M[IndexA]), MaxA = NodeMax(M[IndexA]);
            float BestArea = INFINITY;
            uint16_t BestIndexB = 0xFFFF;
            for (uint16_t IndexB = 0; IndexB < M.size(); IndexB++) {
                if (IndexA == IndexB) continue;
                vec3 MinB = NodeMin(M[IndexB]), MaxB = NodeMax(M[IndexB]);
                vec3 Size = vmax(MaxA, MaxB) - vmin(MinA, MinB);
                float Area = Size.x * Size.y + Size.y * Size.z + Size.z * Size.z;
                if (Area <= BestArea) { BestArea = Area; BestIndexB = IndexB; }
            }
            return BestIndexB;
        };

        if (!Scene->ShapePack.empty()) {
            uint16_t IndexA = 0;
            uint16_t IndexB = FindBestMatch(Map, IndexA);
            while (Map.size() > 1) {
                uint16_t IndexC = FindBestMatch(Map, IndexB);
                if (IndexA == IndexC) {
                    uint16_t NodeIndexA = Map[IndexA];
                    uint16_t NodeIndexB = Map[IndexB];
                    pt_packed_shape_node N;
                    vec3 Mn = vmin(NodeMin(NodeIndexA), NodeMin(NodeIndexB));
                    vec3 Mx = vmax(NodeMax(NodeIndexA), NodeMax(NodeIndexB));
                    N.Minimum[0] = Mn.x; N.Minimum[1] = Mn.y; N.Minimum[2] = Mn.z;
                    N.ChildNodeIndices = uint32_t(NodeIndexA) | uint32_t(NodeIndexB) << 16;
                    N.Maximum[0] = Mx.x; N.Maximum[1] = Mx.y; N.Maximum[2] = Mx.z;
                    N.ShapeIndex = PT_SHAPE_INDEX_NONE;
                    Map[IndexA] = static_cast<uint16_t>(Scene->ShapeNodePack.size());
                    Map[IndexB] = Map.back();
                    Map.pop_back();
                    if (IndexA == Map.size()) IndexA = IndexB;
                    Scene->ShapeNodePack.push_back(N);
                    IndexB = FindBestMatch(Map, IndexA);
                } else {
                    IndexA = IndexB;
                    IndexB = IndexC;
                }
            }
            Scene->ShapeNodePack[0] = Scene->ShapeNodePack[Map[IndexA]];
            Scene->ShapeNodePack[Map[IndexA]] = Scene->ShapeNodePack.back();
            Scene->ShapeNodePack.pop_back();
        } else {
            Scene->ShapeNodePack.clear();
        }
        DirtyFlags |= PT_SCENE_DIRTY_GLOBALS;
    }

    // Cameras (scene.cpp:1501-1539).
    if (DirtyFlags & PT_SCENE_DIRTY_CAMERAS) {
        Scene->CameraPack.clear();
        ForEachEntityWithTransform(&Scene->Root, mat4(1.0f), [Scene](entity* E, const mat4& Transform) {
            if (E->Type != ENTITY_TYPE_CAMERA) return;
            pt_packed_camera P{};
            P.Model = E->CameraModel;
            if (E->CameraModel == PT_CAMERA_MODEL_PINHOLE) {
                const float AspectRatio = 2.0f;
                P.ApertureRadius = E->PinholeApertureDiameterInMM / 2000.0f;
                float Radians = (E->PinholeFieldOfViewInDegrees / 2) * 0.01745329251994329576923690768489f;
                P.SensorSize[0] = 2 * std::tan(Radians);
                P.SensorSize[1] = P.SensorSize[0] / AspectRatio;
                P.SensorDistance = 1.0f;
            }
            if (E->CameraModel == PT_CAMERA_MODEL_THIN_LENS) {
                P.FocalLength = E->ThinLensFocalLengthInMM / 1000.0f;
                P.ApertureRadius = E->ThinLensApertureDiameterInMM / 2000.0f;
                P.SensorDistance = 1.0f / (1000.0f / E->ThinLensFocalLengthInMM - 1.0f / E->ThinLensFocusDistance);
                P.SensorSize[0] = E->ThinLensSensorSizeInMM.x / 1000.0f;
                P.SensorSize[1] = E->ThinLensSensorSizeInMM.y / 1000.0f;
            }
            PackTransform(Transform, &P.Transform);
            E->PackedCameraIndex = static_cast<uint32_t>(Scene->CameraPack.size());
            Scene->CameraPack.push_back(P);
        });
    }

    // Skybox vMF fit (scene.cpp:1542-1604).
    if (DirtyFlags & PT_SCENE_DIRTY_SKYBOX_TEXTURE) {
        pt_packed_scene_globals* G = &Scene->Globals;
        texture* Sky = Scene->Root.SkyboxTexture;
        G->SkyboxTextureIndex = GetPackedTextureIndex(Sky);
        if (Sky) {
            vec3 Mean(0, 0, 0);
            float WeightSum = 0.0f;
            for (uint32_t Y = 0; Y < Sky->Height; Y++) {
                float Theta = (0.5f - (Y + 0.5f) / Sky->Height) * PI;
                for (uint32_t X = 0; X < Sky->Width; X++) {
                    float Phi = ((X + 0.5f) / Sky->Width - 0.5f) * TAU;
                    vec4 C = Sky->Pixels[(size_t)Y * Sky->Width + X];
                    float Luminance = dot(vec3(0.2126f, 0.7152f, 0.0722f), C.xyz());
                    float Area = std::cos(Theta);
                    float Weight = Area * Luminance * Luminance;
                    vec3 Direction(std::cos(Theta) * std::cos(Phi), std::cos(Theta) * std::sin(Phi), std::sin(Theta));
                    Mean += Weight * Direction;
                    WeightSum += Weight;
                }
            }
            Mean = Mean / WeightSum;
            float MeanLength = length(Mean);
            vec3 Dir = Mean / MeanLength;
            G->SkyboxMeanDirection[0] = Dir.x; G->SkyboxMeanDirection[1] = Dir.y; G->SkyboxMeanDirection[2] = Dir.z;
            G->SkyboxConcentration = MeanLength * (3.0f - MeanLength * MeanLength) / (1 - MeanLength * MeanLength);
        }
        DirtyFlags |= PT_SCENE_DIRTY_GLOBALS;
    }

    // Globals (scene.cpp:1607-1616).
    if (DirtyFlags & PT_SCENE_DIRTY_GLOBALS) {
        pt_packed_scene_globals* G = &Scene->Globals;
        G->SkyboxSamplingProbability = Scene->Root.SkyboxSamplingProbability;
        G->SkyboxBrightness = Scene->Root.SkyboxBrightness;
        G->SceneScatterRate = Scene->Root.ScatterRate;
        G->ShapeCount = static_cast<uint32_t>(Scene->ShapePack.size());
    }

    Scene->DirtyFlags = 0;
    return DirtyFlags;
}

void GetScenePacks(scene* Scene, pt_scene_packs* Out)
{
    Out->globals = &Scene->Globals;
    Out->textures = Scene->TexturePack.data();
    Out->texture_count = (uint32_t)Scene->TexturePack.size();
    Out->material_data = Scene->MaterialAttributePack.data();
    Out->material_word_count = (uint32_t)Scene->MaterialAttributePack.size();
    Out->shapes = Scene->ShapePack.data();
    Out->shape_count = (uint32_t)Scene->ShapePack.size();
    Out->shape_nodes = Scene->ShapeNodePack.data();
    Out->shape_node_count = (uint32_t)Scene->ShapeNodePack.size();
    Out->mesh_faces = Scene->MeshFacePack.data();
    Out->mesh_face_count = (uint32_t)Scene->MeshFacePack.size();
    Out->mesh_vertices = Scene->MeshVertexPack.data();
    Out->mesh_vertex_count = (uint32_t)Scene->MeshVertexPack.size();
    Out->mesh_nodes = Scene->MeshNodePack.data();
    Out->mesh_node_count = (uint32_t)Scene->MeshNodePack.size();
    Out->cameras = Scene->CameraPack.data();
    Out->camera_count = (uint32_t)Scene->CameraPack.size();
    Out->atlas = Scene->AtlasFlat.data();
    Out->atlas_width = Scene->AtlasWidth;
    Out->atlas_height = Scene->AtlasHeight;
    Out->atlas_layer_count = (uint32_t)(Scene->AtlasFlat.size() / ((size_t)Scene->AtlasWidth * Scene->AtlasHeight * 4));
}

}  // namespace pth
