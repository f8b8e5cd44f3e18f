// traverse.hpp — Trace() on the device (scene.glsl.inc:304-611): the
// per-lane traversal state machine shared by the extend kernel (kernels.hip)
// and the preview kernel (preview.hip).
#pragma once

#include "pt_device.hpp"

namespace ptd {

#define PT_LDS __attribute__((address_space(3)))
#define PT_GLOBAL __attribute__((address_space(1)))
typedef float f32x4 __attribute__((ext_vector_type(4)));
PT_DEV float4 F4(f32x4 v) { return make_float4(v.x, v.y, v.z, v.w); }


// --- traversal stack: LDS columns + global spill ----------------------------

template <bool SPILL, int CAP, class E = uint32_t>
struct tstack {
    E* lds;               // &smem[tid]; entry i at lds[i * 256] (E: u32, or u16 when every entry fits)
    uint32_t* spill;      // &spill[thread]; entry i (>= CAP) at spill[(i - CAP) * stride]
    uint32_t stride;
    // LDS node cache (dscene::node_cache): BLAS nodes [0, ncn) at nc[2 * node]
    // (a block-wide copy of the scene's first ncn nodes); ncn = 0: none.
    const float4* nc = nullptr;
    uint32_t ncn = 0;
    PT_DEV void put(uint32_t i, uint32_t v)
    {
        if (!SPILL || i < CAP) lds[i * 256] = (E)v;
        else spill[(i - CAP) * stride] = v;
    }
    PT_DEV uint32_t get(uint32_t i) const
    {
        if (!SPILL || i < CAP) return lds[i * 256];
        return spill[(i - CAP) * stride];
    }
};

// --- traversal ------------------------------------------------------------------
//
// Trace() (scene.glsl.inc:468-611) as a resumable state machine: every loop
// iteration advances each active lane by ONE node of its own traversal, in
// exactly the reference's order (near-first children, LIFO Stack[32] per
// level, IntersectShape at TLAS leaves, IntersectMeshNode for mesh instances),
// so every ray reaches the same closest hit bit for bit.  One flat loop over
// both levels keeps a single loop-carried state (no nested divergent loops).

struct lane_state {
    pt3 O, V, Y;         // current-level ray (world at TLAS level, object space
                         // inside a mesh) and its reciprocal velocity
    float Time;          // Hit.Time
    uint32_t Shape;      // Hit.ShapeIndex (0xFFFFFFFE = face of the current mesh)
    uint32_t Prim;       // Hit.PrimitiveIndex
    pt3 C;               // Hit.PrimitiveCoordinates
    uint32_t na, nb;     // node being processed: TLAS {ChildNodeIndices, ShapeIndex},
                         // BLAS {FaceBeginOrNodeIndex, FaceEndIndex}
    uint32_t dT, dB;     // TLAS / BLAS stack depths (<= 32 each)
    uint32_t blas;       // shape index of the mesh being traversed, NONE at TLAS level
    bool exact;          // fast exact slab division applies to the current-level ray
    uint32_t HA, HB;     // hit's mesh face vertex indices, 3 x 21 bits (PackVertexIndices);
                         // an analytic shape's hit: HA = C.x (CompactHit)
};

PT_DEV void SetLevelRay(const dscene& S, lane_state& L, pt3 O, pt3 V)
{
    L.O = O;
    L.V = V;
    L.exact = S.fast_div && FastDivRay(O, V);
    L.Y = v3(1.0f / V.x, 1.0f / V.y, 1.0f / V.z);
}

PT_DEV void LaneBegin(const dscene& S, lane_state& L, pt3 O, pt3 V, float Duration)
{
    L.Time = Duration;
    L.Shape = SHAPE_INDEX_NONE;
    L.Prim = 0;
    L.C = v3s(0);
    L.HA = 0;
    L.HB = 0;
    L.dT = 0;
    L.dB = 0;
    L.blas = SHAPE_INDEX_NONE;
    L.na = __float_as_uint(S.shape_nodes[0].w);
    L.nb = __float_as_uint(S.shape_nodes[1].w);
    if (L.na != 0) {
        SetLevelRay(S, L, O, V);
    } else {
        // The TLAS root is a shape leaf (a one-shape scene): the first step
        // transforms the ray into the shape's space and sets that level's
        // reciprocal; the world-space one would never be read.
        L.O = O;
        L.V = V;
        L.exact = false;
        asm("" : "=v"(L.Y.x), "=v"(L.Y.y), "=v"(L.Y.z));
    }
}

// IntersectShape for the analytic shapes (scene.glsl.inc:413-465).
PT_DEV void IntersectAnalytic(int32_t Type, pt3 O, pt3 V, uint32_t ShapeIndex, lane_state& L)
{
    if (Type == PT_SHAPE_TYPE_PLANE) {
        float T = -O.z / V.z;
        if (T < 0 || T > L.Time) return;
        L.Time = T;
        L.Shape = ShapeIndex;
        L.Prim = 0;
        L.C = O + V * T;
        L.HA = __float_as_uint(L.C.x);
        L.HB = 0;
    } else if (Type == PT_SHAPE_TYPE_SPHERE) {
        float Vv = dot(V, V);
        float P = dot(O, V);
        float Q = dot(O, O) - 1.0f;
        float D2 = P * P - Q * Vv;
        if (D2 < 0) return;
        float D = pt_sqrt(D2);
        if (D < P) return;
        float S0 = -P - D;
        float S1 = -P + D;
        float Sv = S0 < 0 ? S1 : S0;
        if (Sv < 0 || Sv > Vv * L.Time) return;
        L.Time = Sv / Vv;
        L.Shape = ShapeIndex;
        L.Prim = 0;
        L.C = O + V * L.Time;
        L.HA = __float_as_uint(L.C.x);
        L.HB = 0;
    } else if (Type == PT_SHAPE_TYPE_CUBE) {
        pt3 Mn = (v3s(-1) - O) / V;
        pt3 Mx = (v3s(+1) - O) / V;
        pt3 E = vmin(Mn, Mx);
        pt3 Lt = vmax(Mn, Mx);
        float T0 = pt_max(pt_max(E.x, E.y), E.z);
        float T1 = pt_min(pt_min(Lt.x, Lt.y), Lt.z);
        if (T1 < T0) return;
        if (T1 <= 0) return;
        float T = T0 < 0 ? T1 : T0;
        if (T >= L.Time) return;
        L.Time = T;
        L.Shape = ShapeIndex;
        L.Prim = 0;
        L.C = O + V * T;
        L.HA = __float_as_uint(L.C.x);
        L.HB = 0;
    }
}

// IntersectMeshFace (scene.glsl.inc:304-334) on the lane's object-space ray.
// The device face array holds {Position0, Edge1, Edge2} (dscene::mesh_faces):
// the edges are the reference's `Position1 - Position0`, `Position2 -
// Position0`, subtracted once on the host at upload in the same IEEE
// arithmetic, so every later operation sees identical operands.
// The test itself: miss flag, T and the coordinates U, W; L is only read.
// A face's three vertex indices in 64 bits (21 bits each; dscene::vidx21
// scenes, whose vertex count fits): the hit record carries them to shade,
// which then reads the vertices without first reading the face.
PT_DEV void PackVertexIndices(uint32_t v0, uint32_t v1, uint32_t v2, uint32_t& A, uint32_t& B)
{
    A = v0 | (v1 << 21);
    B = (v1 >> 11) | (v2 << 10);
}

PT_DEV void UnpackVertexIndices(uint32_t A, uint32_t B, uint32_t& v0, uint32_t& v1, uint32_t& v2)
{
    v0 = A & 0x1FFFFFu;
    v1 = (A >> 21) | ((B & 0x3FFu) << 11);
    v2 = B >> 10;
}

PT_DEV bool FaceTest(const dscene& S, uint32_t F, const lane_state& L, bool valid, float& T, float& U, float& W,
                     uint32_t& VA, uint32_t& VB)
{
    // valid == false (an empty leaf): face 0 is read and the test forced to
    // miss, instead of a branch around the call.
    uint32_t Fl = valid ? F : 0u;
    const float4* Fp = S.mesh_faces + 3 * (size_t)Fl;   // one address, immediate offsets
    float4 a = Fp[0], b = Fp[1], c = Fp[2];
    pt3 P0 = xyz(a);
    pt3 Edge1 = xyz(b);
    pt3 Edge2 = xyz(c);
    PackVertexIndices(__float_as_uint(a.w), __float_as_uint(b.w), __float_as_uint(c.w), VA, VB);
    // Every quantity is evaluated with the reference's operations and
    // operand order; its early returns become one predicate (no value
    // depends on which test failed first), so the exits collapse into a
    // single select.
    pt3 RCE2 = cross(L.V, Edge2);
    float Det = dot(Edge1, RCE2);
    float InvDet = 1.0f / Det;
    pt3 Sv = L.O - P0;
    U = InvDet * dot(Sv, RCE2);
    pt3 SCE1 = cross(Sv, Edge1);
    W = InvDet * dot(L.V, SCE1);
    T = InvDet * dot(Edge2, SCE1);
    return (pt_abs(Det) < PT_EPSILON) | (U < 0) | (U > 1) | (W < 0) | (U + W > 1) | (T < 0) | (T > L.Time) | !valid;
}

PT_DEV void LaneMeshFace(const dscene& S, uint32_t F, lane_state& L, bool valid = true)
{
    float T, U, W;
    uint32_t VA, VB;
    bool miss = FaceTest(S, F, L, valid, T, U, W, VA, VB);
    // Selects, not a branch: the hit registers are updated in place (a
    // conditional update made the compiler keep and copy a second set).
    L.Time = miss ? L.Time : T;
    L.Shape = miss ? L.Shape : 0xFFFFFFFEu;
    L.Prim = miss ? L.Prim : F;
    L.HA = miss ? L.HA : VA;
    L.HB = miss ? L.HB : VB;
    L.C = v3(miss ? L.C.x : 1 - U - W, miss ? L.C.y : U, miss ? L.C.z : W);
}

// Traversal statistics hooks: no-ops in the render kernel, counters in the
// diagnostic instantiation (ptExtendStats).
struct no_stats {
    PT_DEV void face_step(bool) {}
    PT_DEV void coherence(uint32_t) {}
    PT_DEV void node(bool) {}
    PT_DEV void step() {}
    PT_DEV void internal() {}
    PT_DEV void leaf(uint32_t) {}
    PT_DEV void shape() {}
    PT_DEV void pop() {}
};
struct lane_stats {
    uint32_t steps = 0, internals = 0, leaves = 0, faces = 0, shapes = 0, pops = 0;
    // Wave coherence of internal BLAS steps: wave steps by the number of
    // distinct nodes among the lanes taking the step {1, 2, 3-4, 5-8, >8},
    // counted on the first such lane.
    uint32_t uniq[5] = {0, 0, 0, 0, 0};
    PT_DEV void coherence(uint32_t index)
    {
        uint64_t act = __ballot(1);
        uint32_t first = (uint32_t)__ffsll((long long)act) - 1u;
        uint32_t lane = __lane_id();
        uint32_t u = 0;
        bool done = false;
        for (;;) {
            uint64_t m = __ballot(!done);
            if (m == 0) break;
            uint32_t f = (uint32_t)__shfl(index, (int)(__ffsll((long long)m) - 1), 64);
            if (!done && index == f) done = true;
            u++;
        }
        if (lane == first) uniq[u == 1 ? 0 : u == 2 ? 1 : u <= 4 ? 2 : u <= 8 ? 3 : 4]++;
    }
    PT_DEV void node(bool) {}
    PT_DEV void step() { steps++; }
    PT_DEV void internal() { internals++; }
    PT_DEV void leaf(uint32_t n) { leaves++; faces += n; }
    // FACE_STEP leaves: one call per face; the leaf counts once, on its last.
    PT_DEV void face_step(bool last) { faces++; leaves += last; }
    PT_DEV void shape() { shapes++; }
    PT_DEV void pop() { pops++; }
};

// BLAS stack entries.  When the scene allows (dscene::blas_words, checked on
// the host) an entry is the pushed node's own index words, packed: leaf ->
// 1<<31 | count<<26 | first face (count <= 31, first face < 2^26); internal ->
// child-pair index (< 2^31).  A pop is then an LDS read only.  Otherwise the
// entry is the node index and a pop reloads its words (two global loads).
PT_DEV uint32_t PackBlasEntry(uint32_t w0, uint32_t w1)
{
    return w1 > 0 ? (0x80000000u | ((w1 - w0) << 26) | w0) : w0;
}

PT_DEV void UnpackBlasEntry(uint32_t e, uint32_t& na, uint32_t& nb)
{
    if (e >> 31) {
        na = e & 0x03FFFFFFu;
        nb = na + ((e >> 26) & 31u);
    } else {
        na = e;
        nb = 0;
    }
}

// 16-bit format (dscene::blas_words == 2; the host checks that every entry
// fits): leaf -> 1<<15 | count<<F | first face, internal -> child-pair index
// (< 2^15), F = dscene::blas_firstbits.  Half-width LDS stack columns double
// the blocks a CU can hold (the stack is the extend kernel's LDS).
PT_DEV uint32_t PackBlasEntry16(uint32_t w0, uint32_t w1, uint32_t F)
{
    return w1 > 0 ? (0x8000u | ((w1 - w0) << F) | w0) : w0;
}

PT_DEV void UnpackBlasEntry16(uint32_t e, uint32_t F, uint32_t& na, uint32_t& nb)
{
    uint32_t first = e & ((1u << F) - 1u);
    bool leaf = (e & 0x8000u) != 0;
    na = leaf ? first : e;
    nb = leaf ? first + ((e & 0x7FFFu) >> F) : 0u;
}

// Push / pop encoding by the scene's format.  The extend kernels run format 2
// exactly on a u16 stack (dscene::stack16), so there F2 = (SE is u16) is
// known at compile time; F2_RUNTIME (the preview kernel's u32 stack) checks
// the format.
template <class SE, bool F2_RUNTIME = false>
PT_DEV uint32_t BlasPush(const dscene& S, uint32_t w0, uint32_t w1, uint32_t index)
{
    if (sizeof(SE) == 2 || (F2_RUNTIME && S.blas_words == 2)) return PackBlasEntry16(w0, w1, S.blas_firstbits);
    return S.blas_words ? PackBlasEntry(w0, w1) : index;
}

template <class SE, bool F2_RUNTIME = false>
PT_DEV void BlasPop(const dscene& S, uint32_t E, uint32_t& na, uint32_t& nb)
{
    if (sizeof(SE) == 2 || (F2_RUNTIME && S.blas_words == 2)) {
        UnpackBlasEntry16(E, S.blas_firstbits, na, nb);
    } else if (S.blas_words) {
        UnpackBlasEntry(E, na, nb);
    } else {
        const uint32_t* mesh_words = reinterpret_cast<const uint32_t*>(S.mesh_nodes);
        na = mesh_words[8 * E + 3];
        nb = mesh_words[8 * E + 7];
    }
}

// Hit.SceneComplexity / Hit.MeshComplexity (scene.glsl.inc:117-118): one count
// per Intersect / IntersectMeshNode loop iteration = one LaneStep at that level.
struct complexity_stats {
    uint32_t scene = 0, mesh = 0;
    PT_DEV void coherence(uint32_t) {}
    PT_DEV void face_step(bool last) { mesh += last; }
    PT_DEV void node(bool blas) { if (blas) mesh++; else scene++; }
    PT_DEV void step() {}
    PT_DEV void internal() {}
    PT_DEV void leaf(uint32_t) {}
    PT_DEV void shape() {}
    PT_DEV void pop() {}
};

// Advances one lane by one node.  Returns true when its Trace() is complete.
// Only the two index words of the current node are carried between steps;
// its bounds were already consumed by the parent's box test.
//
// FACE_STEP: a BLAS leaf advances by ONE face per step (na walks up to nb), so
// a divergent wave step costs one face test beside the internal-node lanes'
// box tests instead of the longest leaf's whole face loop.  The faces are
// still tested in the reference's order, each with the Hit.Time left by the
// previous one, and the pop follows the last face, so results are identical.
// The TLAS-level part of a step (scene.glsl.inc:468-520) and the return from
// a finished BLAS (scene.glsl.inc:409-411); rare on mesh scenes, so LaneStep
// runs it as one block after the BLAS work instead of as early exits.
template <bool SPILL, int CAP, class Src, class Stats, class SE>
PT_DEV bool TlasStep(const dscene& S, lane_state& L, tstack<SPILL, CAP, SE>& st, const Src& src, uint32_t slot, Stats& ss)
{
    const uint32_t* mesh_words = reinterpret_cast<const uint32_t*>(S.mesh_nodes);
    const uint32_t* shape_words = reinterpret_cast<const uint32_t*>(S.shape_nodes);
    if (L.blas != SHAPE_INDEX_NONE) {
        // IntersectMeshNode returned; back to the world-space ray for the
        // rest of the shape traversal.
        if (L.Shape == 0xFFFFFFFEu) L.Shape = L.blas;
        L.blas = SHAPE_INDEX_NONE;
        if (L.dT == 0) return true;
        pt3 WO, WV;
        float D;
        src.load(slot, WO, WV, D);
        SetLevelRay(S, L, WO, WV);
    } else {
        // Intersect, one node.
        ss.node(false);
        uint32_t Children = L.na;
        if (Children == 0) {
            ss.shape();
            uint32_t ShapeIndex = L.nb;
            const pt_packed_shape* Shape = &S.shapes[ShapeIndex];
            const float* From = Shape->Transform.From;
            pt3 O = mat4_mul_point(From, L.O);
            pt3 V = mat4_mul_vector(From, L.V);
            int32_t Type = Shape->Type;
            if (Type == PT_SHAPE_TYPE_MESH_INSTANCE) {
                uint32_t Root = Shape->MeshRootNodeIndex;
                SetLevelRay(S, L, O, V);
                L.blas = ShapeIndex;
                L.dB = 0;
                L.na = mesh_words[8 * Root + 3];
                L.nb = mesh_words[8 * Root + 7];
                return false;
            }
            IntersectAnalytic(Type, O, V, ShapeIndex, L);
        } else {
            ss.internal();
            uint32_t IA = Children & 0xFFFF, IB = Children >> 16;
            const float4* Ap = S.shape_nodes + 2 * (size_t)IA;
            const float4* Bp = S.shape_nodes + 2 * (size_t)IB;
            float4 a0 = Ap[0], a1 = Ap[1], b0 = Bp[0], b1 = Bp[1];
            float TA, TB;
            IntersectBoxPair(L.O, L.V, L.Y, L.Time, a0, a1, b0, b1, L.exact, TA, TB);
            // Same decision as the BLAS step (scene.glsl.inc:494-516).
            bool goB = TA > TB;
            bool any = goB | (TA < PT_INFINITY);
            bool push = goB ? (TA < PT_INFINITY) : (TB < PT_INFINITY);
            if (push & (L.dT < 32)) st.put(L.dT++, goB ? IA : IB);
            if (any) {
                L.na = __float_as_uint(goB ? b0.w : a0.w);
                L.nb = __float_as_uint(goB ? b1.w : a1.w);
                return false;
            }
        }
    }
    if (L.dT > 0) {
        ss.pop();
        uint32_t I = st.get(--L.dT);
        L.na = shape_words[8 * I + 3];
        L.nb = shape_words[8 * I + 7];
        return false;
    }
    return true;
}

// Advances one lane by one node.  Returns true when its Trace() is complete.
// Only the two index words of the current node are carried between steps;
// its bounds were already consumed by the parent's box test.
//
// FACE_STEP: a BLAS leaf advances by ONE face per step (na walks up to nb), so
// a divergent wave step costs one face test beside the internal-node lanes'
// box tests instead of the longest leaf's whole face loop.  The faces are
// still tested in the reference's order, each with the Hit.Time left by the
// previous one, and the pop follows the last face, so results are identical.
//
// The BLAS work (IntersectMeshNode, scene.glsl.inc:336-399) has no early
// exit: it ends with the lane either moved to a new node, popped, or handed
// to TlasStep (BLAS finished, or the lane is at the TLAS level).
template <bool SPILL, int CAP, class Src, class Stats = no_stats, bool FACE_STEP = false, class SE = uint32_t>
PT_DEV bool LaneStep(const dscene& S, lane_state& L, tstack<SPILL, CAP, SE>& st, const Src& src, uint32_t slot,
                     Stats& ss)
{
    ss.step();
    bool tlas = L.blas == SHAPE_INDEX_NONE;
    if (FACE_STEP && !tlas) {
        // The divergent part of a BLAS step computes only fresh values (face:
        // miss flag, T, U, W; internal node: TA, TB and the child words); every
        // update of the lane state happens after the join, by selects.  State
        // registers are then written once per step in straight-line code,
        // instead of being copied around the two exec-masked halves.
        const bool face = L.nb > 0;
        // Each half's outputs start undefined (an empty asm defines them: no
        // instruction) and are read only by selects that discard them on the
        // other half's lanes.
        bool fmiss = true;
        float fT, fU, fW, TA, TB;
        uint32_t aw0, aw1, bw0, bw1, fVA, fVB;
        uint32_t pair = L.na;   // child pair whose decision the join applies
        asm("" : "=v"(fT), "=v"(fU), "=v"(fW), "=v"(TA), "=v"(TB), "=v"(fVA), "=v"(fVB));
        asm("" : "=v"(aw0), "=v"(aw1), "=v"(bw0), "=v"(bw1));
        if (face) {
            fmiss = FaceTest(S, L.na, L, L.na < L.nb, fT, fU, fW, fVA, fVB);   // (an empty leaf tests nothing)
            ss.face_step(L.na + 1 >= L.nb);
        } else {
            ss.node(true);
            ss.internal();
            ss.coherence(L.na);
            // The child pair (64 contiguous bytes): from the block's LDS copy
            // of the top pairs when cached (no texture-address work, LDS
            // latency), else from global memory.
            // (Explicit address spaces: the two sides must stay an LDS read
            // and a global load; as generic pointers the compiler merges them
            // into one flat load, which every lane issues through the
            // texture-address path.)
            float4 a0, a1, b0, b1;
            if (L.na < st.ncn) {
                const PT_LDS f32x4* Cp = (const PT_LDS f32x4*)st.nc + 2 * L.na;
                a0 = F4(Cp[0]); a1 = F4(Cp[1]); b0 = F4(Cp[2]); b1 = F4(Cp[3]);
            } else {
                const PT_GLOBAL f32x4* Np = (const PT_GLOBAL f32x4*)S.mesh_nodes + 2 * (size_t)L.na;
                a0 = F4(Np[0]); a1 = F4(Np[1]); b0 = F4(Np[2]); b1 = F4(Np[3]);
            }
            IntersectBoxPair(L.O, L.V, L.Y, L.Time, a0, a1, b0, b1, L.exact, TA, TB);
            aw0 = __float_as_uint(a0.w), aw1 = __float_as_uint(a1.w);
            bw0 = __float_as_uint(b0.w), bw1 = __float_as_uint(b1.w);
        }
        L.Time = fmiss ? L.Time : fT;
        L.Shape = fmiss ? L.Shape : 0xFFFFFFFEu;
        L.Prim = fmiss ? L.Prim : L.na;
        L.HA = fmiss ? L.HA : fVA;
        L.HB = fmiss ? L.HB : fVB;
        L.C = v3(fmiss ? L.C.x : 1 - fU - fW, fmiss ? L.C.y : fU, fmiss ? L.C.z : fW);
        // Internal node: the reference's three-way decision (scene.glsl.inc:366-392).
        // (The child set aside is pushed iff its own time is finite: one
        // select of the time, not of two flags; `moved` as mask logic, not a
        // select between the halves' flags, which the compiler lowered to
        // exec-mask branches.)
        bool goB = TA > TB;
        float Tfar = goB ? TA : TB;
        bool push = !face & (Tfar < PT_INFINITY);
        bool moved = (face & (L.na + 1 < L.nb)) | (!face & (goB | (TA < PT_INFINITY)));
        if (push & (L.dB < 32)) {
            st.put(L.dT + L.dB++, BlasPush<SE>(S, goB ? aw0 : bw0, goB ? aw1 : bw1, pair + (goB ? 0u : 1u)));
        }
        uint32_t na = face ? L.na + 1 : (goB ? bw0 : aw0);
        uint32_t nb = face ? L.nb : (goB ? bw1 : aw1);
        if (!moved) {
            if (L.dB > 0) {
                ss.pop();
                BlasPop<SE>(S, st.get(L.dT + --L.dB), na, nb);
            } else {
                tlas = true;
            }
        }
        L.na = na;
        L.nb = nb;
        if (!tlas) return false;
        return TlasStep(S, L, st, src, slot, ss);
    }
    if (!tlas) {
        bool moved = false;
        if (L.nb > 0) {
            if (FACE_STEP) {
                LaneMeshFace(S, L.na, L, L.na < L.nb);   // (an empty leaf tests nothing)
                bool last = ++L.na >= L.nb;
                ss.face_step(last);
                moved = !last;
            } else {
                ss.node(true);
                ss.leaf(L.nb - L.na);
                for (uint32_t F = L.na; F < L.nb; F++) LaneMeshFace(S, F, L);
            }
        } else {
            ss.node(true);
            ss.internal();
            uint32_t Index = L.na;
            ss.coherence(Index);
            const float4* Np = S.mesh_nodes + 2 * (size_t)Index;   // child pair: 64 contiguous bytes
            float4 a0 = Np[0], a1 = Np[1], b0 = Np[2], b1 = Np[3];
            float TA, TB;
            IntersectBoxPair(L.O, L.V, L.Y, L.Time, a0, a1, b0, b1, L.exact, TA, TB);
            // The reference's three-way decision (scene.glsl.inc:366-392) as
            // selects: B strictly closer -> continue with B, set A aside if
            // hit; otherwise continue with A if hit, setting B aside if it
            // was hit too; nothing hit -> pop.
            bool goB = TA > TB;
            moved = goB | (TA < PT_INFINITY);
            bool push = goB ? (TA < PT_INFINITY) : (TB < PT_INFINITY);
            uint32_t aw0 = __float_as_uint(a0.w), aw1 = __float_as_uint(a1.w);
            uint32_t bw0 = __float_as_uint(b0.w), bw1 = __float_as_uint(b1.w);
            if (push & (L.dB < 32)) {
                st.put(L.dT + L.dB++, BlasPush<SE, !FACE_STEP>(S, goB ? aw0 : bw0, goB ? aw1 : bw1, Index + (goB ? 0u : 1u)));
            }
            if (moved) {
                L.na = goB ? bw0 : aw0;
                L.nb = goB ? bw1 : aw1;
            }
        }
        if (!moved) {
            if (L.dB > 0) {
                ss.pop();
                BlasPop<SE, !FACE_STEP>(S, st.get(L.dT + --L.dB), L.na, L.nb);
            } else {
                tlas = true;
            }
        }
    }
    if (!tlas) return false;
    return TlasStep(S, L, st, src, slot, ss);
}

// The compact hit record extend stores for shade: {Time, Shape, z, w} and
// {C.y, C.z}.  In a vidx21 scene z, w are a mesh face's packed vertex indices
// and C.x = 1 - C.y - C.z is re-evaluated by the reader (the face test's own
// expression on the same operands), or for an analytic shape z = C.x;
// otherwise z = Prim, w = C.x.
PT_DEV float4 CompactHit(const lane_state& Ln, bool vidx21)
{
    return make_float4(Ln.Time, __uint_as_float(Ln.Shape), __uint_as_float(vidx21 ? Ln.HA : Ln.Prim),
                       vidx21 ? __uint_as_float(Ln.HB) : Ln.C.x);
}

// Hit attribute reconstruction (scene.glsl.inc:535-608).  Mesh faces: the
// vertex indices come packed in the hit record (vidx21) or from the face.
// uv_if_textured: the caller reads the texture coordinates only through the
// hit material's textures (shade), so a sphere hit on a shape whose material
// samples none (the device shape record's PT_SHAPE_FLAG_UV, loaded with its
// type) leaves them 0 instead of computing them (an atan2: C2 shade -1.2 %,
// C5 -1 %).  Other shapes compute them anyway: skipping a mesh's three
// vertex V loads behind the flag measured C3 shade +1.7 %.  prims false
// (the shade instantiation of a mesh-only scene) compiles out the other
// shape types.
PT_DEV void HitAttributesV(const dscene& S, uint32_t ShapeIndex, bool packed, uint32_t Z, uint32_t Wd, pt3 C,
                           uint32_t& Material, pt3& Normal, pt3& TangentX, pt2& UV, bool uv_if_textured = false,
                           bool prims = true);

PT_DEV void HitAttributes(const dscene& S, uint32_t ShapeIndex, uint32_t Prim, pt3 C, uint32_t& Material, pt3& Normal,
                          pt3& TangentX, pt2& UV)
{
    HitAttributesV(S, ShapeIndex, false, Prim, 0u, C, Material, Normal, TangentX, UV);
}

// From a compact hit record (h = {Time, Shape, z, w}, c = {C.y, C.z}).
PT_DEV void HitAttributesRecord(const dscene& S, uint32_t ShapeIndex, float4 h, float2 c, uint32_t& Material,
                                pt3& Normal, pt3& TangentX, pt2& UV, bool uv_if_textured = false, bool prims = true)
{
    const bool mesh = !prims || S.shapes[ShapeIndex].Type == PT_SHAPE_TYPE_MESH_INSTANCE;
    if (S.vidx21) {
        pt3 C = mesh ? v3(1 - c.x - c.y, c.x, c.y) : v3(h.z, c.x, c.y);
        HitAttributesV(S, ShapeIndex, true, __float_as_uint(h.z), __float_as_uint(h.w), C, Material, Normal, TangentX, UV,
                       uv_if_textured, prims);
    } else {
        HitAttributesV(S, ShapeIndex, false, __float_as_uint(h.z), 0u, v3(h.w, c.x, c.y), Material, Normal, TangentX, UV,
                       uv_if_textured, prims);
    }
}

PT_DEV void HitAttributesV(const dscene& S, uint32_t ShapeIndex, bool packed, uint32_t Z, uint32_t Wd, pt3 C,
                           uint32_t& Material, pt3& Normal, pt3& TangentX, pt2& UV, bool uv_if_textured, bool prims)
{
    UV = v2(0.0f, 0.0f);
    const pt_packed_shape* Shape = &S.shapes[ShapeIndex];
    Material = Shape->MaterialIndex;
    const bool uv = !uv_if_textured || (Shape->Pad0 & PT_SHAPE_FLAG_UV);
    int32_t Type = Shape->Type;
    const float* To = Shape->Transform.To;
    const float* From = Shape->Transform.From;
    // Each shape type yields its object-space normal and tangent; the
    // transforms to world space run once after the join (a wave with
    // spheres, cubes and planes runs them once, not per type).
    // prims false: the scene has mesh instances only (PT_MATS_PRIMS clear).
    const bool mesh = !prims || Type == PT_SHAPE_TYPE_MESH_INSTANCE;
    pt3 N, T = v3s(0.0f);
    if (mesh) {
        uint32_t i0, i1, i2;
        if (packed) {
            UnpackVertexIndices(Z, Wd, i0, i1, i2);
        } else {
            const float4* Fp = S.mesh_faces + 3 * (size_t)Z;   // Z = Prim
            i0 = __float_as_uint(Fp[0].w); i1 = __float_as_uint(Fp[1].w); i2 = __float_as_uint(Fp[2].w);
        }
        // The vertices' normals and UVs come decoded (dscene::vertex_attr:
        // UnpackUnitVector and the half -> float conversions run once per
        // vertex at upload, with the same functions, so the same bits).
        float4 A0 = S.vertex_attr[i0];
        float4 A1 = S.vertex_attr[i1];
        float4 A2 = S.vertex_attr[i2];
        N = SafeNormalize(xyz(A0) * C.x + xyz(A1) * C.y + xyz(A2) * C.z);
        pt2 UV0 = v2(A0.w, S.vertex_v[i0]);
        pt2 UV1 = v2(A1.w, S.vertex_v[i1]);
        pt2 UV2 = v2(A2.w, S.vertex_v[i2]);
        UV = UV0 * C.x + UV1 * C.y + UV2 * C.z;
    } else if (Type == PT_SHAPE_TYPE_PLANE) {
        N = v3(0, 0, 1);
        T = v3(1, 0, 0);
        UV = v2(pt_fract(C.x), pt_fract(C.y));
    } else if (Type == PT_SHAPE_TYPE_SPHERE) {
        pt3 P = C;
        N = P;
        T = cross(P, v3(-P.y, P.x, 0));
        if (uv) {
            float U = (pt_atan2(P.y, P.x) + PT_PI) / PT_TAU;
            float W = (P.z + 1.0f) / 2.0f;
            UV = v2(U, W);
        }
    } else {
        pt3 P = C;
        pt3 Q = vabs(P);
        if (Q.x >= Q.y && Q.x >= Q.z) {
            float Sg = pt_sign(P.x);
            N = v3(Sg, 0, 0); T = v3(0, Sg, 0);
            UV = 0.5f * v2(1.0f + P.y, 1.0f + P.z);
        } else if (Q.y >= Q.x && Q.y >= Q.z) {
            float Sg = pt_sign(P.y);
            N = v3(0, Sg, 0); T = v3(0, 0, Sg);
            UV = 0.5f * v2(1.0f + P.x, 1.0f + P.z);
        } else {
            float Sg = pt_sign(P.z);
            N = v3(0, 0, Sg); T = v3(Sg, 0, 0);
            UV = 0.5f * v2(1.0f + P.x, 1.0f + P.y);
        }
    }
    Normal = TransformNormal(N, From);
    TangentX = mesh ? ComputeTangentVector(Normal) : TransformDirection(T, To);
}

}  // namespace ptd
