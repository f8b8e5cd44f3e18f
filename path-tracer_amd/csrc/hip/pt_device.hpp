// pt_device.hpp — device-side integrator functions for gfx950.
//
// GPU restatement of the reference's device code (src/scene/scene.glsl.inc,
// src/scene/basic_*.glsl.inc, src/core/common.glsl.inc,
// src/core/spectrum.glsl.inc, src/integrator/basic_scatter.glsl) under the
// numerics convention of include/pt_fp.h.  Scene data is read through
// 16-byte vector loads; the traversal stack lives in LDS with a global
// spill area for depth beyond its LDS capacity (PT_EXTEND_CAP, kernels.hip).
#pragma once

#include <hip/hip_runtime.h>
#include "../../../include/pt_glsl.h"
#include "../../../include/pt_packed.h"

#define PT_DEV __device__ __forceinline__

namespace ptd {

constexpr uint32_t SHAPE_INDEX_NONE = 0xFFFFFFFFu;
constexpr uint32_t TEXTURE_INDEX_NONE = 0xFFFFFFFFu;
constexpr uint32_t PT_SHAPE_FLAG_UV = 1u;   // pt_packed_shape::Pad0 on the device (runtime.hip)

// Device view of the packed scene (the 11 descriptor bindings of
// scene.glsl.inc:121-179).
struct dscene {
    pt_packed_scene_globals g;
    const pt_packed_texture* textures;
    const uint32_t* material;
    const pt_packed_shape* shapes; // device copy: Pad0 bit 0 = the shape's material samples a texture
                                   // (shade needs the hit's UV; PT_SHAPE_FLAG_UV)
    const float4* shape_nodes;     // 2 x float4 per node
    const float4* mesh_faces;      // 3 x float4 per face: {Position0, Edge1, Edge2}, .w = vertex indices
    const uint2* mesh_vertices;
    const float4* vertex_attr;     // per vertex, decoded once at upload (vertex_decode_kernel):
                                   // {UnpackUnitVector(PackedNormal), U as float}
    const float* vertex_v;         // per vertex: V as float
    const float4* mesh_nodes;      // 2 x float4 per node
    const pt_packed_camera* cameras;
    const float4* atlas;
    uint32_t atlas_w, atlas_h, atlas_layers;
    uint32_t atlas_tiled;          // atlas stored in 4x2-texel blocks (AtlasIndex), not row-major
    uint32_t fast_div;             // every BVH box coordinate is 0 or in [2^-50, 2^40] (IntersectBoundingBox)
    uint32_t blas_words;           // BLAS stack entry format: 0 node index, 1 packed words (PackBlasEntry),
                                   // 2 16-bit packed words (PackBlasEntry16, blas_firstbits)
    uint32_t blas_firstbits;       // format 2: bits of a leaf's first face index (count above them)
    uint32_t stack16;              // every stack entry fits 16 bits: extend runs the u16-stack kernel
    uint32_t mat_classes;          // shapes use more than one material type: extend classes hits by type
    uint32_t vidx21;               // every vertex index fits 21 bits: hit records carry a face's vertex indices
    float vmf_inv_kappa, vmf_exp_m2k, vmf_norm;   // VmfConstants(g.SkyboxConcentration), set on upload
    float sky_flat;                // SampleParametricSpectrum((0, 0, 100), L) for any finite L (SkyFlat)
    uint32_t node_cache;           // BLAS nodes [0, node_cache) are the top child pairs the extend kernel
                                   // keeps in LDS (NodeCacheLayout, runtime.hip); 0: no cache
};

// LDS node cache of the extend kernel: this many BLAS child pairs (64 B
// each), the top levels of the scene's BLASes, are loaded into LDS once per
// block (10 KB beside the 10 KB u16 stack: 8 blocks per CU, the occupancy the
// kernel's VGPRs allow).
#ifndef PT_NODE_CACHE_PAIRS
#define PT_NODE_CACHE_PAIRS 160
#endif

struct ray { pt3 Origin; pt3 Velocity; float Duration; };
struct medium { uint32_t Priority; pt4 IOR, AbsorptionRate, ScatteringRate; float ScatteringAnisotropy; };

PT_DEV pt3 xyz(float4 a) { return v3(a.x, a.y, a.z); }

// --- common.glsl.inc ------------------------------------------------------

PT_DEV pt3 TransformNormal(pt3 N, const float* From) { return normalize(vec_mul_mat4(N, From)); }
PT_DEV pt3 TransformDirection(pt3 D, const float* To) { return normalize(mat4_mul_vector(To, D)); }

PT_DEV pt3 SafeNormalize(pt3 V)
{
    float LenSq = dot(V, V);
    if (LenSq < 1e-12f) return v3(0, 0, 1);
    return V / pt_sqrt(LenSq);
}

PT_DEV pt3 ComputeTangentVector(pt3 N)
{
    pt3 V = pt_abs(N.x) < 0.9f ? v3(1, 0, 0) : v3(0, 1, 0);
    return normalize(cross(V, N));
}

PT_DEV void ComputeCoordinateFrame(pt3 Z, pt3& X, pt3& Y)
{
    pt3 V = pt_abs(Z.x) < 0.9f ? v3(1, 0, 0) : v3(0, 1, 0);
    X = normalize(cross(V, Z));
    Y = cross(X, Z);
}

PT_DEV uint32_t PackUnitVector(pt3 V)
{
    float s = 1.0f / (pt_abs(V.x) + pt_abs(V.y) + pt_abs(V.z));
    float Px = V.x * s, Py = V.y * s;
    if (V.z <= 0.0f) {
        float Sx = Px >= 0.0f ? 1.0f : -1.0f, Sy = Py >= 0.0f ? 1.0f : -1.0f;
        float Nx = (1.0f - pt_abs(Py)) * Sx;
        float Ny = (1.0f - pt_abs(Px)) * Sy;
        Px = Nx; Py = Ny;
    }
    return pt_pack_snorm16(Px) | (pt_pack_snorm16(Py) << 16);
}

PT_DEV pt3 UnpackUnitVector(uint32_t P)
{
    float Px = pt_unpack_snorm16(P & 0xFFFFu), Py = pt_unpack_snorm16(P >> 16);
    float Z = 1.0f - pt_abs(Px) - pt_abs(Py);
    if (Z < 0.0f) {
        float Sx = Px >= 0.0f ? 1.0f : -1.0f, Sy = Py >= 0.0f ? 1.0f : -1.0f;
        float Nx = (1.0f - pt_abs(Py)) * Sx;
        float Ny = (1.0f - pt_abs(Px)) * Sy;
        Px = Nx; Py = Ny;
    }
    return normalize(v3(Px, Py, Z));
}

// Correctly rounded a / b given y = RN(1/b): q = RN(a*y), one FMA residual
// correction (Markstein) -> RN(a/b).  Outside the guarded range (b or a/b
// beyond 2^+-100, b = 0, a = 0, NaN) it falls back to IEEE division, so the
// result is always bit-identical to a / b; ptCheckFastDivision verifies this
// over >10^9 operand pairs on the device.  (The slab test uses the same
// correction without a per-quotient guard: FastQuot below.)
PT_DEV float RecipForDiv(float b)
{
    float m = pt_abs(b);
    return (m >= 0x1p-100f && m <= 0x1p100f) ? 1.0f / b : pt_u2f(0x7fc00000u);
}

PT_DEV float XDiv(float a, float b, float y)
{
    float q = a * y;
    float r = __builtin_fmaf(-q, b, a);
    float q1 = __builtin_fmaf(r, y, q);
    float m = pt_abs(q1);
    if (!(m >= 0x1p-100f && m <= 0x1p100f)) q1 = a / b;
    return q1;
}

// Operands are results of arithmetic (never signalling NaNs), so minnum /
// maxnum lower to bare v_min/v_max (+ v_min3/v_max3) with no canonicalising
// moves; for a quiet NaN they keep the other operand, as fminf/fmaxf do on
// the host.
PT_DEV float HwMin(float a, float b) { return __builtin_fminf(a, b); }
PT_DEV float HwMax(float a, float b) { return __builtin_fmaxf(a, b); }
PT_DEV float HwMin3(float a, float b, float c) { return __builtin_fminf(__builtin_fminf(a, b), c); }
PT_DEV float HwMax3(float a, float b, float c) { return __builtin_fmaxf(__builtin_fmaxf(a, b), c); }

// RN(1/d) from the hardware reciprocal (1 ulp) and one FMA Newton step.
// Bit-identical to the IEEE quotient 1.0f / d for every float with
// 2^-126 <= |d| < 2^126 (all 2^32 bit patterns checked on the device:
// ptCheckFastReciprocal, tests/test_gpu_parity.py); callers keep IEEE
// division outside that range.
PT_DEV float FastRcp(float d)
{
    float y = __builtin_amdgcn_rcpf(d);
    float e = __builtin_fmaf(-d, y, 1.0f);
    return __builtin_fmaf(e, y, y);
}

// Not used by the traversal: it measured 1 % slower on C3 extend than the
// IEEE division sequence (round 2); ptCheckFastReciprocal keeps
// its bit-equality checked.

PT_DEV bool FastRcpRange(float d)
{
    float m = pt_abs(d);
    return (m >= 0x1p-126f) & (m < 0x1p126f);
}


// Exact fast slab division.  With y = RN(1/b), q = RN(a*y), r = fma(-q,b,a),
// q' = fma(r,y,q) equals IEEE a/b whenever r is exact and q, r*y, q' stay
// normal (Markstein).  That holds for every plane of every box if
//   * every box coordinate and ray-origin component is 0 or has magnitude in
//     [2^-50, 2^40]  ->  every nonzero a = Min - O has |a| >= 2^-73, |a| <= 2^41
//   * every ray-velocity component has magnitude in [2^-59, 2^27]
// so |a/b| lies in [2^-100, 2^100] and r is exact (|a| >= 2^-103).  a = 0
// gives q' = +-0, whose sign may differ from IEEE's; the slab test only
// compares its quotients, where -0 == +0.  The box-coordinate condition is
// checked once per scene on the host (dscene::fast_div), the ray condition
// once per ray and traversal level (FastDivRay); rays outside it take IEEE
// division.  No NaN reaches the fast path, so plain hardware min/max give the
// same comparisons as fminf/fmaxf.
PT_DEV bool FastDivRay(pt3 O, pt3 V)
{
    bool ok = true;
#define PT_CHECK_O(c) { float m = pt_abs(c); ok &= (m == 0.0f) | ((m >= 0x1p-50f) & (m <= 0x1p40f)); }
#define PT_CHECK_V(c) { float m = pt_abs(c); ok &= (m >= 0x1p-59f) & (m <= 0x1p27f); }
    PT_CHECK_O(O.x) PT_CHECK_O(O.y) PT_CHECK_O(O.z)
    PT_CHECK_V(V.x) PT_CHECK_V(V.y) PT_CHECK_V(V.z)
#undef PT_CHECK_O
#undef PT_CHECK_V
    return ok;
}

PT_DEV float FastQuot(float a, float b, float y)
{
    float q = a * y;
    float r = __builtin_fmaf(-q, b, a);
    return __builtin_fmaf(r, y, q);
}

// Slab test (common.glsl.inc:153-185) with IEEE division (Min - O) / V, the
// numerics convention of SURVEY.md §7/§8(c).  `exact`: the
// lane's ray satisfies FastDivRay and the scene's boxes the coordinate
// condition, so FastQuot gives the IEEE quotients; otherwise true division.
// With true division a zero velocity component and a plane through the
// origin give 0 / 0 = NaN, which minnum / maxnum drop as fminf / fmaxf do.
PT_DEV float SlabEntry(float ax, float ay, float az, float bx, float by, float bz, float Reach)
{
    float EntryT = HwMax3(HwMin(ax, bx), HwMin(ay, by), HwMin(az, bz));
    float ExitT = HwMin3(HwMax(ax, bx), HwMax(ay, by), HwMax(az, bz));
    bool miss = (ExitT < EntryT) | (ExitT <= 0.0f) | (EntryT >= Reach);
    return miss ? PT_INFINITY : EntryT;
}

PT_DEV float IntersectBoundingBox(pt3 O, pt3 V, pt3 Y, float Reach, float4 MinAndX, float4 MaxAndX, bool exact)
{
    pt3 A = xyz(MinAndX) - O, B = xyz(MaxAndX) - O;
    if (exact)
        return SlabEntry(FastQuot(A.x, V.x, Y.x), FastQuot(A.y, V.y, Y.y), FastQuot(A.z, V.z, Y.z),
                         FastQuot(B.x, V.x, Y.x), FastQuot(B.y, V.y, Y.y), FastQuot(B.z, V.z, Y.z), Reach);
    return SlabEntry(A.x / V.x, A.y / V.y, A.z / V.z, B.x / V.x, B.y / V.y, B.z / V.z, Reach);
}

// Both child boxes of an internal node under one `exact` branch (one
// divergent branch per node instead of one per box).
PT_DEV void IntersectBoxPair(pt3 O, pt3 V, pt3 Y, float Reach, float4 a0, float4 a1, float4 b0, float4 b1, bool exact,
                             float& TA, float& TB)
{
    if (exact) {
        TA = IntersectBoundingBox(O, V, Y, Reach, a0, a1, true);
        TB = IntersectBoundingBox(O, V, Y, Reach, b0, b1, true);
    } else {
        TA = IntersectBoundingBox(O, V, Y, Reach, a0, a1, false);
        TB = IntersectBoundingBox(O, V, Y, Reach, b0, b1, false);
    }
}

struct rng {
    uint32_t State;
    PT_DEV float R01() { return pt_random01(&State); }
};

PT_DEV pt2 RandomPointOnDisk(rng& G)
{
    float R = pt_sqrt(G.R01());
    float Theta = G.R01() * PT_TAU;
    return R * v2(pt_cos(Theta), pt_sin(Theta));
}

PT_DEV pt3 RandomDirection(rng& G)
{
    float Z = 2 * G.R01() - 1;
    float R = pt_sqrt(1 - Z * Z);
    float Phi = PT_TAU * G.R01();
    return v3(R * pt_cos(Phi), R * pt_sin(Phi), Z);
}

// The sky lobe's Kappa-only factors (common.glsl.inc:222-276), evaluated once
// per scene upload on the host with the same pt_fp.h functions (IEEE f32, the
// same FMA polynomials), so the per-hit expressions below see the same bits
// as the inline ones of the reference restatement.
struct vmf_consts {
    float inv_kappa;   // 1 / Kappa
    float exp_m2k;     // exp(-2 Kappa)
    float norm;        // Kappa / (2 pi (1 - exp(-2 Kappa)))
};
PT_HD vmf_consts VmfConstants(float Kappa)
{
    vmf_consts c;
    c.inv_kappa = 1 / Kappa;
    c.exp_m2k = pt_exp(-2 * Kappa);
    c.norm = Kappa / (2 * PT_PI * (1 - pt_exp(-2 * Kappa)));
    return c;
}

PT_DEV pt3 RandomVonMisesFisher(rng& G, const vmf_consts& K, pt3 Mu)
{
    float Xi = G.R01();
    float Z = 1 + K.inv_kappa * pt_log(Xi + (1 - Xi) * K.exp_m2k);
    float R = pt_sqrt(1 - Z * Z);
    float Phi = G.R01() * PT_TAU;
    pt3 V = v3(R * pt_cos(Phi), R * pt_sin(Phi), Z);
    pt3 MuX, MuY;
    ComputeCoordinateFrame(Mu, MuX, MuY);
    return SafeNormalize(V.x * MuX + V.y * MuY + V.z * Mu);
}

PT_DEV float VonMisesFisherPDF(float Kappa, const vmf_consts& K, pt3 Mu, pt3 Direction)
{
    if (Kappa < PT_EPSILON) return 1.0f / (4 * PT_PI);
    return K.norm * pt_exp(Kappa * (dot(Mu, Direction) - 1.0f));
}

PT_DEV pt3 SampleDirectionHG(float Anisotropy, float U1, float U2)
{
    float Z;
    if (pt_abs(Anisotropy) < 1e-3f) {
        Z = 1 - 2 * U1;
    } else {
        float G = Anisotropy;
        float S = (1 - G * G) / (1 + G - 2 * G * U1);
        Z = -(1 + G * G - S * S) / (2 * G);
    }
    float R = pt_sqrt(1 - Z * Z);
    float Phi = U2 * PT_TAU;
    return v3(R * pt_cos(Phi), R * pt_sin(Phi), Z);
}

PT_DEV pt2 GGXRoughnessAlpha(float Roughness, float Anisotropy)
{
    float R = Roughness;
    float S = 1 - Anisotropy;
    float AlphaX = R * R * pt_sqrt(2 / (1 + S * S));
    return v2(AlphaX, S * AlphaX);
}

PT_DEV float GGXSmithG1(pt3 D, pt2 A)
{
    pt3 DSq = D * D;
    if (DSq.z < PT_EPSILON) return 0.0f;
    pt2 ASq = A * A;
    float T = dot(ASq, v2(DSq.x, DSq.y)) / DSq.z;
    return 2.0f / (1.0f + pt_sqrt(1.0f + T));
}

PT_DEV pt3 GGXVisibleNormal(pt3 D, pt2 A, float U1, float U2)
{
    pt3 Vz = SafeNormalize(v3(A.x * D.x, A.y * D.y, D.z));
    float LengthSq = dot(v2(Vz.x, Vz.y), v2(Vz.x, Vz.y));
    pt3 Vx = LengthSq > 0 ? v3(-Vz.y, Vz.x, 0) / pt_sqrt(LengthSq) : v3(1, 0, 0);
    pt3 Vy = cross(Vz, Vx);
    float R = pt_sqrt(U1);
    float Phi = PT_TAU * U2;
    float S = 0.5f * (1.0f + Vz.z);
    float Tx = R * pt_cos(Phi);
    float Ty = (1.0f - S) * pt_sqrt(1.0f - Tx * Tx) + S * R * pt_sin(Phi);
    float Tz = pt_sqrt(pt_max(0.0f, 1.0f - Tx * Tx - Ty * Ty));
    pt3 N = Tx * Vx + Ty * Vy + Tz * Vz;
    return SafeNormalize(v3(A.x * N.x, A.y * N.y, pt_max(0.0f, N.z)));
}

PT_DEV float GGXDistribution(pt3 N, pt2 A)
{
    pt2 I = v2(1.0f / A.x, 1.0f / A.y);
    float B = dot(N * N, v3(I.x * I.x, I.y * I.y, 1.0f));
    return 1.0f / (PT_PI * A.x * A.y * B * B);
}

PT_DEV pt4 CauchyEmpiricalIOR(float BaseIOR, float AbbeNumber, pt4 Lambda)
{
    const float LC = 656.3f, Ld = 587.6f, LF = 486.1f;
    float B = (BaseIOR - 1) / (AbbeNumber * (1.0f / (LF * LF) - 1.0f / (LC * LC)));
    float A = BaseIOR - B / (Ld * Ld);
    return A + B / (Lambda * Lambda);
}

PT_DEV float ComputeCosThetaRefracted(float Eta, float CosTheta)
{
    float C2 = 1 - Eta * Eta * (1 - CosTheta * CosTheta);
    return -pt_sign(CosTheta) * pt_sqrt(pt_max(C2, 0.0f));
}

PT_DEV pt4 ComputeCosThetaRefracted(pt4 Eta, pt4 CosTheta)
{
    pt4 C2 = 1 - Eta * Eta * (1 - CosTheta * CosTheta);
    return -vsign(CosTheta) * vsqrt(vmax(C2, 0.0f));
}

PT_DEV float FresnelDielectric(float Eta, float C1, float C2)
{
    float Ks = Eta * C1;
    float Rs = (Ks + C2) / (Ks - C2);
    float Kp = Eta * C2;
    float Rp = (Kp + C1) / (Kp - C1);
    return 0.5f * (Rs * Rs + Rp * Rp);
}

PT_DEV pt4 FresnelDielectric(pt4 Eta, pt4 C1, pt4 C2)
{
    pt4 Ks = Eta * C1;
    pt4 Rs = (Ks + C2) / (Ks - C2);
    pt4 Kp = Eta * C2;
    pt4 Rp = (Kp + C1) / (Kp - C1);
    return 0.5f * (Rs * Rs + Rp * Rp);
}

PT_DEV pt4 FresnelDielectric(pt4 Eta, pt4 C1) { return FresnelDielectric(Eta, C1, ComputeCosThetaRefracted(Eta, C1)); }

PT_DEV float Pow5(float x) { float x2 = x * x; return (x2 * x2) * x; }
PT_DEV float Pow6(float x) { float x2 = x * x; return (x2 * x2) * x2; }

PT_DEV pt4 SchlickFresnelMetal(pt4 Base, pt4 Specular, float CosTheta)
{
    const float CosThetaMax = 1 / 7.0f;
    pt4 FSchlick = Base + (1 - Base) * Pow5(1.0f - CosTheta);
    pt4 FSchlickMax = Base + (1 - Base) * Pow5(1 - CosThetaMax);
    pt4 FMax = Specular * FSchlickMax;
    const float Denominator = CosThetaMax * Pow6(1 - CosThetaMax);
    float Nominator = CosTheta * Pow6(1.0f - CosTheta);
    return FSchlick - (Nominator / Denominator) * (FSchlickMax - FMax);
}

// --- spectrum.glsl.inc ----------------------------------------------------

PT_DEV pt3 SampleStandardObserver(float L)
{
    pt3 R;
    {
        float T1 = (L - 442.0f) * (L < 442.0f ? 0.0624f : 0.0374f);
        float T2 = (L - 599.8f) * (L < 599.8f ? 0.0264f : 0.0323f);
        float T3 = (L - 501.1f) * (L < 501.1f ? 0.0490f : 0.0382f);
        R.x = 0.362f * pt_exp(-0.5f * T1 * T1) + 1.056f * pt_exp(-0.5f * T2 * T2) - 0.065f * pt_exp(-0.5f * T3 * T3);
    }
    {
        float T1 = (L - 568.8f) * (L < 568.8f ? 0.0213f : 0.0247f);
        float T2 = (L - 530.9f) * (L < 530.9f ? 0.0613f : 0.0322f);
        R.y = 0.821f * pt_exp(-0.5f * T1 * T1) + 0.286f * pt_exp(-0.5f * T2 * T2);
    }
    {
        float T1 = (L - 437.0f) * (L < 437.0f ? 0.0845f : 0.0278f);
        float T2 = (L - 459.0f) * (L < 459.0f ? 0.0385f : 0.0725f);
        R.z = 1.217f * pt_exp(-0.5f * T1 * T1) + 0.681f * pt_exp(-0.5f * T2 * T2);
    }
    return R;
}

PT_DEV float SampleParametricSpectrum(pt3 B, float L)
{
    float X = (B.x * L + B.y) * L + B.z;
    return 0.5f + X / (2.0f * pt_sqrt(1.0f + X * X));
}

// The untextured sky's spectrum (0, 0, 100) at any finite wavelength:
// (0 * L + 0) * L + 100 = 100 exactly, so every wavelength gives this value;
// evaluated once per scene upload with the same pt_fp.h operations.
PT_HD float SkyFlat()
{
    const float X = 100.0f;
    return 0.5f + X / (2.0f * pt_sqrt(1.0f + X * X));
}

PT_DEV pt4 SampleParametricSpectrum(pt3 B, pt4 L)
{
    return v4(SampleParametricSpectrum(B, L.x), SampleParametricSpectrum(B, L.y), SampleParametricSpectrum(B, L.z),
              SampleParametricSpectrum(B, L.w));
}

// --- scene data access ----------------------------------------------------

// Device atlas layout.  Row-major (the packed layout) needs two 128-byte
// lines for every bilinear footprint (its two rows are a whole atlas row
// apart) and four when it straddles a line; 4x2-texel blocks of 128 bytes
// (one line each, blocks row-major) put a footprint in one line 3/8 of the
// time: 1.875 lines per sample instead of 2.25, and a pixel tile's primary
// hits share blocks in both directions.  Used when W % 4 == 0 and
// H % 2 == 0 (every reference atlas: 4096^2); the texel values are the same.
PT_DEV size_t AtlasIndex(const dscene& S, uint32_t Layer, uint32_t X, uint32_t Y)
{
    size_t layer = (size_t)Layer * S.atlas_h * S.atlas_w;
    if (!S.atlas_tiled) return layer + (size_t)Y * S.atlas_w + X;
    return layer + ((size_t)((Y >> 1) * (S.atlas_w >> 2) + (X >> 2)) << 3) + ((Y & 1u) << 2) + (X & 3u);
}

template <bool UNIT>
PT_DEV float4 Texel(const dscene& S, uint32_t Layer, int X, int Y)
{
    if (S.atlas_layers == 0) return make_float4(0, 0, 0, 0);
    int W = (int)S.atlas_w, H = (int)S.atlas_h;
    // REPEAT wrap.  UNIT: every texture's placement lies in [0, 1] (the
    // lean shade instantiation, whose scenes the host checked: kernels.hpp
    // PT_MATS_TEXWRAP), so SampleTexture's coordinates lie in [-1, W] (U in
    // [0, 1] up to rounding: floor(U * W - 0.5) >= -1, floor(U * W) <= W),
    // where one add or subtract of W is the remainder -- two selects per axis
    // instead of a signed integer remainder (about 22 VALU with two
    // quarter-rate multiplies each, 8 per bilinear sample).
    if (UNIT) {
        X = X < 0 ? X + W : X; X = X >= W ? X - W : X;
        Y = Y < 0 ? Y + H : Y; Y = Y >= H ? Y - H : Y;
    } else {
        X %= W; if (X < 0) X += W;
        Y %= H; if (Y < 0) Y += H;
    }
    if (Layer >= S.atlas_layers) Layer = S.atlas_layers - 1;
    return S.atlas[AtlasIndex(S, Layer, (uint32_t)X, (uint32_t)Y)];
}

PT_DEV pt4 f4(float4 a) { return v4(a.x, a.y, a.z, a.w); }

// SampleTexture (scene.glsl.inc:181-205) with software REPEAT filtering.
template <bool UNIT = false>
PT_DEV pt4 SampleTexture(const dscene& S, uint32_t Index, pt2 UV)
{
    const pt_packed_texture T = S.textures[Index];
    float U = pt_mix(T.AtlasPlacementMinimum[0], T.AtlasPlacementMaximum[0], pt_fract(UV.x));
    float V = pt_mix(T.AtlasPlacementMinimum[1], T.AtlasPlacementMaximum[1], pt_fract(UV.y));
    float W = (float)S.atlas_w, H = (float)S.atlas_h;
    if (T.Flags & PT_TEXTURE_FLAG_FILTER_NEAREST)
        return f4(Texel<UNIT>(S, T.AtlasImageIndex, (int)pt_floor(U * W), (int)pt_floor(V * H)));
    float Us = U * W - 0.5f, Vs = V * H - 0.5f;
    float Fi = pt_floor(Us), Fj = pt_floor(Vs);
    float A = Us - Fi, B = Vs - Fj;
    int I0 = (int)Fi, J0 = (int)Fj;
    pt4 T00 = f4(Texel<UNIT>(S, T.AtlasImageIndex, I0, J0)), T10 = f4(Texel<UNIT>(S, T.AtlasImageIndex, I0 + 1, J0));
    pt4 T01 = f4(Texel<UNIT>(S, T.AtlasImageIndex, I0, J0 + 1)), T11 = f4(Texel<UNIT>(S, T.AtlasImageIndex, I0 + 1, J0 + 1));
    return ((1 - A) * (1 - B)) * T00 + (A * (1 - B)) * T10 + ((1 - A) * B) * T01 + (A * B) * T11;
}

// SampleSkyboxSpectrum (scene.glsl.inc:209-221)
PT_DEV pt4 SampleSkyboxSpectrum(const dscene& S, pt3 D)
{
    if (S.g.SkyboxTextureIndex == TEXTURE_INDEX_NONE) return v4(0, 0, 100, 1);
    float Phi = pt_atan2(D.y, D.x);
    float Theta = pt_asin(D.z);
    float U = 0.5f + Phi / PT_TAU;
    float V = 0.5f + Theta / PT_PI;
    return SampleTexture(S, S.g.SkyboxTextureIndex, v2(U, V));
}

// SampleSkyboxRadiance (scene.glsl.inc:225-229)
PT_DEV pt4 SampleSkyboxRadiance(const dscene& S, pt3 D, pt4 Lambda)
{
    // Untextured sky: (1 * SampleParametricSpectrum((0, 0, 100), Lambda)) is
    // the per-scene constant sky_flat at every (finite) wavelength.
    if (S.g.SkyboxTextureIndex == TEXTURE_INDEX_NONE) return v4s(S.sky_flat) * S.g.SkyboxBrightness;
    pt4 Spectrum = SampleSkyboxSpectrum(S, D);
    return (Spectrum.w * SampleParametricSpectrum(v3(Spectrum.x, Spectrum.y, Spectrum.z), Lambda)) * S.g.SkyboxBrightness;
}

PT_DEV uint32_t MUint(const dscene& S, uint32_t M, uint32_t A) { return S.material[32 * (size_t)M + A]; }
PT_DEV float MFloat(const dscene& S, uint32_t M, uint32_t A) { return pt_u2f(MUint(S, M, A)); }
PT_DEV pt3 MVec3(const dscene& S, uint32_t M, uint32_t A) { return v3(MFloat(S, M, A), MFloat(S, M, A + 1), MFloat(S, M, A + 2)); }

template <bool UNIT = false>
PT_DEV pt4 MaterialTexturableReflectance(const dscene& S, uint32_t M, uint32_t A, pt4 Lambda, pt2 UV)
{
    pt4 Value = SampleParametricSpectrum(MVec3(S, M, A), Lambda);
    uint32_t Tx = MUint(S, M, A + 3);
    if (Tx != TEXTURE_INDEX_NONE) {
        pt4 T = SampleTexture<UNIT>(S, Tx, UV);
        Value = Value * SampleParametricSpectrum(v3(T.x, T.y, T.z), Lambda);
    }
    return Value;
}

PT_DEV float MaterialTexturableValue(const dscene& S, uint32_t M, uint32_t A, pt2 UV)
{
    float Value = MFloat(S, M, A);
    uint32_t Tx = MUint(S, M, A + 1);
    if (Tx != TEXTURE_INDEX_NONE) Value *= SampleTexture(S, Tx, UV).x;
    return Value;
}

}  // namespace ptd
