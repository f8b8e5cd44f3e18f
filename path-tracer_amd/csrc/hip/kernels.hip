// kernels.hip — the wavefront integrator for gfx950.
//
//   raygen  : GenerateNewPath for every slot + zero the accumulator
//             (ResetBasicRenderer, basic_scatter.glsl:330-336)
//   extend  : Trace() of every slot's ray -> hit record
//             (basic_trace.glsl:7-16, scene.glsl.inc:304-611)
//   shade   : Scatter() + accumulate + regenerate
//             (basic_scatter.glsl:44-360)
//
// Slot state is SoA-of-float4 indexed by slot (16-byte coalesced accesses):
//   ray  = {origin.xyz, packed velocity}, hit = {time, shape|mat, n, t},
//   uv, throughput, probability, {sample.xyz, lambda0}, active-shape stack.
// Slot s covers pixel (tx*16 + s%16, band*16 + (s%256)/16) of the tile
// t = s/256, so a renderer can own an arbitrary set of 16-row bands.
//
// Ray order (TileOrder): the path arrays (thr, prob, lam, act) are indexed by
// slot, the ray and hit arrays by POSITION within the same tile.  Whenever a
// block of 256 slots (one tile) emits its rays, it sorts them by direction
// octant with a block counting sort and stores slot s's ray at position
// pos(s); extend runs one thread per position, so a wave traces rays of one
// octant from one 16x16 pixel tile (0.91x extend time on C3 vs pixel order,
// tools/exp_reorder.py).  Every ray is still traced and shaded with its own
// slot's data, so results do not depend on the order.
#include "pt_device.hpp"
#include "traverse.hpp"
#include "kernels.hpp"

#include <type_traits>
#include <map>
#include <mutex>
#include <tuple>

namespace ptd {

// --- shade branch statistics (experiment build only) ---------------------------
//
// Built with -DPT_SHADE_STATS=1 (tools/shade_stats.py via tools/build_variant.py),
// each mark ShadeMark(k) records, once per wave that reaches it, the number of
// lanes active there: waves[k] and lanes[k] summed over the launch, so
// lanes[k] / waves[k] is the SIMD occupancy of that branch of Scatter.  The
// product build compiles every mark to nothing.
#ifndef PT_SHADE_STATS
#define PT_SHADE_STATS 0
#endif
enum : uint32_t {
    SM_ENTRY, SM_HIT, SM_ESCAPE, SM_MEDIUM_EVENT, SM_SURFACE, SM_REAL, SM_LIGHT, SM_LIGHT_BELOW,
    SM_DIFFUSE_COSINE, SM_DIFFUSE_EVAL, SM_METAL_EVAL, SM_METAL_SAMPLE, SM_TRANS_EVAL, SM_TRANS_SAMPLE,
    SM_TRANS_REFLECT, SM_TRANS_REFRACT, SM_OPENPBR, SM_NOT_REAL, SM_ROULETTE, SM_COMPLETED, SM_CONTINUE,
    SM_EXTERIOR_MEDIUM, SM_MESH_HIT, SM_SPHERE_HIT, SM_CUBE_HIT, SM_PLANE_HIT, SM_COUNT
};
#if PT_SHADE_STATS
__device__ unsigned long long g_shade_stats[2 * 32];
PT_DEV uint32_t* ShadeStatLds()
{
    __shared__ uint32_t a[2 * 32];
    return a;
}
PT_DEV void ShadeMark(uint32_t k)
{
    const uint64_t m = __ballot(1);
    const uint32_t first = (uint32_t)__ffsll((unsigned long long)m) - 1u;
    if ((threadIdx.x & 63u) == first) {
        atomicAdd(&ShadeStatLds()[2 * k], 1u);
        atomicAdd(&ShadeStatLds()[2 * k + 1], (uint32_t)__popcll(m));
    }
}
PT_DEV void ShadeStatsBegin()
{
    if (threadIdx.x < 64) ShadeStatLds()[threadIdx.x] = 0;
    __syncthreads();
}
PT_DEV void ShadeStatsEnd()
{
    __syncthreads();
    if (threadIdx.x < 2 * SM_COUNT) atomicAdd(&g_shade_stats[threadIdx.x], (unsigned long long)ShadeStatLds()[threadIdx.x]);
}
#else
PT_DEV void ShadeMark(uint32_t) {}
PT_DEV void ShadeStatsBegin() {}
PT_DEV void ShadeStatsEnd() {}
#endif

// --- slot / pixel mapping ---------------------------------------------------

// t / tiles_x by the host-computed reciprocal (exact for t * tiles_x < 2^32).
// (tiles_x == 1: the reciprocal 2^32 does not fit, the row is t itself.)
PT_DEV uint32_t TileRow(const dframe& F, uint32_t t)
{
    return F.tiles_x == 1 ? t : __umulhi(t, F.tiles_x_magic);
}

// Path stream of tile t, and t's tile within its stream.
PT_DEV uint32_t TileStream(const dframe& F, uint32_t& t)
{
    if (F.streams == 1) return 0;
    const uint32_t k = __umulhi(t, F.stream_magic);
    t -= k * F.stream_tiles;
    return k;
}

// The seed of slot s's stream (FrameIndex + (stream << 24)) and its
// accumulator.
PT_DEV uint32_t StreamSeed(uint32_t seed, uint32_t stream) { return seed + (stream << 24); }
PT_DEV float4* StreamAccum(const dframe& F, uint32_t stream)
{
    return F.streams == 1 ? F.accum : F.accx + (size_t)stream * F.width * F.height;
}

PT_DEV bool SlotPixel(const dframe& F, uint32_t s, uint32_t& x, uint32_t& y, uint32_t& stream)
{
    uint32_t t = s >> 8, l = s & 255u;
    stream = TileStream(F, t);
    uint32_t k = TileRow(F, t);
    uint32_t tx = t - k * F.tiles_x;
    uint32_t band = F.rank + k * F.nranks;
    x = tx * 16 + (l & 15u);
    y = band * 16 + (l >> 4);
    return x < F.width && y < F.height;
}

// Valid positions of a tile are the first (pixels of the tile inside the
// image): TileOrder sorts the slots outside the image to the end.
PT_DEV bool SlotPixel(const dframe& F, uint32_t s, uint32_t& x, uint32_t& y)
{
    uint32_t stream;
    return SlotPixel(F, s, x, y, stream);
}

PT_DEV bool PositionValid(const dframe& F, uint32_t q)
{
    uint32_t t = q >> 8;
    (void)TileStream(F, t);
    uint32_t k = TileRow(F, t);
    uint32_t tx = t - k * F.tiles_x;
    uint32_t band = F.rank + k * F.nranks;
    uint32_t nx = min(16u, F.width - tx * 16u);
    uint32_t ny = band * 16u < F.height ? min(16u, F.height - band * 16u) : 0u;
    return (q & 255u) < nx * ny;
}

// Position of slot s's current ray / last traced hit.
PT_DEV uint32_t RayPos(const dslots& L, uint32_t s, uint32_t p16) { return (s & ~255u) | (p16 >> 8); }
PT_DEV uint32_t HitPos(const dslots& L, uint32_t s, uint32_t p16) { return (s & ~255u) | (p16 & 255u); }

// --- materials ---------------------------------------------------------------

struct bsdf_parameters { uint32_t MaterialIndex; pt2 TextureUV; pt4 Lambda; pt4 ExteriorIOR; };

// The basic BSDFs (basic_diffuse / basic_metal / basic_translucent.glsl.inc)
// take their material parameters already fetched (bsdf_material, below):
// SampleSurfaceIntegrand reads them once per hit, in code shared by the
// material types and by the light-sample evaluation and the BSDF sample,
// instead of once in each of those divergent branches.  The expressions are
// the reference's, so the results are the same bits.

// Texture-able material parameters of a basic material (MaterialEvaluateBSDF /
// MaterialSampleBSDF's *_GetParameters): Refl = the base reflectance
// (diffuse / metal), Aux = the metal's specular reflectance or the
// translucent's relative IOR, A / Rough = the GGX alpha of metal and
// translucent materials.
static_assert(PT_BASIC_DIFFUSE_BASE_SPECTRUM == PT_BASIC_METAL_BASE_SPECTRUM, "shared base reflectance word");
struct bsdf_material {
    pt4 Refl, Aux;
    pt2 A;
    bool Rough;
};

PT_DEV bool Diffuse_Evaluate(const bsdf_material& Q, pt3 In, pt4& T, pt4& Pr)
{
    Pr = v4s(In.z / PT_PI);
    T = Pr * Q.Refl;
    return true;
}

PT_DEV bool Metal_Evaluate(const bsdf_material& Q, pt3 In, pt3 Out, pt4& T, pt4& Pr)
{
    const pt2 A = Q.A;
    if (In.z <= 0.0f || Out.z <= 0.0f || !Q.Rough) return false;
    pt3 Half = SafeNormalize(In + Out);
    float Gm = GGXSmithG1(In, A);
    float D = GGXDistribution(Half, A);
    Pr = v4s(Gm * D / (4 * In.z));
    float Gs = GGXSmithG1(Out, A);
    pt4 F = SchlickFresnelMetal(Q.Refl, Q.Aux, dot(In, Half));
    T = Pr * Gs * F;
    return true;
}

PT_DEV bool Metal_Sample(rng& G, const bsdf_material& Q, pt3 In, pt3& Out, pt4& T, pt4& Pr)
{
    const pt2 A = Q.A;
    if (In.z <= 0.0f) return false;
    float U1 = G.R01();
    float U2 = G.R01();
    pt3 N = GGXVisibleNormal(In, A, U1, U2);
    float CosThetaIn = pt_min(dot(N, In), 1.0f);
    Out = 2 * CosThetaIn * N - In;
    if (Out.z <= 0.0f) return false;
    Pr = v4s(1.0f);
    if (Q.Rough) {
        float Gm = GGXSmithG1(In, A);
        float D = GGXDistribution(N, A);
        Pr = Pr * v4s(Gm * D / (4 * In.z));
    }
    float Gs = GGXSmithG1(Out, A);
    pt4 F = SchlickFresnelMetal(Q.Refl, Q.Aux, CosThetaIn);
    T = Pr * Gs * F;
    return true;
}

// Q.Aux = RelativeIOR: Interior / Exterior when In.z < 0, else Exterior /
// Interior (basic_translucent.glsl.inc GetParameters), In the direction
// towards the viewer (Scatter's Out).
PT_DEV bool Translucent_Evaluate(const bsdf_material& Q, pt3 In, pt3 Out, pt4& T, pt4& Pr)
{
    const pt4 RelIOR = Q.Aux;
    const pt2 A = Q.A;
    if (!Q.Rough) { Pr = v4s(0.0f); T = v4s(0.0f); return true; }
    float Gm = GGXSmithG1(In, A);
    if (In.z * Out.z > 0) {
        pt3 Half = SafeNormalize(Out + In);
        float CosThetaIn = dot(Half, In);
        pt4 F = FresnelDielectric(RelIOR, v4s(CosThetaIn));
        float D = GGXDistribution(Half, A);
        Pr = F * Gm * D / (4 * In.z);
    } else {
        pt3 H1 = SafeNormalize(Out + In * RelIOR.x);
        pt3 H2 = SafeNormalize(Out + In * RelIOR.y);
        pt3 H3 = SafeNormalize(Out + In * RelIOR.z);
        pt3 H4 = SafeNormalize(Out + In * RelIOR.w);
        pt4 Ci = v4(dot(In, H1), dot(In, H2), dot(In, H3), dot(In, H4));
        pt4 Co = v4(dot(Out, H1), dot(Out, H2), dot(Out, H3), dot(Out, H4));
        pt4 F = FresnelDielectric(RelIOR, Ci, Co);
        pt4 D = v4s(0.0f);
        if (Ci.x * Co.x < 0.0f) D.x = GGXDistribution(H1, A);
        if (Ci.y * Co.y < 0.0f) D.y = GGXDistribution(H2, A);
        if (Ci.z * Co.z < 0.0f) D.z = GGXDistribution(H3, A);
        if (Ci.w * Co.w < 0.0f) D.w = GGXDistribution(H4, A);
        pt4 Sq = Ci * RelIOR + Co;
        pt4 J = vabs(Co) / (Sq * Sq);
        Pr = D * (1 - F) * Gm * J * vabs(Ci / In.z);
    }
    float Gs = GGXSmithG1(Out, A);
    T = Pr * Gs;
    return true;
}

PT_DEV bool Translucent_Sample(rng& G, const bsdf_material& Q, pt3 In, pt3& Out, pt4& T, pt4& Pr)
{
    const pt4 RelIOR = Q.Aux;
    const pt2 A = Q.A;
    float U1 = G.R01();
    float U2 = G.R01();
    pt3 N = GGXVisibleNormal(In * pt_sign(In.z), A, U1, U2);
    float CosThetaIn = pt_clamp(dot(N, In), -1.0f, +1.0f);
    float CosThetaRefracted = ComputeCosThetaRefracted(RelIOR.x, CosThetaIn);
    float Reflectance = FresnelDielectric(RelIOR.x, CosThetaIn, CosThetaRefracted);
    if (G.R01() < Reflectance) {
        ShadeMark(SM_TRANS_REFLECT);
        Out = 2 * CosThetaIn * N - In;
        if (Out.z * In.z <= 0) return false;
        pt4 F = FresnelDielectric(RelIOR, v4s(CosThetaIn));
        Pr = F;
        if (Q.Rough) {
            float Gm = GGXSmithG1(In, A);
            float D = GGXDistribution(N, A);
            Pr = Pr * (Gm * D / (4 * pt_abs(In.z)));
        }
        float Gs = GGXSmithG1(Out, A);
        T = Pr * Gs;
        return true;
    }
    ShadeMark(SM_TRANS_REFRACT);
    Out = (CosThetaRefracted + RelIOR.x * CosThetaIn) * N - RelIOR.x * In;
    if (Out.z * In.z >= 0) return false;
    if (Q.Rough) {
        pt3 N2 = SafeNormalize(Out + In * RelIOR.y);
        pt3 N3 = SafeNormalize(Out + In * RelIOR.z);
        pt3 N4 = SafeNormalize(Out + In * RelIOR.w);
        pt4 Ci = v4(CosThetaIn, dot(In, N2), dot(In, N3), dot(In, N4));
        pt4 Co = v4(CosThetaRefracted, dot(Out, N2), dot(Out, N3), dot(Out, N4));
        pt4 F = FresnelDielectric(RelIOR, Ci, Co);
        pt4 D = v4s(0.0f);
        D.x = GGXDistribution(N, A);
        if (Ci.y * Co.y < 0.0f) D.y = GGXDistribution(N2, A);
        if (Ci.z * Co.z < 0.0f) D.z = GGXDistribution(N3, A);
        if (Ci.w * Co.w < 0.0f) D.w = GGXDistribution(N4, A);
        float Gm = GGXSmithG1(In, A);
        pt4 Sq = Ci * RelIOR + Co;
        pt4 J = vabs(Co) / (Sq * Sq);
        Pr = D * (1 - F) * Gm * J * vabs(Ci / In.z);
    } else {
        Pr = v4(1 - Reflectance, 0, 0, 0);
    }
    float Gs = GGXSmithG1(Out, A);
    T = Pr * Gs;
    return true;
}

// --- OpenPBR (src/scene/openpbr.glsl.inc) ----------------------------------------
// The reference packs OpenPBR materials but never shades them (its include is
// commented out, scene.glsl.inc:685, and DISPATCH_MATERIAL has no OpenPBR
// case), so by default an OpenPBR hit ends the path as there.  With
// ptSetBasicRendererOpenPBR the layered sampler below is dispatched instead
// (PT_MATS_OPENPBR instantiation): a sampling-only BSDF (HasDirac true, so no
// skybox light sampling), the medium of openpbr.glsl.inc:160-191.  Deviations
// from the uncompiled text: the coat's FresnelDielectric
// arguments are put in signature order; Emission, computed but never read by
// OpenPBR_Sample, is not evaluated; a LayerBounceLimit of 0 leaves In = -Out
// (the reference's out parameter is unassigned).

struct openpbr_parameters {                       // openpbr.glsl.inc:30-47
    uint32_t LayerBounceLimit;
    bool BaseIsMetal, BaseIsTranslucent, CoatIsPresent;
    pt4 BaseReflectance;
    float BaseDiffuseRoughness;
    pt4 CoatRelativeIOR, CoatTransmittance;
    pt2 CoatRoughnessAlpha;
    float SpecularWeight;
    pt4 SpecularRelativeIOR, SpecularReflectance;
    pt2 SpecularRoughnessAlpha;
};

// OpenPBR_Parameters (:66-158): three stochastic layer choices, then the
// spectral parameters at the cluster wavelengths.
PT_DEV openpbr_parameters OpenPBR_Parameters(const dscene& S, rng& G, const bsdf_parameters& P)
{
    const uint32_t M = P.MaterialIndex;
    openpbr_parameters Q;
    Q.CoatIsPresent = G.R01() < MFloat(S, M, PT_OPENPBR_COAT_WEIGHT);
    Q.BaseIsMetal = G.R01() < MFloat(S, M, PT_OPENPBR_BASE_METALNESS);
    Q.BaseIsTranslucent = !Q.BaseIsMetal && G.R01() < MFloat(S, M, PT_OPENPBR_TRANSMISSION_WEIGHT);
    Q.BaseReflectance = MFloat(S, M, PT_OPENPBR_BASE_WEIGHT) *
                        SampleParametricSpectrum(MVec3(S, M, PT_OPENPBR_BASE_SPECTRUM), P.Lambda);
    Q.BaseDiffuseRoughness = MFloat(S, M, PT_OPENPBR_BASE_DIFFUSE_ROUGHNESS);
    uint32_t Tx = MUint(S, M, PT_OPENPBR_BASE_SPECTRUM_TEXTURE_INDEX);
    if (Tx != TEXTURE_INDEX_NONE) {
        pt4 V = SampleTexture(S, Tx, P.TextureUV);
        Q.BaseReflectance = Q.BaseReflectance * SampleParametricSpectrum(v3(V.x, V.y, V.z), P.Lambda);
    }
    const float CoatIOR = MFloat(S, M, PT_OPENPBR_COAT_IOR);
    Q.CoatRelativeIOR = v4s(1.0f); Q.CoatTransmittance = v4s(1.0f); Q.CoatRoughnessAlpha = v2(0.0f, 0.0f);
    if (Q.CoatIsPresent) {
        Q.CoatRelativeIOR = P.ExteriorIOR / CoatIOR;
        Q.CoatTransmittance = SampleParametricSpectrum(MVec3(S, M, PT_OPENPBR_COAT_COLOR_SPECTRUM), P.Lambda);
        Q.CoatRoughnessAlpha = GGXRoughnessAlpha(MFloat(S, M, PT_OPENPBR_COAT_ROUGHNESS),
                                                 MFloat(S, M, PT_OPENPBR_COAT_ROUGHNESS_ANISOTROPY));
    }
    Q.SpecularWeight = MFloat(S, M, PT_OPENPBR_SPECULAR_WEIGHT);
    Q.SpecularReflectance = SampleParametricSpectrum(MVec3(S, M, PT_OPENPBR_SPECULAR_SPECTRUM), P.Lambda);
    pt4 SpecularIOR = CauchyEmpiricalIOR(MFloat(S, M, PT_OPENPBR_SPECULAR_IOR),
                                         MFloat(S, M, PT_OPENPBR_TRANSMISSION_DISPERSION_ABBE_NUMBER), P.Lambda);
    Q.SpecularRelativeIOR = Q.CoatIsPresent ? CoatIOR / SpecularIOR : P.ExteriorIOR / SpecularIOR;
    float SpecularRoughness = MFloat(S, M, PT_OPENPBR_SPECULAR_ROUGHNESS);
    Tx = MUint(S, M, PT_OPENPBR_SPECULAR_ROUGHNESS_TEXTURE_INDEX);
    if (Tx != TEXTURE_INDEX_NONE) SpecularRoughness = SpecularRoughness * SampleTexture(S, Tx, P.TextureUV).x;
    Q.SpecularRoughnessAlpha = GGXRoughnessAlpha(SpecularRoughness, MFloat(S, M, PT_OPENPBR_SPECULAR_ROUGHNESS_ANISOTROPY));
    Q.LayerBounceLimit = MUint(S, M, PT_OPENPBR_LAYER_BOUNCE_LIMIT);
    return Q;
}

// OpenPBR_Medium (:160-191)
PT_DEV void OpenPBR_Medium(const dscene& S, uint32_t M, pt4 Lambda, medium& Md)
{
    Md.IOR = CauchyEmpiricalIOR(MFloat(S, M, PT_OPENPBR_SPECULAR_IOR),
                                MFloat(S, M, PT_OPENPBR_TRANSMISSION_DISPERSION_ABBE_NUMBER), Lambda);
    float TD = MFloat(S, M, PT_OPENPBR_TRANSMISSION_DEPTH);
    if (TD > 0.0f) {
        pt4 Ext = -vlog(SampleParametricSpectrum(MVec3(S, M, PT_OPENPBR_TRANSMISSION_SPECTRUM), Lambda)) / TD;
        pt4 Sc = SampleParametricSpectrum(MVec3(S, M, PT_OPENPBR_TRANSMISSION_SCATTER_SPECTRUM), Lambda) / TD;
        Md.AbsorptionRate = vmax(Ext - Sc, 0.0f);
        Md.ScatteringRate = Sc;
        Md.ScatteringAnisotropy = MFloat(S, M, PT_OPENPBR_TRANSMISSION_SCATTER_ANISOTROPY);
    } else {
        Md.AbsorptionRate = v4s(0.0f);
        Md.ScatteringRate = v4s(0.0f);
        Md.ScatteringAnisotropy = 0.0f;
    }
}

// OpenPBR_CoatSample (:194-283)
PT_DEV void OpenPBR_CoatSample(rng& G, const openpbr_parameters& Q, pt3 Out, pt3& In, pt4& T, pt4& D)
{
    if (!Q.CoatIsPresent) { In = -Out; return; }
    float U1 = G.R01();
    float U2 = G.R01();
    pt3 N = GGXVisibleNormal(Out * pt_sign(Out.z), Q.CoatRoughnessAlpha, U1, U2);
    float Cosine = dot(N, Out);
    pt4 R = Q.CoatRelativeIOR;
    if (Out.z < 0) R = 1.0f / R;
    float RefractedCosineSquared = 1 - R.x * R.x * (1 - Cosine * Cosine);
    float RefractedCosine = -pt_sign(Out.z) * pt_sqrt(pt_max(RefractedCosineSquared, 0.0f));
    float Reflectance = FresnelDielectric(R.x, Cosine, RefractedCosine);
    if (G.R01() < Reflectance) {
        In = 2 * Cosine * N - Out;
        if (In.z * Out.z <= 0) { D = v4s(0.0f); return; }
        T = T * GGXSmithG1(In, Q.CoatRoughnessAlpha);
        if (Out.z < 0) {
            float Exponent = -(0.5f / Out.z + 0.5f / In.z);
            T = T * vpow(Q.CoatTransmittance, Exponent);
        }
    } else {
        In = (R.x * Cosine + RefractedCosine) * N - R.x * Out;
        if (In.z * Out.z > 0) { D = v4s(0.0f); return; }
        T = T * GGXSmithG1(In, Q.CoatRoughnessAlpha);
        if (Out.z < 0) T = T * vpow(Q.CoatTransmittance, -0.5f / Out.z);
        else T = T * vpow(Q.CoatTransmittance, -0.5f / In.z);
    }
}

// OpenPBR_BaseSpecularSample (:286-435)
PT_DEV void OpenPBR_BaseSpecularSample(rng& G, const openpbr_parameters& Q, pt3 Out, pt3& In, pt4& T, pt4& D)
{
    const pt2 A = Q.SpecularRoughnessAlpha;
    float U1 = G.R01();
    float U2 = G.R01();
    pt3 N = GGXVisibleNormal(Out * pt_sign(Out.z), A, U1, U2);
    float Cosine = dot(N, Out);
    if (Q.BaseIsMetal) {
        In = 2 * Cosine * N - Out;
        if (Out.z * In.z <= 0) { D = v4s(0.0f); return; }
        float Shadowing = GGXSmithG1(Out, A);
        pt4 F = Q.SpecularWeight * SchlickFresnelMetal(Q.BaseReflectance, Q.SpecularReflectance, pt_abs(Cosine));
        T = T * (F * Shadowing);
        return;
    }
    pt4 R = Q.SpecularRelativeIOR;
    if (Out.z < 0) R = 1.0f / R;
    if (Q.SpecularWeight < 1.0f) {
        pt4 Rw = pt_sqrt(Q.SpecularWeight) * (1.0f - R) / (1.0f + R);
        R = (1.0f - Rw) / (1.0f + Rw);
    }
    float RefractedCosine = ComputeCosThetaRefracted(R.x, Cosine);
    float Reflectance = FresnelDielectric(R.x, Cosine, RefractedCosine);
    if (G.R01() < Reflectance) {
        In = 2 * Cosine * N - Out;
        if (In.z * Out.z <= 0) { D = v4s(0.0f); return; }
        if (Out.z > 0) T = T * Q.SpecularReflectance;
        T = T * GGXSmithG1(In, A);
        return;
    }
    In = (R.x * Cosine + RefractedCosine) * N - R.x * Out;
    if (In.z * Out.z > 0) { D = v4s(0.0f); return; }
    float Shadowing = GGXSmithG1(In, A);
    if (length(A) > PT_EPSILON) {
        pt4 F = v4s(0.0f);   // the reference's "TODO: This is broken for now!" (:390-391)
        pt3 N2 = SafeNormalize(In + Out * R.y);
        pt3 N3 = SafeNormalize(In + Out * R.z);
        pt3 N4 = SafeNormalize(In + Out * R.w);
        pt4 Dn = v4s(0.0f);
        Dn.x = GGXDistribution(N, A);
        if (dot(In, N2) * dot(Out, N2) < 0.0f) Dn.y = GGXDistribution(N2, A);
        if (dot(In, N3) * dot(Out, N3) < 0.0f) Dn.z = GGXDistribution(N3, A);
        if (dot(In, N4) * dot(Out, N4) < 0.0f) Dn.w = GGXDistribution(N4, A);
        Dn = Dn / pt_max(PT_EPSILON, max4(Dn));
        T = T * (Dn * F * Shadowing);
        D = D * (Dn * F);
    } else {
        T = T * v4(Shadowing, 0, 0, 0);
        D = D * v4(1, 0, 0, 0);
    }
}

// OpenPBR_BaseDiffuseSample (:438-461): Oren-Nayar-weighted cosine sampling.
PT_DEV void OpenPBR_BaseDiffuseSample(rng& G, const openpbr_parameters& Q, pt3 Out, pt3& In, pt4& T)
{
    if (Q.BaseIsTranslucent) { In = -Out; return; }
    In = SafeNormalize(RandomDirection(G) + v3(0, 0, 1));
    float Sv = dot(In, Out) - In.z * Out.z;
    float Tv = Sv > 0 ? pt_max(In.z, Out.z) : 1.0f;
    float SigmaSq = Q.BaseDiffuseRoughness * Q.BaseDiffuseRoughness;
    pt4 A = (1 - 0.5f * SigmaSq / (SigmaSq + 0.33f)) + 0.17f * Q.BaseReflectance * SigmaSq / (SigmaSq + 0.13f);
    float B = 0.45f * SigmaSq / (SigmaSq + 0.09f);
    T = T * (Q.BaseReflectance * (B * Sv / Tv + A));
}

// OpenPBR_Sample (:463-515): a random walk through the layer stack.
PT_DEV bool OpenPBR_Sample(rng& G, const openpbr_parameters& Q, pt3 Out, pt3& In, pt4& T, pt4& D)
{
    enum { EXTERNAL = -1, COAT = 0, BASE_SPECULAR = 1, BASE_DIFFUSE = 2 };
    int Layer = (Out.z > 0 && Q.CoatIsPresent) ? COAT : BASE_SPECULAR;
    T = v4s(1.0f);
    D = v4s(1.0f);
    In = -Out;
    for (uint32_t I = 0; I < Q.LayerBounceLimit; I++) {
        if (Layer == COAT) {
            OpenPBR_CoatSample(G, Q, Out, In, T, D);
            Layer = In.z < 0 ? BASE_SPECULAR : EXTERNAL;
        } else if (Layer == BASE_SPECULAR) {
            OpenPBR_BaseSpecularSample(G, Q, Out, In, T, D);
            Layer = In.z < 0 ? BASE_DIFFUSE : COAT;
        } else if (Layer == BASE_DIFFUSE) {
            OpenPBR_BaseDiffuseSample(G, Q, Out, In, T);
            Layer = In.z < 0 ? EXTERNAL : BASE_SPECULAR;
        } else {
            break;
        }
        if (max4(D) < PT_EPSILON) return false;
        Out = -In;
    }
    return true;
}

// Material-type specialisation of the shade kernel: MATS is a superset of the
// types referenced by the scene's shapes (computed on the host at upload), so
// dispatch branches for absent types are compiled out without changing any
// result.  PT_MATS_SCATTER: some medium can scatter (SceneScatterRate > 0 or
// a translucent / shaded OpenPBR material exists).  PT_MATS_OPENPBR: OpenPBR
// shading is enabled and the scene has OpenPBR shapes.
template <uint32_t MATS>
PT_DEV void LoadMedium(const dscene& S, uint32_t M, pt4 Lambda, medium& Md)
{
    Md.IOR = v4s(1.0f); Md.AbsorptionRate = v4s(0.0f); Md.ScatteringRate = v4s(0.0f); Md.ScatteringAnisotropy = 0.0f;
    if (!(MATS & (PT_MATS_TRANSLUCENT | PT_MATS_OPENPBR))) return;
    uint32_t Type = MUint(S, M, 0);
    if ((MATS & PT_MATS_OPENPBR) && Type == PT_MATERIAL_TYPE_OPENPBR) { OpenPBR_Medium(S, M, Lambda, Md); return; }
    if (!(MATS & PT_MATS_TRANSLUCENT) || Type != PT_MATERIAL_TYPE_BASIC_TRANSLUCENT) return;
    Md.IOR = CauchyEmpiricalIOR(MFloat(S, M, PT_BASIC_TRANSLUCENT_IOR), MFloat(S, M, PT_BASIC_TRANSLUCENT_ABBE_NUMBER), Lambda);
    float TD = MFloat(S, M, PT_BASIC_TRANSLUCENT_TRANSMISSION_DEPTH);
    if (TD > 0.0f) {
        pt4 Ext = -vlog(SampleParametricSpectrum(MVec3(S, M, PT_BASIC_TRANSLUCENT_TRANSMISSION_SPECTRUM), Lambda)) / TD;
        pt4 Sc = SampleParametricSpectrum(MVec3(S, M, PT_BASIC_TRANSLUCENT_SCATTERING_SPECTRUM), Lambda) / TD;
        Md.AbsorptionRate = vmax(Ext - Sc, 0.0f);
        Md.ScatteringRate = Sc;
        Md.ScatteringAnisotropy = MFloat(S, M, PT_BASIC_TRANSLUCENT_SCATTERING_ANISOTROPY);
    }
}

template <uint32_t MATS>
PT_DEV medium ResolveMedium(const dscene& S, uint32_t ShapeIndex, pt4 Lambda)
{
    medium Md;
    if (ShapeIndex == SHAPE_INDEX_NONE) {
        Md.Priority = 0xFFFFFFFFu;
        Md.IOR = v4s(1.0f);
        Md.AbsorptionRate = v4s(0.0f);
        Md.ScatteringRate = v4s(S.g.SceneScatterRate);
        Md.ScatteringAnisotropy = 0.0f;
    } else {
        LoadMedium<MATS>(S, S.shapes[ShapeIndex].MaterialIndex, Lambda, Md);
        Md.Priority = ShapeIndex;
    }
    return Md;
}

// SampleSurfaceIntegrand (basic_scatter.glsl:68-109).  The material's
// parameters are fetched once, in code shared by the types: the metal and
// translucent roughness / anisotropy (HasDirac reads the same roughness
// value) before the light choice, the reflectances after the sampled
// direction is known (a sky sample below the surface ends the path first).
template <uint32_t MATS, uint32_t CLS = 0xFFFFFFFFu>
PT_DEV bool SampleSurfaceIntegrand(const dscene& S, rng& G, pt3 Nrm, pt3 TX, pt3 TY, const bsdf_parameters& P, pt3 Out,
                                   pt3& In, pt4& Throughput, pt4& Probability)
{
    const uint32_t M = P.MaterialIndex;
    const uint32_t Type = MUint(S, M, 0);
    // CLS: the BSDF types this instantiation samples (a class-pure launch
    // compiles only its class's; the medium code still follows MATS).
    constexpr uint32_t B = MATS & CLS;
    const bool diffuse = (B & PT_MATS_DIFFUSE) && Type == PT_MATERIAL_TYPE_BASIC_DIFFUSE;
    const bool metal = (B & PT_MATS_METAL) && Type == PT_MATERIAL_TYPE_BASIC_METAL;
    const bool trans = (B & PT_MATS_TRANSLUCENT) && Type == PT_MATERIAL_TYPE_BASIC_TRANSLUCENT;
    const bool openpbr = (B & PT_MATS_OPENPBR) && Type == PT_MATERIAL_TYPE_OPENPBR;
    bsdf_material Q;
    Q.Rough = false;
    // HasDirac (basic_metal / basic_translucent .glsl.inc: roughness < 1e-3;
    // OpenPBR: sampling only, HasDirac true).
    bool Dirac = openpbr;
    if ((B & (PT_MATS_METAL | PT_MATS_TRANSLUCENT)) && (metal || trans)) {
        const float Roughness = MaterialTexturableValue(
            S, M, metal ? PT_BASIC_METAL_ROUGHNESS : PT_BASIC_TRANSLUCENT_ROUGHNESS, P.TextureUV);
        const float Anisotropy = MaterialTexturableValue(
            S, M, metal ? PT_BASIC_METAL_ROUGHNESS_ANISOTROPY : PT_BASIC_TRANSLUCENT_ROUGHNESS_ANISOTROPY, P.TextureUV);
        Q.A = GGXRoughnessAlpha(Roughness, Anisotropy);
        Q.Rough = Q.A.x * Q.A.y > PT_EPSILON;
        Dirac = Roughness < 1e-3f;
    }
    float LightProbability = Dirac ? 0.0f : S.g.SkyboxSamplingProbability;
    pt4 MaterialPDF = v4s(0.0f);
    pt3 SMD = v3(S.g.SkyboxMeanDirection[0], S.g.SkyboxMeanDirection[1], S.g.SkyboxMeanDirection[2]);
    pt3 Mu = v3(dot(SMD, TX), dot(SMD, TY), dot(SMD, Nrm));
    bool ok;
    // Without PT_MATS_SKY the probability is +-0, so the draw (still made:
    // the RNG sequence is the reference's) never selects the light.
    const float Ul = G.R01();
    const bool light = (MATS & PT_MATS_SKY) && Ul < LightProbability;
    // A diffuse hit draws In by the light choice -- the sky lobe or the
    // material's cosine sample -- and then evaluates the material with the
    // same arguments either way (MaterialEvaluateBSDF / MaterialSampleBSDF of
    // basic_diffuse.glsl.inc), so the evaluation runs once after the join.
    //
    // The sky lobe (RandomVonMisesFisher) and the cosine lobe (RandomDirection
    // + Z) draw the same two numbers into the same spherical construction and
    // differ only in its height Z and its frame, so a wave holding both kinds
    // of lane runs the sqrt, the sine / cosine and the normalization once.
    if (light || diffuse) {
        const float Xi = G.R01();
        float Z;
        pt3 MuX = v3s(0.0f), MuY = v3s(0.0f);
        if (light) {
            ShadeMark(SM_LIGHT);
            Z = 1 + S.vmf_inv_kappa * pt_log(Xi + (1 - Xi) * S.vmf_exp_m2k);
            ComputeCoordinateFrame(Mu, MuX, MuY);
        } else {
            ShadeMark(SM_DIFFUSE_COSINE);
            Z = 2 * Xi - 1;
        }
        const float R = pt_sqrt(1 - Z * Z);
        const float Phi = G.R01() * PT_TAU;
        const pt3 D = v3(R * pt_cos(Phi), R * pt_sin(Phi), Z);
        In = SafeNormalize(light ? D.x * MuX + D.y * MuY + D.z * Mu : D + v3(0, 0, 1));
        if (light && In.z < 0.0f) { ShadeMark(SM_LIGHT_BELOW); return false; }
    }
    // Reflectances: the diffuse and metal base spectrum share a material word
    // (BASE_SPECTRUM = 1), the metal's specular spectrum; the translucent's
    // Cauchy IOR relative to the exterior on Out's side.
    if (diffuse || metal)
        Q.Refl = MaterialTexturableReflectance<MATS == PT_MATS_DIFFUSE>(S, M, PT_BASIC_METAL_BASE_SPECTRUM, P.Lambda,
                                                                        P.TextureUV);
    if (metal) Q.Aux = MaterialTexturableReflectance(S, M, PT_BASIC_METAL_SPECULAR_SPECTRUM, P.Lambda, P.TextureUV);
    if (trans) {
        pt4 Interior = CauchyEmpiricalIOR(MFloat(S, M, PT_BASIC_TRANSLUCENT_IOR),
                                          MFloat(S, M, PT_BASIC_TRANSLUCENT_ABBE_NUMBER), P.Lambda);
        if (Out.z < 0.0f) Q.Aux = Interior / P.ExteriorIOR;
        else Q.Aux = P.ExteriorIOR / Interior;
    }
    if (diffuse) {
        ShadeMark(SM_DIFFUSE_EVAL);
        ok = Diffuse_Evaluate(Q, Out, Throughput, MaterialPDF);
        if (!ok) return false;
    } else if (light) {
        // MaterialEvaluateBSDF(Parameters, Out, In, ...)
        if (metal) {
            ShadeMark(SM_METAL_EVAL);
            ok = Metal_Evaluate(Q, Out, In, Throughput, MaterialPDF);
        } else if (trans) {
            ShadeMark(SM_TRANS_EVAL);
            ok = Translucent_Evaluate(Q, Out, In, Throughput, MaterialPDF);
        } else ok = false;
        if (!ok) return false;
    } else {
        // MaterialSampleBSDF(Parameters, Out, In, ...)
        if (metal) {
            ShadeMark(SM_METAL_SAMPLE);
            ok = Metal_Sample(G, Q, Out, In, Throughput, MaterialPDF);
        } else if (trans) {
            ShadeMark(SM_TRANS_SAMPLE);
            ok = Translucent_Sample(G, Q, Out, In, Throughput, MaterialPDF);
        } else if (openpbr) {
            ShadeMark(SM_OPENPBR);
            openpbr_parameters O = OpenPBR_Parameters(S, G, P);
            ok = OpenPBR_Sample(G, O, Out, In, Throughput, MaterialPDF);
        } else {
            ok = false;
        }
        if (!ok) return false;
    }
    if (!(MATS & PT_MATS_SKY)) {
        // LightProbability = +0 and a finite sky pdf (the host's
        // PT_MATS_SKY rule): +0 * pdf + 1 * MaterialPDF = MaterialPDF + 0.
        Probability = MaterialPDF + v4s(0.0f);
        return true;
    }
    pt4 SkyboxPDF = v4s(VonMisesFisherPDF(S.g.SkyboxConcentration, vmf_consts{S.vmf_inv_kappa, S.vmf_exp_m2k, S.vmf_norm},
                                          Mu, In));
    Probability = LightProbability * SkyboxPDF + (1 - LightProbability) * MaterialPDF;
    return true;
}

// --- path state ----------------------------------------------------------------


struct path {
    float Lambda0;
    pt4 Throughput, Probability;
    pt3 Sample;
    uint32_t Active[4];
};

// The path's four wavelengths from its normalized Lambda0
// (basic_scatter.glsl:118-122).
PT_DEV pt4 PathLambda(float L0)
{
    return v4(pt_mix(PT_CIE_LAMBDA_MIN, PT_CIE_LAMBDA_MAX, L0),
              pt_mix(PT_CIE_LAMBDA_MIN, PT_CIE_LAMBDA_MAX, pt_fract(L0 + 0.25f)),
              pt_mix(PT_CIE_LAMBDA_MIN, PT_CIE_LAMBDA_MAX, pt_fract(L0 + 0.50f)),
              pt_mix(PT_CIE_LAMBDA_MIN, PT_CIE_LAMBDA_MAX, pt_fract(L0 + 0.75f)));
}

// An escaped path's contribution (basic_scatter.glsl:165-173): the sky's
// radiance along V times the throughput, observed (CIE XYZ) and divided by
// the cluster PDF.
PT_DEV pt3 EscapeContribution(const dscene& S, pt3 V, pt4 Lambda, pt4 Throughput, float ClusterPDF)
{
    pt4 Emission = SampleSkyboxRadiance(S, V, Lambda);
    pt4 E = Emission * Throughput;
    // Left-to-right sum over the four wavelengths (the reference's
    // expression order) as a rolled loop: one observer evaluation's
    // registers at a time.
    float Lv[4] = {Lambda.x, Lambda.y, Lambda.z, Lambda.w};
    float Ev[4] = {E.x, E.y, E.z, E.w};
    pt3 XYZ = SampleStandardObserver(Lv[0]) * Ev[0];
#pragma unroll 1
    for (int I = 1; I < 4; I++) XYZ = XYZ + SampleStandardObserver(Lv[I]) * Ev[I];
    return XYZ / ClusterPDF;
}

// Path record (basic.glsl.inc:159-198 StorePathVertex) minus Sample: Scatter
// adds to Sample only on escape, and the escape zeroes Probability, which
// ends the path in the same shade (its Sample goes to the accumulator and a
// new path starts with Sample = 0).  So every path alive between rounds has
// Sample == 0 and only lambda0 is stored (4 bytes instead of 16); the state
// readback reports the zero.
// `act_none`: the slot's stored active-shape stack is already empty (all
// four entries NONE), as a new path's is, so its 8-byte record is not
// rewritten (a partial-line store for every completed path otherwise).
//
// GreyRecord: when the renderer's shade mask has no translucent and no
// OpenPBR material (pt_grey_mats), every factor Scatter multiplies into a
// path's Probability is the same for the four wavelengths -- the diffuse and
// metal pdfs are scalars (basic_diffuse.glsl.inc:30-33, basic_metal.glsl.inc),
// the sky pdf too, the medium density of the vacuum-or-scene-fog medium is
// v4(SceneScatterRate) based (basic_scatter.glsl:137-163), the roulette
// factor is a scalar (:295-298) -- and a new path starts at vec4(1); so the
// four components are the same bits, and the slot stores one float
// (L.prob1).  The active-shape stack can only grow on a refraction into a
// shape (In.z * Out.z < 0 with Out.z > 0, :266-282), which needs a
// translucent (or OpenPBR) BSDF: diffuse / metal directions have In.z >= 0,
// a sky sample below the surface ends the path, and a non-real hit seen from
// outside cannot occur with an empty stack; so it stays empty and is neither
// read nor written.  The host switches a renderer's live paths between the
// forms (pt_launch_grey_convert) when its shade mask changes.
PT_DEV void StorePathVertex(const dslots& L, uint32_t s, const path& P, bool act_none = false)
{
    L.thr[s] = make_float4(P.Throughput.x, P.Throughput.y, P.Throughput.z, P.Throughput.w);
    if (L.prob1) L.prob1[s] = P.Probability.x;
    else L.prob[s] = make_float4(P.Probability.x, P.Probability.y, P.Probability.z, P.Probability.w);
    L.lam[s] = P.Lambda0;
    if (!act_none) L.act[s] = make_uint2((P.Active[1] << 16) | P.Active[0], (P.Active[3] << 16) | P.Active[2]);
}

// Position of the k-th set bit (k < popcount) of a 64-bit word: a 6-step
// binary search over popcounts of the low halves.
PT_DEV uint32_t SelectBit64(uint64_t m, uint32_t k)
{
    uint32_t pos = 0;
    uint32_t lo = (uint32_t)m, hi = (uint32_t)(m >> 32);
    uint32_t c = (uint32_t)__popc(lo);
    uint32_t w = lo;
    if (k >= c) { k -= c; w = hi; pos = 32; }
#pragma unroll
    for (uint32_t width = 16; width >= 1; width >>= 1) {
        uint32_t cw = (uint32_t)__popc(w & ((1u << width) - 1u));
        if (k >= cw) { k -= cw; w >>= width; pos += width; }
    }
    return pos;
}

// ShadeOrder: the position shaded by thread u of a tile: the positions of
// outcome class 0 first (in position order), then class 1, ... (miss last),
// from the tile's class masks (extend).  Tile-uniform mask words (scalar
// loads and counts), no barrier.
// Two classes (single-material scenes): hits first, then the miss mask.
PT_DEV uint32_t ShadePosition2(const uint64_t* miss, uint32_t u)
{
    uint64_t m0 = miss[0], m1 = miss[1], m2 = miss[2], m3 = miss[3];
    uint32_t c0 = (uint32_t)__popcll(~m0), c1 = (uint32_t)__popcll(~m1), c2 = (uint32_t)__popcll(~m2);
    uint32_t nhit = c0 + c1 + c2 + (uint32_t)__popcll(~m3);
    bool hit = u < nhit;
    uint32_t k = hit ? u : u - nhit;
    uint64_t w0 = hit ? ~m0 : m0, w1 = hit ? ~m1 : m1, w2 = hit ? ~m2 : m2, w3 = hit ? ~m3 : m3;
    uint32_t n0 = hit ? c0 : 64u - c0, n1 = hit ? c1 : 64u - c1, n2 = hit ? c2 : 64u - c2;
    uint32_t word = 0;
    uint64_t w = w0;
    if (k >= n0) { k -= n0; word = 1; w = w1;
        if (k >= n1) { k -= n1; word = 2; w = w2;
            if (k >= n2) { k -= n2; word = 3; w = w3; } } }
    return word * 64 + SelectBit64(w, k);
}

PT_DEV uint32_t ShadePosition(const uint64_t* mask, uint32_t u)
{
    uint32_t cnt[PT_OUTCOME_CLASSES][4], before = 0;
    uint32_t cls = 0, k = u;
#pragma unroll
    for (uint32_t c = 0; c < PT_OUTCOME_CLASSES; c++) {
        uint32_t n = 0;
#pragma unroll
        for (uint32_t w = 0; w < 4; w++) {
            cnt[c][w] = (uint32_t)__popcll(mask[4 * c + w]);
            n += cnt[c][w];
        }
        if (u >= before) { cls = c; k = u - before; }   // last class whose start is <= u
        before += n;
    }
    // Empty classes share their start with the next class, so the last
    // class starting at or before u holds u.
    uint32_t word = 0;
    uint32_t c0 = cnt[0][0], c1 = cnt[0][1], c2 = cnt[0][2];
#pragma unroll
    for (uint32_t c = 1; c < PT_OUTCOME_CLASSES; c++)
        if (cls == c) { c0 = cnt[c][0]; c1 = cnt[c][1]; c2 = cnt[c][2]; }
    if (k >= c0) { k -= c0; word = 1;
        if (k >= c1) { k -= c1; word = 2;
            if (k >= c2) { k -= c2; word = 3; } } }
    return word * 64 + SelectBit64(mask[4 * cls + word], k);
}

// TileOrder: called by all 256 threads of a block (one tile) once their new
// rays are known.  Sort key: direction octant (0-7) for valid slots, 8 for
// slots outside the image.  Per wave, a ballot per key gives each lane its
// rank among the wave's lanes of that key; one wave-wide exclusive scan of the
// 4 x 9 (key-major) counts gives every (key, wave) its base.  `hitbyte` is
// the position of the slot's last traced hit (shade: the ray it just
// consumed, where extend wrote the hit; raygen: unchanged).
PT_DEV uint32_t TileOrderKey(bool valid, pt3 V)
{
    return valid ? ((V.x < 0.0f ? 1u : 0u) | (V.y < 0.0f ? 2u : 0u) | (V.z < 0.0f ? 4u : 0u)) : 8u;
}

// The same for a ray already packed ({O.xyz, PackUnitVector(V)}) with its key.
PT_DEV void TileOrderStoreKeyed(const dslots& L, uint32_t s, uint32_t key, float4 ray, uint32_t hitbyte)
{
    __shared__ uint32_t cnt[64];
    uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    uint32_t rank = 0;
#pragma unroll
    for (uint32_t k = 0; k < 9; k++) {
        uint64_t m = __ballot(key == k);
        uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if (key == k) rank = below;
        if (lane == 0) cnt[k * 4 + w] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    uint32_t v = lane < 36 ? cnt[lane] : 0u;
    uint32_t incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t t = (uint32_t)__shfl_up((int)incl, o, 64);
        if ((int)lane >= o) incl += t;
    }
    uint32_t base = (uint32_t)__shfl((int)(incl - v), (int)(key * 4 + w), 64);
    uint32_t p = base + rank;
    uint32_t q = (s & ~255u) | p;
    L.ray[q] = ray;
    L.pos[s] = (uint16_t)((p << 8) | hitbyte);
    L.slotof[q] = (uint8_t)(s & 255u);
}

PT_DEV void TileOrderStoreRay(const dslots& L, uint32_t s, bool valid, pt3 O, pt3 V, uint32_t hitbyte)
{
    TileOrderStoreKeyed(L, s, TileOrderKey(valid, V), make_float4(O.x, O.y, O.z, __uint_as_float(PackUnitVector(V))),
                        hitbyte);
}

// GenerateNewPath (basic_scatter.glsl:7-42) + GenerateCameraRay (scene.glsl.inc:613-655)
PT_DEV void GenerateNewPath(const dscene& S, const dslots& L, const dframe& F, const dparams& Pm, rng& G, uint32_t s,
                            uint32_t x, uint32_t y, pt3& RO, pt3& RV, bool act_none = false)
{
    float SPx = (float)x, SPy = (float)y;
    if (Pm.render_flags & PT_RENDER_FLAG_SAMPLE_JITTER) {
        float JX = G.R01();
        float JY = G.R01();
        SPx = SPx + JX; SPy = SPy + JY;
    } else {
        SPx = SPx + 0.5f; SPy = SPy + 0.5f;
    }
    float Nx = SPx / (float)F.width, Ny = SPy / (float)F.height;
    const pt_packed_camera* Cam = &S.cameras[Pm.camera_index];
    uint32_t Model = Cam->Model;
    pt3 O, V;
    if (Model == PT_CAMERA_MODEL_PINHOLE || Model == PT_CAMERA_MODEL_THIN_LENS) {
        pt3 SP = v3(-Cam->SensorSize[0] * (Nx - 0.5f), -Cam->SensorSize[1] * (0.5f - Ny), Cam->SensorDistance);
        if (Model == PT_CAMERA_MODEL_PINHOLE) {
            pt2 D = Cam->ApertureRadius * RandomPointOnDisk(G);
            O = v3(D.x, D.y, 0);
            V = normalize(O - SP);
        } else {
            pt3 OP = -SP * Cam->FocalLength / (SP.z - Cam->FocalLength);
            pt2 D = Cam->ApertureRadius * RandomPointOnDisk(G);
            O = v3(D.x, D.y, 0);
            V = normalize(OP - O);
        }
    } else if (Model == PT_CAMERA_MODEL_360) {
        float Phi = (Nx - 0.5f) * PT_TAU;
        float Theta = (0.5f - Ny) * PT_PI;
        O = v3(0, 0, 0);
        V = v3(pt_cos(Theta) * pt_sin(Phi), pt_sin(Theta), -pt_cos(Theta) * pt_cos(Phi));
    } else {
        O = v3s(0); V = v3s(0);
    }
    const float* To = Cam->Transform.To;
    RO = mat4_mul_point(To, O);
    RV = mat4_mul_vector(To, V);
    path P;
    P.Lambda0 = G.R01();
    P.Throughput = v4s(1.0f);
    P.Probability = v4s(1.0f);
    P.Sample = v3s(0.0f);
    P.Active[0] = P.Active[1] = P.Active[2] = P.Active[3] = SHAPE_INDEX_NONE;
    StorePathVertex(L, s, P, act_none);
}

// Scatter (basic_scatter.glsl:114-310).  Returns true if an extension ray was
// produced (written to O, V).
template <uint32_t MATS, uint32_t CLS = 0xFFFFFFFFu>
PT_DEV bool Scatter(const dscene& S, rng& G, float PTP, path& Path, pt3& O, pt3& V, uint32_t HitShape,
                    uint32_t HitMaterial, float HitTime, uint32_t PN, uint32_t PT, pt2 UV)
{
    pt4 Lambda = PathLambda(Path.Lambda0);

    uint32_t Active = SHAPE_INDEX_NONE;
    for (int I = 0; I < 4; I++) Active = pt_umin(Active, Path.Active[I]);

    medium Md = ResolveMedium<MATS>(S, Active, Lambda);
    // Without translucent (or shaded OpenPBR) materials every medium is vacuum: exp(-0 * t) = 1
    // exactly, so the multiply is an identity and is skipped.
    if (MATS & (PT_MATS_TRANSLUCENT | PT_MATS_OPENPBR)) Path.Throughput = Path.Throughput * vexp(-Md.AbsorptionRate * HitTime);

    float ScatteringTime = PT_HIT_TIME_LIMIT;
    if ((MATS & PT_MATS_SCATTER) && Md.ScatteringRate.x > 0.0f) ScatteringTime = -pt_log(G.R01()) / Md.ScatteringRate.x;

    if (HitTime >= ScatteringTime) {
        if (ScatteringTime < PT_HIT_TIME_LIMIT) {
            ShadeMark(SM_MEDIUM_EVENT);
            O = O + V * ScatteringTime;
            pt3 X, Y, Z = V;
            ComputeCoordinateFrame(Z, X, Y);
            float U1 = G.R01();
            float U2 = G.R01();
            pt3 Sc = SampleDirectionHG(Md.ScatteringAnisotropy, U1, U2);
            pt4 Density = Md.ScatteringRate * vexp(-Md.ScatteringRate * ScatteringTime);
            Density = Density / pt_max(PT_EPSILON, max4(Density));
            Path.Throughput = Path.Throughput * Density;
            Path.Probability = Path.Probability * Density;
            V = normalize(X * Sc.x + Y * Sc.y + Z * Sc.z);
        } else {
            ShadeMark(SM_ESCAPE);
            float ClusterPDF = Path.Probability.x + Path.Probability.y + Path.Probability.z + Path.Probability.w;
            Path.Sample = Path.Sample + EscapeContribution(S, V, Lambda, Path.Throughput, ClusterPDF);
            Path.Probability = v4s(0.0f);
        }
        return max4(Path.Probability) > PT_EPSILON;
    }

    ShadeMark(SM_SURFACE);
    pt3 Nrm = UnpackUnitVector(PN);
    pt3 TX = UnpackUnitVector(PT);
    pt3 TY = cross(Nrm, TX);
    pt3 Position = O + HitTime * V;

    pt3 Out = -v3(dot(V, TX), dot(V, TY), dot(V, Nrm));
    bool IsReal;
    pt4 ExteriorIOR = v4s(1.0f);
    uint32_t ShapePriority = HitShape;
    if (Out.z > 0) {
        IsReal = Md.Priority > ShapePriority;
        if (IsReal) ExteriorIOR = Md.IOR;
    } else {
        IsReal = Md.Priority == ShapePriority;
        if (IsReal) {
            ShadeMark(SM_EXTERIOR_MEDIUM);
            uint32_t Ext = SHAPE_INDEX_NONE;
            for (int I = 0; I < 4; I++) {
                if (Path.Active[I] == Active) continue;
                Ext = pt_umin(Ext, Path.Active[I]);
            }
            ExteriorIOR = ResolveMedium<MATS>(S, Ext, Lambda).IOR;
        }
    }

    pt3 In;
    if (IsReal) {
        ShadeMark(SM_REAL);
        bsdf_parameters P;
        P.MaterialIndex = HitMaterial;
        P.TextureUV = UV;
        P.Lambda = Lambda;
        P.ExteriorIOR = ExteriorIOR;
        pt4 T, Pr;
        if (!SampleSurfaceIntegrand<MATS, CLS>(S, G, Nrm, TX, TY, P, Out, In, T, Pr)) return false;
        float Scale = 1.0f / pt_max(PT_EPSILON, max4(Pr));
        Path.Throughput = Path.Throughput * (T * Scale);
        Path.Probability = Path.Probability * (Pr * Scale);
    } else {
        ShadeMark(SM_NOT_REAL);
        In = -Out;
    }

    // Active-shape stack update (basic_scatter.glsl:266-282): first free slot
    // on entry, first matching slot on exit; constant indices keep the four
    // slots in registers.
    if (In.z * Out.z < 0) {
        uint32_t* A = Path.Active;
        if (Out.z > 0) {
            if (A[0] == SHAPE_INDEX_NONE) A[0] = HitShape;
            else if (A[1] == SHAPE_INDEX_NONE) A[1] = HitShape;
            else if (A[2] == SHAPE_INDEX_NONE) A[2] = HitShape;
            else if (A[3] == SHAPE_INDEX_NONE) A[3] = HitShape;
        } else {
            if (A[0] == HitShape) A[0] = SHAPE_INDEX_NONE;
            else if (A[1] == HitShape) A[1] = SHAPE_INDEX_NONE;
            else if (A[2] == HitShape) A[2] = SHAPE_INDEX_NONE;
            else if (A[3] == HitShape) A[3] = SHAPE_INDEX_NONE;
        }
    }

    ShadeMark(SM_ROULETTE);
    if (G.R01() < PTP) return false;
    Path.Probability = Path.Probability * (1.0f - PTP);

    V = In.x * TX + In.y * TY + In.z * Nrm;
    O = Position + 1e-3f * V;
    return max4(Path.Probability) > PT_EPSILON;
}

// --- kernels -------------------------------------------------------------------

// One block per tile (the slot count is a multiple of 256): TileOrder needs
// every thread of the block, so no thread returns early.

__global__ __launch_bounds__(256) void raygen_kernel(dscene S, dslots L, dframe F, dparams Pm)
{
    uint32_t s = blockIdx.x * 256 + threadIdx.x;
    uint32_t x, y, stream;
    bool valid = SlotPixel(F, s, x, y, stream);
    pt3 O = v3s(0), V = v3s(0);
    if (valid) {
        rng G;
        G.State = pt_seed(x, y, StreamSeed(Pm.seed, stream));
        GenerateNewPath(S, L, F, Pm, G, s, x, y, O, V);
        StreamAccum(F, stream)[(size_t)y * F.width + x] = make_float4(0, 0, 0, 0);
    }
    TileOrderStoreRay(L, s, valid, O, V, L.pos[s] & 255u);
}

// State write (ptWriteBasicRendererState): the restored rays of one tile,
// given by slot, go to their TileOrder positions like a shade's new rays;
// every position of the tile gets a miss record (no trace of the restored
// rays exists until the next extend, which overwrites it).  The order does
// not change any result (TileOrder).
__global__ __launch_bounds__(256) void restore_rays_kernel(dslots L, dframe F, const float4* rays, uint32_t tile0)
{
    const uint32_t s = (tile0 + blockIdx.x) * 256 + threadIdx.x;
    uint32_t x, y;
    const bool valid = SlotPixel(F, s, x, y);
    const float4 r = rays[s - tile0 * 256];
    const uint32_t key = TileOrderKey(valid, UnpackUnitVector(__float_as_uint(r.w)));
    L.hit[s] = make_float4(0.0f, __uint_as_float(SHAPE_INDEX_NONE), 0.0f, 0.0f);
    L.uv[s] = make_float2(0.0f, 0.0f);
    TileOrderStoreKeyed(L, s, key, r, 0u);
}

// Ray sources of the extend kernel: the renderer's slots, or the arrays of
// the ray-query API.

struct ray_source_slots {
    dslots L;
    dframe F;
    // s is a ray POSITION (TileOrder), not a slot.
    PT_DEV bool load(uint32_t s, pt3& O, pt3& V, float& D) const
    {
        if (!PositionValid(F, s)) return false;
        float4 r = L.ray[s];
        O = v3(r.x, r.y, r.z);
        V = UnpackUnitVector(__float_as_uint(r.w));
        D = PT_HIT_TIME_LIMIT;
        return true;
    }
    PT_DEV void store(uint32_t s, const lane_state& Ln, bool vidx21) const
    {
        L.hit[s] = CompactHit(Ln, vidx21);
        L.uv[s] = make_float2(Ln.C.y, Ln.C.z);
    }
    // ShadeOrder: each wave, once all its rays are traced, stores one ballot
    // per outcome class (one word per 64 positions and class; no atomics,
    // no barrier).
    // Single-material scenes store the miss class only (ShadePosition reads
    // nothing else for them).
    PT_DEV void outcome(uint32_t q, uint32_t cls, bool classes) const
    {
        uint64_t* m = L.outcome + (size_t)(q >> 8) * (4 * PT_OUTCOME_CLASSES) + ((q >> 6) & 3u);
        if (!classes) {
            uint64_t b = __ballot(cls == PT_OUTCOME_CLASSES - 1);
            if ((q & 63u) == 0) m[4 * (PT_OUTCOME_CLASSES - 1)] = b;
            return;
        }
#pragma unroll
        for (uint32_t c = 0; c < PT_OUTCOME_CLASSES; c++) {
            uint64_t b = __ballot(cls == c);
            if ((q & 63u) == 0) m[4 * c] = b;
        }
    }
};

struct ray_source_arrays {
    PT_DEV void outcome(uint32_t, uint32_t, bool) const {}
    const float* origins;
    const uint32_t* vel;
    const float* dur;
    float4* hit;
    float2* hc;
    PT_DEV bool load(uint32_t i, pt3& O, pt3& V, float& D) const
    {
        O = v3(origins[3 * i], origins[3 * i + 1], origins[3 * i + 2]);
        V = UnpackUnitVector(vel[i]);
        D = dur[i];
        return true;
    }
    PT_DEV void store(uint32_t i, const lane_state& Ln, bool vidx21) const
    {
        hit[i] = CompactHit(Ln, vidx21);
        hc[i] = make_float2(Ln.C.y, Ln.C.z);
    }
};

template <class Src>
constexpr bool kRendererSource = std::is_same<Src, ray_source_slots>::value;

// Extend: one ray per thread, LaneStep run to completion.  (A persistent
// variant with per-wave dynamic ray fetch was measured 1.6x slower on C3: the
// refill bookkeeping cost more than the idle lanes it recovered.  Persistent
// waves claiming 64-ray chunks from a launch-wide counter, each ray traced to
// completion, were 1.5x slower too (extend 0.592 vs 0.387 ms): a CU's waves
// then trace unrelated chunks, losing the L1 reuse of a tile's four waves,
// and the dispatcher already balances the 8100 one-tile blocks.)
//
// One ray: Trace() by LaneStep to completion, the compact hit stored, and
// the ray's ShadeOrder outcome class ballotted (positions outside the image:
// class 0, shade skips them).
template <bool SPILL, int CAP, class E, class Src>
PT_DEV void ExtendRay(const dscene& S, const Src& src, tstack<SPILL, CAP, E>& st, uint32_t slot)
{
    pt3 O, V;
    float D;
    uint32_t cls = 0;
    if (src.load(slot, O, V, D)) {
        lane_state Ln;
        LaneBegin(S, Ln, O, V, D);
        no_stats ns;
        if (S.g.ShapeCount != 0) {
            while (!LaneStep<SPILL, CAP, Src, no_stats, true, E>(S, Ln, st, src, slot, ns)) {}
        }
        src.store(slot, Ln, S.vidx21 != 0);
        if (Ln.Shape == SHAPE_INDEX_NONE) {
            cls = 4;
        } else if (S.mat_classes) {
            uint32_t T = S.material[32 * (size_t)S.shapes[Ln.Shape].MaterialIndex];
            cls = T == PT_MATERIAL_TYPE_BASIC_DIFFUSE ? 0u
                : T == PT_MATERIAL_TYPE_BASIC_METAL ? 1u
                : T == PT_MATERIAL_TYPE_BASIC_TRANSLUCENT ? 2u : 3u;
        }
    }
    src.outcome(slot, cls, S.mat_classes != 0);
}

// One tile of extend: thread i traces the ray at position tile*256 + i.
template <class Src, bool SPILL, int CAP, class E>
PT_DEV void ExtendTile(const dscene& S, const Src& src, uint32_t n, uint32_t* spill, uint32_t spill_stride, E* smem,
                       uint32_t tile, bool timed, const float4* nc = nullptr, uint32_t ncn = 0)
{
    uint64_t t0 = timed ? __builtin_amdgcn_s_memtime() : 0;
    uint32_t slot = tile * 256 + threadIdx.x;
    if (slot >= n) return;
    tstack<SPILL, CAP, E> st;
    st.lds = &smem[threadIdx.x];
    st.spill = spill + slot;
    st.stride = spill_stride;
    st.nc = nc;
    st.ncn = ncn;
    ExtendRay<SPILL, CAP, E>(S, src, st, slot);
    if constexpr (kRendererSource<Src>) {
        if (timed && (threadIdx.x & 63u) == 0)
            src.L.tilecost[tile * 4 + (threadIdx.x >> 6)] = (uint32_t)(__builtin_amdgcn_s_memtime() - t0);
    }
}

// The LDS node cache's fill: nodes [0, S.node_cache) of the scene (the top
// child pairs, NodeCacheLayout), 16 B per thread and load, then a barrier
// before any lane traverses.
PT_DEV uint32_t NodeCacheFill(const dscene& S, float4* nc)
{
    const uint32_t nodes = min(S.node_cache, 2u * PT_NODE_CACHE_PAIRS);
    for (uint32_t i = threadIdx.x; i < 2 * nodes; i += 256) nc[i] = S.mesh_nodes[i];
    __syncthreads();
    return nodes;
}

template <class Src, bool SPILL, int MINW, int CAP, class E = uint32_t, bool NC = false>
__global__ __launch_bounds__(256, MINW) void extend_kernel(dscene S, Src src, uint32_t n, uint32_t* spill,
                                                                  uint32_t spill_stride)
{
    __shared__ E smem[CAP * 256];
    __shared__ float4 ncache[NC ? 4 * PT_NODE_CACHE_PAIRS : 1];
    if constexpr (kRendererSource<Src>) {
        if (src.L.stop && *src.L.stop) return;   // a guarded round past the frame's target
    }
    const uint32_t ncn = NC ? NodeCacheFill(S, ncache) : 0u;
    // Tile order: the slot renderer dispatches the tiles whose waves took
    // longest in the previous round first (tile_order_kernel), so the
    // kernel's tail holds short blocks; each wave records its own time.
    uint32_t tile = blockIdx.x;
    bool timed = false;
    if constexpr (kRendererSource<Src>) {
        if (src.L.order) {
            tile = src.L.order[blockIdx.x];
            timed = true;
        }
    }
    ExtendTile<Src, SPILL, CAP, E>(S, src, n, spill, spill_stride, smem, tile, timed, ncache, ncn);
}

// Longest-first dispatch order for the next extend: tiles by their slowest
// wave's time, descending, by a one-block counting sort over 512 log-spaced
// buckets (16 per octave).  Any order gives the same results; only the
// kernel's tail changes.
//
// Tile groups (ptSetBasicRendererSplit): group g of K owns the tiles
// t = g, g + K, ... and its segment order[start, start + count) of the
// dispatch order, which it sorts on its own stream; K = 1 is the whole frame.
__global__ __launch_bounds__(1024) void tile_order_kernel(const uint32_t* cost, uint32_t* order, uint32_t tiles,
                                                          uint32_t groups, uint32_t group, uint32_t start)
{
    const uint32_t nt = pt_tile_group_count(tiles, groups, group);
    __shared__ uint32_t count[512];
    for (uint32_t i = threadIdx.x; i < 512; i += 1024) count[i] = 0;
    __syncthreads();
    auto key = [&](uint32_t t) -> uint32_t {
        uint32_t c = max(max(cost[4 * t], cost[4 * t + 1]), max(cost[4 * t + 2], cost[4 * t + 3]));
        if (c < 16) return 511u;                               // untimed / trivial: last
        uint32_t e = 31u - __clz(c);                           // octave
        uint32_t m = (c >> (e - 4)) & 15u;                     // 16 steps inside it
        uint32_t k = min(e * 16u + m, 511u);
        return 511u - k;                                       // longest first
    };
    for (uint32_t i = threadIdx.x; i < nt; i += 1024) atomicAdd(&count[key(pt_tile_group_tile(tiles, groups, group, i))], 1u);
    __syncthreads();
    // Exclusive scan of the 512 buckets: eight waves scan 64 each with
    // shuffles, then add the totals of the waves before them (a serial scan
    // by one thread was most of this kernel's 11 us).
    __shared__ uint32_t wsum[8];
    uint32_t c = 0, incl = 0;
    if (threadIdx.x < 512) {
        c = count[threadIdx.x];
        incl = c;
        for (int o = 1; o < 64; o <<= 1) {
            uint32_t t = (uint32_t)__shfl_up((int)incl, o, 64);
            if ((threadIdx.x & 63u) >= (uint32_t)o) incl += t;
        }
        if ((threadIdx.x & 63u) == 63u) wsum[threadIdx.x >> 6] = incl;
    }
    __syncthreads();
    if (threadIdx.x < 512) {
        uint32_t before = 0;
        for (uint32_t w = 0; w < (threadIdx.x >> 6); w++) before += wsum[w];
        count[threadIdx.x] = before + incl - c;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nt; i += 1024) {
        const uint32_t t = pt_tile_group_tile(tiles, groups, group, i);
        order[start + atomicAdd(&count[key(t)], 1u)] = t;
    }
}

// Guarded rounds (ptRenderFrame's last rounds, enqueued without a read-back
// between them): before each, the paths completed since the Reset -- the sum
// of the per-wave done words, as ptGetStats adds them -- against the frame's
// target.  Reached: flags[0] = 1, and this and every later launch of the
// frame returns at once (dslots.stop); else the round runs and flags[1]
// counts it.  So the frame still ends at the first round whose total reaches
// the target.
__global__ __launch_bounds__(1024) void guard_kernel(const uint32_t* done, uint32_t words, unsigned long long target,
                                                     uint32_t* flags)
{
    __shared__ unsigned long long part[1024];
    unsigned long long s = 0;
    for (uint32_t i = threadIdx.x; i < words; i += 1024) s += done[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (uint32_t h = 512; h > 0; h >>= 1) {
        if (threadIdx.x < h) part[threadIdx.x] += part[threadIdx.x + h];
        __syncthreads();
    }
    if (threadIdx.x == 0 && flags[0] == 0u) {
        if (part[0] >= target) flags[0] = 1u;
        else flags[1] += 1u;
    }
}

// Mesh vertices decoded once per upload for HitAttributes: the octahedral
// normal (UnpackUnitVector) and the half-float UV, the functions the hit
// reconstruction applied per hit before, so every hit sees the same bits.
__global__ __launch_bounds__(256) void vertex_decode_kernel(const uint2* v, uint32_t n, float4* attr, float* vv)
{
    uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint2 V = v[i];
    pt3 N = UnpackUnitVector(V.x);
    attr[i] = make_float4(N.x, N.y, N.z, pt_half_to_float(V.y & 0xFFFF));
    vv[i] = pt_half_to_float(V.y >> 16);
}

// Row-major packed atlas -> the device's 4x2-texel block layout (AtlasIndex):
// one thread per destination texel, so the stores are contiguous.
__global__ __launch_bounds__(256) void atlas_tile_kernel(const float4* src, float4* dst, uint32_t w, uint32_t h,
                                                         uint64_t texels)
{
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < texels; i += (uint64_t)gridDim.x * 256) {
        uint64_t plane = (uint64_t)w * h;
        uint64_t layer = i / plane, r = i - layer * plane;
        uint32_t blk = (uint32_t)(r >> 3), in = (uint32_t)(r & 7u);
        uint32_t by = blk / (w >> 2), bx = blk - by * (w >> 2);
        uint32_t x = bx * 4 + (in & 3u), y = by * 2 + (in >> 2);
        dst[i] = src[layer * plane + (uint64_t)y * w + x];
    }
}

// Path streams' merge (ptMergeBasicRendererStreams): for every pixel of the
// renderer's bands, accum = ((accx[0] + accx[1]) + accx[2]) ... in stream
// order; the streams' own accumulators keep running.
__global__ __launch_bounds__(256) void merge_streams_kernel(float4* accum, float4* accx, uint32_t width, uint32_t height,
                                                            uint32_t rank, uint32_t nranks, uint32_t streams)
{
    const size_t frame = (size_t)width * height;
    for (uint32_t y = blockIdx.y; y < height; y += gridDim.y) {
        if (((y >> 4) % nranks) != rank) continue;
        for (uint32_t x = blockIdx.x * 256 + threadIdx.x; x < width; x += gridDim.x * 256) {
            const size_t p = (size_t)y * width + x;
            float4 v = accx[p];
            for (uint32_t k = 1; k < streams; k++) {
                float4 a = accx[(size_t)k * frame + p];
                v.x = v.x + a.x; v.y = v.y + a.y; v.z = v.z + a.z; v.w = v.w + a.w;
            }
            accum[p] = v;
        }
    }
}

// Record forms of the live paths (GreyRecord, StorePathVertex).  Only slots
// of pixels inside the image hold paths.
__global__ __launch_bounds__(256) void grey_check_kernel(dslots L, dframe F, uint32_t* count)
{
    const uint32_t s = blockIdx.x * 256 + threadIdx.x;
    uint32_t x, y;
    bool bad = false;
    if (s < L.n && SlotPixel(F, s, x, y)) {
        const float4 p = L.prob[s];
        const uint2 a = L.act[s];
        const uint32_t b = __float_as_uint(p.x);
        bad = b != __float_as_uint(p.y) || b != __float_as_uint(p.z) || b != __float_as_uint(p.w) ||
              (a.x & a.y) != 0xFFFFFFFFu;
    }
    const uint64_t m = __ballot(bad);
    if ((threadIdx.x & 63u) == 0 && m) atomicAdd(count, (uint32_t)__popcll(m));
}

__global__ __launch_bounds__(256) void grey_convert_kernel(dslots L, dframe F, float* prob1, bool to_grey)
{
    const uint32_t s = blockIdx.x * 256 + threadIdx.x;
    uint32_t x, y;
    if (s >= L.n || !SlotPixel(F, s, x, y)) return;
    if (to_grey) {
        prob1[s] = L.prob[s].x;
    } else {
        const float c = prob1[s];
        L.prob[s] = make_float4(c, c, c, c);
        L.act[s] = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
    }
}

__global__ __launch_bounds__(256) void zero_unowned_kernel(float4* accum, uint32_t width, uint32_t height,
                                                           uint32_t rank, uint32_t nranks)
{
    for (uint32_t y = blockIdx.y; y < height; y += gridDim.y) {
        if (((y >> 4) % nranks) == rank) continue;
        for (uint32_t x = blockIdx.x * 256 + threadIdx.x; x < width; x += gridDim.x * 256)
            accum[(size_t)y * width + x] = make_float4(0, 0, 0, 0);
    }
}

PT_DEV uint32_t WaveSum(uint32_t v)
{
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

PT_DEV uint32_t WaveMax(uint32_t v)
{
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor(v, o, 64));
    return v;
}

// Diagnostic extend: the same traversal with per-lane counters, reduced per
// wave into out[]: {rays, lane steps, wave steps x 64, internal nodes, BLAS
// leaves, faces tested, stack pops, TLAS leaves (shapes), waves, then the
// internal-BLAS wave steps by distinct node count 1, 2, 3-4, 5-8, >8}.  SIMD
// efficiency of the traversal loop = lane steps / (wave steps x 64).
template <class Src, bool SPILL, int CAP, class E = uint32_t>
__global__ __launch_bounds__(256) void extend_stats_kernel(dscene S, Src src, uint32_t n, uint32_t* spill,
                                                           uint32_t spill_stride, unsigned long long* out,
                                                           uint32_t* steps)
{
    __shared__ E smem[CAP * 256];
    uint32_t slot = blockIdx.x * 256 + threadIdx.x;
    tstack<SPILL, CAP, E> st;
    st.lds = &smem[threadIdx.x];
    st.spill = spill + slot;
    st.stride = spill_stride;
    lane_stats ss;
    pt3 O, V;
    float D;
    uint32_t ray = 0;
    if (slot < n && src.load(slot, O, V, D)) {
        ray = 1;
        lane_state Ln;
        LaneBegin(S, Ln, O, V, D);
        if (S.g.ShapeCount != 0)
            while (!LaneStep<SPILL, CAP, Src, lane_stats, true, E>(S, Ln, st, src, slot, ss)) {}
        src.store(slot, Ln, S.vidx21 != 0);
    }
    if (steps && slot < n) steps[slot] = ss.steps;   // per position (0: no ray)
    uint32_t v[14] = {WaveSum(ray), WaveSum(ss.steps), WaveMax(ss.steps) * 64u, WaveSum(ss.internals),
                      WaveSum(ss.leaves), WaveSum(ss.faces), WaveSum(ss.pops), WaveSum(ss.shapes), 1u,
                      WaveSum(ss.uniq[0]), WaveSum(ss.uniq[1]), WaveSum(ss.uniq[2]), WaveSum(ss.uniq[3]),
                      WaveSum(ss.uniq[4])};
    if ((threadIdx.x & 63u) == 0)
        for (int i = 0; i < 14; i++) atomicAdd(&out[i], (unsigned long long)v[i]);
}

// Compact hit -> the reference's packed trace record (StoreTraceHit,
// basic.glsl.inc:142-157): {time, shape<<16|material, packed normal, packed
// tangent} + uv.  Used by the ray-query API and the state readback.
__global__ __launch_bounds__(256) void finalize_kernel(dscene S, uint32_t n, const float4* hit, const float2* hc,
                                                       float4* rec, float2* uv)
{
    uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float4 h = hit[i];
    uint32_t Shape = __float_as_uint(h.y);
    if (Shape == SHAPE_INDEX_NONE) {
        rec[i] = make_float4(0, __uint_as_float(0xFFFFFFFFu), 0, 0);
        uv[i] = make_float2(0, 0);
        return;
    }
    float2 c = hc[i];
    uint32_t Material;
    pt3 N, TX;
    pt2 UV;
    HitAttributesRecord(S, Shape, h, c, Material, N, TX, UV);
    rec[i] = make_float4(h.x, __uint_as_float((Shape << 16) | Material), __uint_as_float(PackUnitVector(N)),
                         __uint_as_float(PackUnitVector(TX)));
    uv[i] = make_float2(UV.x, UV.y);
}

#ifndef PT_SHADE_DIFFUSE_MINW
#define PT_SHADE_DIFFUSE_MINW 5
#endif
// Occupancy floor of the other shade instantiations (metal / translucent /
// medium code compiled in): 5 waves per SIMD (96 VGPRs, a few spills of
// rarely live values) beat the compiler's 106-108 VGPRs at 4 waves: C5
// shade 0.190 -> 0.179 ms, C2 0.111 -> 0.104 ms.
#ifndef PT_SHADE_OTHER_MINW
#define PT_SHADE_OTHER_MINW 5
#endif
// The OpenPBR instantiation (opt-in) carries the layered sampler as well:
// 160 VGPRs (3 waves/SIMD) unbounded; a 4-wave floor caps it at 128 with
// 84 B of spills and is faster (OpenPBR test scene at 1080p: shade 0.523 vs
// 0.568 ms, profiles/r02_next).
#ifndef PT_SHADE_OPENPBR_MINW
#define PT_SHADE_OPENPBR_MINW 4
#endif
template <uint32_t MATS>
constexpr int ShadeMinWaves()
{
    return (MATS & ~(uint32_t)PT_MATS_SCENE) == PT_MATS_DIFFUSE ? PT_SHADE_DIFFUSE_MINW
         : (MATS & PT_MATS_OPENPBR) ? PT_SHADE_OPENPBR_MINW : PT_SHADE_OTHER_MINW;
}
// A completed path (basic_scatter.glsl:344-359): its Sample accumulated into
// the pixel (alpha counts the sample) and a new camera path generated with
// the slot's RNG continuing from Scatter's draws.
PT_DEV void CompletePath(const dscene& S, const dslots& L, const dframe& F, const dparams& Pm, rng& G, uint32_t s,
                         uint32_t x, uint32_t y, uint32_t stream, pt3 Sample, bool act_none, pt3& O, pt3& V)
{
    float4* A = &StreamAccum(F, stream)[(size_t)y * F.width + x];
    float4 Val = make_float4(Sample.x, Sample.y, Sample.z, 1.0f);
    if (Pm.render_flags & PT_RENDER_FLAG_ACCUMULATE) {
        float4 Old = *A;
        Val.x = Val.x + Old.x; Val.y = Val.y + Old.y; Val.z = Val.z + Old.z; Val.w = Val.w + Old.w;
    }
    *A = Val;
    GenerateNewPath(S, L, F, Pm, G, s, x, y, O, V, act_none);
}

// Shade one slot (basic_scatter.glsl:main): load its path and its ray's hit
// (at position p16 >> 8), Scatter, store the continuing path or complete it.
// COMPACT: a completed path is left to the block's completion queue (its RNG
// state, Sample and empty-stack flag in cstate / csample / cactnone); else it
// is completed here and its new camera ray returned in O, V.
template <uint32_t MATS, bool COMPACT, uint32_t CLS = 0xFFFFFFFFu>
PT_DEV void ShadeSlot(const dscene& S, const dslots& L, const dframe& F, const dparams& Pm, uint32_t s, uint32_t p16,
                      uint32_t x, uint32_t y, uint32_t stream, bool valid, pt3& O, pt3& V, bool& completed,
                      uint32_t& cstate, pt3& csample, bool& cactnone)
{
    if (valid) {
        ShadeMark(SM_ENTRY);
        rng G;
        G.State = pt_seed(x, y, StreamSeed(Pm.seed, stream));

        // LoadPath (basic.glsl.inc:159-198).  Grey record form (StorePathVertex):
        // one Probability float, and the empty stack without a load.
        const bool grey = pt_grey_mats(MATS) && L.prob1 != nullptr;
        path P;
        float4 thr = L.thr[s];
        uint2 act;
        if (grey) {
            P.Probability = v4s(L.prob1[s]);
            act = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
        } else {
            float4 prob = L.prob[s];
            P.Probability = v4(prob.x, prob.y, prob.z, prob.w);
            act = L.act[s];
        }
        P.Throughput = v4(thr.x, thr.y, thr.z, thr.w);
        P.Sample = v3s(0.0f);          // always 0 between rounds (StorePathVertex)
        P.Lambda0 = L.lam[s];
        P.Active[0] = act.x & 0xFFFF; P.Active[1] = act.x >> 16;
        P.Active[2] = act.y & 0xFFFF; P.Active[3] = act.y >> 16;
        for (int I = 0; I < 4; I++)
            if (P.Active[I] == 0xFFFF) P.Active[I] = SHAPE_INDEX_NONE;

        // LoadTraceResult (basic.glsl.inc:99-131).  The extend kernel leaves a
        // compact hit at the ray's position; the trace record's attributes
        // (Trace, scene.glsl.inc:535-608) are rebuilt here and go through the
        // same octahedral snorm16 quantisation as the reference's
        // StoreTraceHit / LoadTraceResult.
        uint32_t q = RayPos(L, s, p16);
        float4 r = L.ray[q];
        O = v3(r.x, r.y, r.z);
        V = UnpackUnitVector(__float_as_uint(r.w));
        float4 h = L.hit[q];
        uint32_t HitShape = __float_as_uint(h.y), HitMaterial = 0;
        float HitTime = PT_HIT_TIME_LIMIT;
        uint32_t PN = 0, PTg = 0;
        pt2 UV = v2(0, 0);
        if (HitShape != SHAPE_INDEX_NONE) {
            ShadeMark(SM_HIT);
#if PT_SHADE_STATS
            {
                const int32_t Ty = S.shapes[HitShape].Type;
                if (Ty == PT_SHAPE_TYPE_MESH_INSTANCE) ShadeMark(SM_MESH_HIT);
                else if (Ty == PT_SHAPE_TYPE_SPHERE) ShadeMark(SM_SPHERE_HIT);
                else if (Ty == PT_SHAPE_TYPE_PLANE) ShadeMark(SM_PLANE_HIT);
                else ShadeMark(SM_CUBE_HIT);
            }
#endif
            float2 c = L.uv[q];
            pt3 N, TX;
            HitAttributesRecord(S, HitShape, h, c, HitMaterial, N, TX, UV, /*uv_if_textured=*/true,
                                /*prims=*/(MATS & PT_MATS_PRIMS) != 0);
            HitMaterial &= 0xFFFFu;
            HitShape &= 0xFFFFu;
            HitTime = h.x;
            PN = PackUnitVector(N);
            PTg = PackUnitVector(TX);
        }

        if (Scatter<MATS, CLS>(S, G, Pm.termination_probability, P, O, V, HitShape, HitMaterial, HitTime, PN, PTg, UV)) {
            // StorePathVertex of a continuing path: Scatter changes Sample only
            // on escape (which terminates the path) and never Lambda0, so lam
            // is unchanged; the active-shape stack is written when it moved.
            ShadeMark(SM_CONTINUE);
            L.thr[s] = make_float4(P.Throughput.x, P.Throughput.y, P.Throughput.z, P.Throughput.w);
            if (grey) {
                L.prob1[s] = P.Probability.x;
            } else {
                L.prob[s] = make_float4(P.Probability.x, P.Probability.y, P.Probability.z, P.Probability.w);
                uint2 na = make_uint2((P.Active[1] << 16) | P.Active[0], (P.Active[3] << 16) | P.Active[2]);
                if ((na.x != act.x) | (na.y != act.y)) L.act[s] = na;
            }
        } else {
            ShadeMark(SM_COMPLETED);
            completed = true;
            if constexpr (COMPACT) {
                cstate = G.State;
                csample = P.Sample;
                cactnone = (act.x & act.y) == 0xFFFFFFFFu;
            } else {
                CompletePath(S, L, F, Pm, G, s, x, y, stream, P.Sample, (act.x & act.y) == 0xFFFFFFFFu, O, V);
            }
        }
    }
}

// Completion queue (COMPACT shade).  Paths that end at a surface (a sky
// sample below the horizon, roulette, a failed BSDF sample) are scattered over
// the tile's hit waves, so the completion work -- accumulate, then a new
// camera path (GenerateNewPath) -- ran in nearly every wave at a third of its
// lanes (C2: 99 % of waves, 25 lanes).  Here the completed slots of the block
// (cm: this wave's ballot) are queued in LDS in thread order, the first
// threads of the block complete them in full waves, and the new rays come
// back through LDS to their slots' threads.  The same operations on the same
// values: bit-identical.
PT_DEV void CompletionQueue(const dscene& S, const dslots& L, const dframe& F, const dparams& Pm, uint32_t s,
                            bool completed, uint64_t cm, uint32_t cstate, pt3 csample, bool cactnone, pt3& O, pt3& V)
{
    __shared__ uint32_t cq_slot[256], cq_rng[256], cq_count[4];
    __shared__ float cq_f[6][256];
    const uint32_t w = threadIdx.x >> 6;
    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(cm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)cm, 0u));
    if ((threadIdx.x & 63u) == 0) cq_count[w] = (uint32_t)__popcll(cm);
    __syncthreads();
    uint32_t qi = below, total = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
        const uint32_t c = cq_count[k];
        qi += k < w ? c : 0u;
        total += c;
    }
    if (completed) {
        cq_slot[qi] = s | (cactnone ? 0x80000000u : 0u);   // slots < 2^31 (renderer creation)
        cq_rng[qi] = cstate;
        cq_f[0][qi] = csample.x; cq_f[1][qi] = csample.y; cq_f[2][qi] = csample.z;
    }
    __syncthreads();
    const uint32_t t = threadIdx.x;
    if (t < total) {
        const uint32_t e = cq_slot[t];
        const uint32_t s2 = e & 0x7FFFFFFFu;
        uint32_t x2, y2, stream2;
        (void)SlotPixel(F, s2, x2, y2, stream2);
        rng G2;
        G2.State = cq_rng[t];
        pt3 O2, V2;
        CompletePath(S, L, F, Pm, G2, s2, x2, y2, stream2, v3(cq_f[0][t], cq_f[1][t], cq_f[2][t]),
                     (e & 0x80000000u) != 0, O2, V2);
        cq_f[0][t] = O2.x; cq_f[1][t] = O2.y; cq_f[2][t] = O2.z;   // each thread rewrites only its own entry
        cq_f[3][t] = V2.x; cq_f[4][t] = V2.y; cq_f[5][t] = V2.z;
    }
    __syncthreads();
    if (completed) {
        O = v3(cq_f[0][qi], cq_f[1][qi], cq_f[2][qi]);
        V = v3(cq_f[3][qi], cq_f[4][qi], cq_f[5][qi]);
    }
}

// One tile of shade (basic_scatter.glsl:main for the tile's 256 slots).
// COMPACT: completion queue, for scenes whose paths also end at surfaces
// (ShadeCompact, runtime.hip).
template <uint32_t MATS, bool COMPACT = false>
PT_DEV void ShadeTile(const dscene& S, const dslots& L, const dframe& F, const dparams& Pm, uint32_t tile)
{
    // One block per tile, no early exit (TileOrder).  ShadeOrder: thread u
    // shades the slot whose ray sits at ShadePosition(u), so the waves of a
    // tile run the surface path or the escape path, mostly not both; path
    // state is read and written by slot (gathers within the tile's records).
    // The position is the ray's own (slotof inverts TileOrder's slot ->
    // position map), so the ray / hit / uv records load from it directly,
    // beside the slotof lookup instead of after a pos[s] lookup.
    const uint32_t base = tile * 256;
    const uint64_t* om = L.outcome + (size_t)tile * (4 * PT_OUTCOME_CLASSES);
    const uint32_t pq = S.mat_classes ? ShadePosition(om, threadIdx.x)
                                      : ShadePosition2(om + 4 * (PT_OUTCOME_CLASSES - 1), threadIdx.x);
    const uint32_t s = base | L.slotof[base | pq];
    const uint32_t p16 = pq << 8;   // RayPos(s, p16) == base | pq (shade -1 % vs gathering pos[s])
    uint32_t x, y, stream;
    bool valid = SlotPixel(F, s, x, y, stream);
    pt3 O = v3s(0), V = v3s(0);
    bool completed = false;
    uint32_t cstate = 0;
    pt3 csample = v3s(0.0f);
    bool cactnone = false;
    ShadeSlot<MATS, COMPACT>(S, L, F, Pm, s, p16, x, y, stream, valid, O, V, completed, cstate, csample, cactnone);
    // Completed paths per wave (ptGetStats): one counter word per 64 slots,
    // updated by the wave's first lane (no atomics: a wave owns its word).
    uint64_t cm = __ballot(completed);
    if ((threadIdx.x & 63u) == 0) L.done[(base | threadIdx.x) >> 6] += (uint32_t)__popcll(cm);
    if constexpr (COMPACT) CompletionQueue(S, L, F, Pm, s, completed, cm, cstate, csample, cactnone, O, V);
    TileOrderStoreRay(L, s, valid, O, V, p16 >> 8);
}

template <uint32_t MATS, bool COMPACT>
__global__ __launch_bounds__(256, ShadeMinWaves<MATS>()) void shade_kernel(dscene S, dslots L, dframe F,
                                                                                    dparams Pm)
{
    // Tiles in extend's longest-first order too: tiles with long traversals
    // also shade more hits (C5 shade -3 %).
    if (L.stop && *L.stop) return;   // a guarded round past the frame's target
    ShadeStatsBegin();
    ShadeTile<MATS, COMPACT>(S, L, F, Pm, L.order ? L.order[blockIdx.x] : blockIdx.x);
    ShadeStatsEnd();
}

// Class-pure shade (round 5).  Every position of a round
// goes to the global list of its outcome class (extend's ShadeOrder classes:
// hit diffuse / metal / translucent / other material, miss), and
// shade_classq_kernel gives each block 256 entries of one class, so every
// wave shades one class with that class's BSDF code alone (ShadeSlot's CLS).
// A new ray stays at the position it replaces: TileOrder needs a tile's 256
// new rays together, which a class-pure block does not hold; the slot <->
// position map is unchanged, so the results are identical.  Used inside tile
// groups (runtime.hip ClassLists), where the lists' latency and the gathers'
// extra bytes overlap the other groups' launches: C2 +6 %, C5 +6 %; on one
// stream the lists cost more than the lanes gain.
//
// class_list_kernel builds the lists between extend and shade.  A block
// lists CQ_TILES tiles: one wave scans the (tile, wave word) counts of every
// class and takes the block's run of each class's list with one atomic per
// class, lanes 0..C-1 at once (a tile per block instead: 4096 atomics per
// address per C2 round, serialised, 26 us).  Block 0 clears the other
// parity's counters for the next round.
constexpr uint32_t CQ_TILES = 16;
__global__ __launch_bounds__(256) void class_list_kernel(dslots L, uint32_t mat_classes, uint32_t* counts,
                                                         uint32_t* next_counts, uint32_t* list, uint32_t capk,
                                                         uint32_t tiles_all, uint32_t groups, uint32_t group)
{
    // L.tile_count tiles of tile group `group` (all tiles: groups = 1).
    if (L.stop && *L.stop) return;   // a guarded round past the frame's target
    auto TILE = [&](uint32_t j) { return pt_tile_group_tile(tiles_all, groups, group, j); };
    constexpr uint32_t C = PT_OUTCOME_CLASSES;
    static_assert(CQ_SUB == 1 && 4 * CQ_TILES <= 64, "one list per class; one wave scans the block's counts");
    __shared__ uint64_t om_s[CQ_TILES * 4 * C];
    __shared__ uint32_t off[C][4 * CQ_TILES];
    __shared__ uint32_t base[C];
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    const uint32_t tile0 = blockIdx.x * CQ_TILES;
    const uint32_t ntiles = L.tile_count - tile0 < CQ_TILES ? L.tile_count - tile0 : CQ_TILES;
    if (blockIdx.x == 0 && t < C) next_counts[t] = 0u;
    for (uint32_t i = t; i < ntiles * 4 * C; i += 256)
        om_s[i] = L.outcome[(size_t)TILE(tile0 + i / (4 * C)) * (4 * C) + i % (4 * C)];
    __syncthreads();
    auto mask = [&](uint32_t j, uint32_t c, uint32_t k) -> uint64_t {
        const uint64_t* om = om_s + j * (4 * C);
        if (mat_classes) return om[4 * c + k];
        const uint64_t miss = om[4 * (C - 1) + k];
        return c == C - 1 ? miss : c == 0 ? ~miss : 0ull;
    };
    if (t < 64) {
        const uint32_t j = t >> 2, k = t & 3u;
        uint32_t total = 0;
#pragma unroll
        for (uint32_t c = 0; c < C; c++) {
            const uint32_t n = j < ntiles ? (uint32_t)__popcll(mask(j, c, k)) : 0u;
            uint32_t x = n;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
                if ((int)lane >= o) x += y;
            }
            off[c][t] = x - n;
            const uint32_t xt = (uint32_t)__shfl((int)x, 63, 64);
            if (lane == c) total = xt;
        }
        if (lane < C) base[lane] = total ? atomicAdd(&counts[lane], total) : 0u;
    }
    __syncthreads();
    for (uint32_t j = 0; j < ntiles; j++) {
        const uint32_t q = TILE(tile0 + j) * 256 + t;
#pragma unroll
        for (uint32_t c = 0; c < C; c++) {
            const uint64_t m = mask(j, c, w);
            if ((m >> lane) & 1ull) {
                const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                list[(size_t)c * capk + base[c] + off[c][4 * j + w] + r] = q;
            }
        }
    }
}

template <uint32_t MATS, bool COMPACT>
__global__ __launch_bounds__(256, ShadeMinWaves<MATS>()) void shade_classq_kernel(dscene S, dslots L, dframe F,
                                                                                         dparams Pm,
                                                                                         const uint32_t* counts,
                                                                                         const uint32_t* list,
                                                                                         uint32_t capk)
{
    constexpr uint32_t C = PT_OUTCOME_CLASSES;
    if (L.stop && *L.stop) return;   // a guarded round past the frame's target
    // Sub-list starts and class totals from the CQ_SUB x C counters
    // (uniform scalar loads; no barrier).
    uint32_t pre[C][CQ_SUB], tot[C];
#pragma unroll
    for (uint32_t k = 0; k < C; k++) {
        uint32_t x = 0;
#pragma unroll
        for (uint32_t j = 0; j < CQ_SUB; j++) { pre[k][j] = x; x += counts[k * CQ_SUB + j]; }
        tot[k] = x;
    }
    uint32_t c = C, i0 = 0, n = 0, start = 0;
#pragma unroll
    for (uint32_t k = 0; k < C; k++) {
        const uint32_t nk = tot[k];
        const uint32_t bk = (nk + 255u) / 256u;
        if (c == C && blockIdx.x < start + bk) { c = k; i0 = (blockIdx.x - start) * 256u; n = nk; }
        start += bk;
    }
    if (c == C) return;   // whole block: past every list
    const uint32_t i = i0 + threadIdx.x;
    const bool in = i < n;
    uint32_t sub = 0, first = 0;   // the last sub-list starting at or before i
#pragma unroll
    for (uint32_t k = 0; k < C; k++) {
        if (k != c) continue;
#pragma unroll
        for (uint32_t j = 1; j < CQ_SUB; j++)
            if (pre[k][j] <= i) { sub = j; first = pre[k][j]; }
    }
    const uint32_t q = in ? list[((size_t)c * CQ_SUB + sub) * capk + (i - first)] : 0u;
    const uint32_t s = (q & ~255u) | L.slotof[q];
    uint32_t x = 0, y = 0, stream = 0;
    const bool valid = in && SlotPixel(F, s, x, y, stream);
    const uint32_t p16 = (q & 255u) << 8;
    pt3 O = v3s(0), V = v3s(0);
    bool completed = false;
    uint32_t cstate = 0;
    pt3 csample = v3s(0.0f);
    bool cactnone = false;
    switch (c) {
    case 0:
        ShadeSlot<MATS, COMPACT, PT_MATS_DIFFUSE>(S, L, F, Pm, s, p16, x, y, stream, valid, O, V, completed, cstate,
                                                  csample, cactnone);
        break;
    case 1:
        ShadeSlot<MATS, COMPACT, PT_MATS_METAL>(S, L, F, Pm, s, p16, x, y, stream, valid, O, V, completed, cstate,
                                                csample, cactnone);
        break;
    case 2:
        ShadeSlot<MATS, COMPACT, PT_MATS_TRANSLUCENT>(S, L, F, Pm, s, p16, x, y, stream, valid, O, V, completed,
                                                      cstate, csample, cactnone);
        break;
    case PT_OUTCOME_CLASSES - 1:
        ShadeSlot<MATS, COMPACT, 0u>(S, L, F, Pm, s, p16, x, y, stream, valid, O, V, completed, cstate, csample,
                                     cactnone);
        break;
    default:
        ShadeSlot<MATS, COMPACT>(S, L, F, Pm, s, p16, x, y, stream, valid, O, V, completed, cstate, csample, cactnone);
        break;
    }
    const uint64_t cm = __ballot(completed);
    const uint32_t words = L.n / 64;
    if ((threadIdx.x & 63u) == 0 && cm && words)
        atomicAdd(&L.done[((blockIdx.x * 256u + threadIdx.x) >> 6) % words], (uint32_t)__popcll(cm));
    if constexpr (COMPACT) CompletionQueue(S, L, F, Pm, s, completed, cm, cstate, csample, cactnone, O, V);
    if (valid) {
        L.ray[q] = make_float4(O.x, O.y, O.z, __uint_as_float(PackUnitVector(V)));
        L.pos[s] = (uint16_t)(((q & 255u) << 8) | (q & 255u));
    }
}


// One round (extend + shade) of a tile per block, for partitions whose tiles
// all fit on the GPU at once (a rank's share of a strongly scaled frame):
// a tile is shaded as soon as its own rays are traced, so the shading of
// most tiles runs beside the few long traversals that end the round instead
// of after them, and one launch replaces two.  Same per-tile work and order
// as extend_kernel then shade_kernel, so the results are identical.
template <uint32_t MATS, int CAP, class E>
__global__ __launch_bounds__(256, ShadeMinWaves<MATS>()) void round_kernel(
    dscene S, dslots L, dframe F, dparams Pm)
{
    __shared__ E smem[CAP * 256];
    if (L.stop && *L.stop) return;   // a guarded round past the frame's target
    const uint32_t tile = L.order ? L.order[blockIdx.x] : blockIdx.x;
    ExtendTile<ray_source_slots, false, CAP, E>(S, ray_source_slots{L, F}, L.n, nullptr, 0, smem, tile,
                                                 L.order != nullptr);
    // The tile's hits and outcome masks (global, written by all four waves)
    // are complete and visible to the block after the barrier.
    __syncthreads();
    ShadeTile<MATS>(S, L, F, Pm, tile);
}

// Round batches: Pm.rounds rounds of one tile per block.  A slot's round
// depends only on its own previous round (its ray, path record and pixel;
// the seed is the round's FrameIndex), so tiles need no grid-wide barrier
// between rounds: a block runs its tile's extend and shade Pm.rounds times
// with the seeds of consecutive Run(1) calls (seed_step 1) or of one Run(R)
// (seed_step 0), and the launch has one tail per batch instead of two per
// round.  Barriers between the phases make the tile's hits (extend -> shade)
// and new rays (shade -> next extend, TileOrder positions) visible to the
// block's other waves.  The block's whole time is the tile's cost for the
// next batch's longest-first order.
template <uint32_t MATS, int CAP, class E>
__global__ __launch_bounds__(256, ShadeMinWaves<MATS>()) void rounds_kernel(
    dscene S, dslots L, dframe F, dparams Pm)
{
    __shared__ E smem[CAP * 256];
    const uint32_t tile = L.order ? L.order[blockIdx.x] : blockIdx.x;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    dparams P = Pm;
    for (uint32_t i = 0; i < Pm.rounds; i++) {
        ExtendTile<ray_source_slots, false, CAP, E>(S, ray_source_slots{L, F}, L.n, nullptr, 0, smem, tile, false);
        __syncthreads();
        ShadeTile<MATS>(S, L, F, P, tile);
        __syncthreads();
        P.seed += Pm.seed_step;
    }
    if (L.order && (threadIdx.x & 63u) == 0)
        L.tilecost[tile * 4 + (threadIdx.x >> 6)] = (uint32_t)(__builtin_amdgcn_s_memtime() - t0);
}

// Exhaustive check of FastRcp: every bit pattern d = i (i < 2^32); counts
// d in FastRcpRange whose FastRcp(d) differs from 1.0f / d in any bit.
__global__ __launch_bounds__(256) void rcp_check_kernel(unsigned long long* mismatches)
{
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint64_t stride = (uint64_t)gridDim.x * 256;
    unsigned long long bad = 0;
    for (; i < (1ull << 32); i += stride) {
        float d = __uint_as_float((uint32_t)i);
        if (!FastRcpRange(d)) continue;
        bad += __float_as_uint(FastRcp(d)) != __float_as_uint(1.0f / d);
    }
    if (bad) atomicAdd(mismatches, bad);
}

// Checks XDiv against IEEE division on device-generated operands: counts
// mismatching bit patterns (test infrastructure for the convention).
__global__ __launch_bounds__(256) void xdiv_check_kernel(uint64_t n, uint32_t seed, unsigned long long* mismatches)
{
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint64_t stride = (uint64_t)gridDim.x * 256;
    unsigned long long bad = 0;
    for (; i < n; i += stride) {
        uint32_t s = (uint32_t)i * 2654435761u ^ seed;
        uint32_t ra = pt_random(&s), rb = pt_random(&s), rc = pt_random(&s);
        // exponents spread over +-2^40 around 1, random signs and mantissas
        float a = pt_u2f(((87u + (ra >> 26) + (rc & 15)) << 23) | (ra & 0x7fffffu) | ((rc >> 31) << 31));
        float b = pt_u2f(((107u + ((rb >> 27) & 31)) << 23) | (rb & 0x7fffffu) | (((rc >> 30) & 1u) << 31));
        if ((rc & 0xff0) == 0) a = 0.0f;
        if ((rc & 0xff00) == 0) b = 0.0f;
        float y = RecipForDiv(b);
        float q = XDiv(a, b, y);
        float e = a / b;
        if (pt_f2u(q) != pt_f2u(e) && !(q != q && e != e)) bad++;
    }
    if (bad) atomicAdd(mismatches, bad);
}

}  // namespace ptd

// --- launchers (called from runtime.cpp) ----------------------------------------

namespace {
inline uint32_t Blocks(uint32_t n) { return (n + 255) / 256; }
}

hipError_t pt_launch_raygen(const ptd::dscene& S, const ptd::dslots& L, const ptd::dframe& F, const ptd::dparams& P,
                            hipStream_t st)
{
    if (L.n == 0) return hipSuccess;
    hipLaunchKernelGGL(ptd::raygen_kernel, dim3(Blocks(L.n)), dim3(256), 0, st, S, L, F, P);
    return hipGetLastError();
}

// Extend occupancy: min waves per SIMD and LDS stack entries per thread
// (entries beyond the LDS capacity spill to a global buffer).  Compile-time
// only (tools/build_variant.py -DPT_EXTEND_MINW=.. -DPT_EXTEND_CAP=..); the
// round kernels share PT_EXTEND_CAP.  Measured alternatives (4/24, 6/16,
// 4/32, 8/16, 8/12) were all slower on C3.  Scenes whose
// stack entries all fit 16 bits (dscene::stack16) run a u16 stack.
#ifndef PT_EXTEND_MINW
#define PT_EXTEND_MINW 5
#endif
#ifndef PT_EXTEND_CAP
#define PT_EXTEND_CAP 20
#endif

uint32_t pt_extend_stack_cap() { return PT_EXTEND_CAP; }

template <class Src, class E>
static void LaunchExtendE(const ptd::dscene& S, const Src& src, uint32_t n, uint32_t blocks, uint32_t* spill,
                          hipStream_t st)
{
    // The LDS node cache rides beside the u16 stack only (with the u32
    // stack's 20 KB it would cost occupancy).
    if constexpr (sizeof(E) == 2) {
        if (!spill && S.node_cache) {
            hipLaunchKernelGGL((ptd::extend_kernel<Src, false, PT_EXTEND_MINW, PT_EXTEND_CAP, E, true>), dim3(blocks),
                               dim3(256), 0, st, S, src, n, spill, n);
            return;
        }
    }
    if (spill)
        hipLaunchKernelGGL((ptd::extend_kernel<Src, true, PT_EXTEND_MINW, PT_EXTEND_CAP, E>), dim3(blocks), dim3(256),
                           0, st, S, src, n, spill, n);
    else
        hipLaunchKernelGGL((ptd::extend_kernel<Src, false, PT_EXTEND_MINW, PT_EXTEND_CAP, E>), dim3(blocks),
                           dim3(256), 0, st, S, src, n, spill, n);
}

// n: rays (the spill stride and the bound of the ray index); blocks: the
// launch's 256-ray blocks (the renderer's tiles).
template <class Src>
static hipError_t LaunchExtend(const ptd::dscene& S, const Src& src, uint32_t n, uint32_t blocks, uint32_t* spill,
                               hipStream_t st)
{
    if (n == 0 || blocks == 0) return hipSuccess;
    if (S.stack16) LaunchExtendE<Src, uint16_t>(S, src, n, blocks, spill, st);
    else LaunchExtendE<Src, uint32_t>(S, src, n, blocks, spill, st);
    return hipGetLastError();
}

template <class Src>
static hipError_t LaunchExtendStats(const ptd::dscene& S, const Src& src, uint32_t n, uint32_t* spill,
                                    unsigned long long* out, uint32_t* steps, hipStream_t st)
{
    // The same LDS stack capacity and entry width as the render kernel.
    if (S.stack16) {
        if (spill)
            hipLaunchKernelGGL((ptd::extend_stats_kernel<Src, true, PT_EXTEND_CAP, uint16_t>), dim3(Blocks(n)),
                               dim3(256), 0, st, S, src, n, spill, n, out, steps);
        else
            hipLaunchKernelGGL((ptd::extend_stats_kernel<Src, false, PT_EXTEND_CAP, uint16_t>), dim3(Blocks(n)),
                               dim3(256), 0, st, S, src, n, spill, n, out, steps);
    } else {
        if (spill)
            hipLaunchKernelGGL((ptd::extend_stats_kernel<Src, true, PT_EXTEND_CAP, uint32_t>), dim3(Blocks(n)),
                               dim3(256), 0, st, S, src, n, spill, n, out, steps);
        else
            hipLaunchKernelGGL((ptd::extend_stats_kernel<Src, false, PT_EXTEND_CAP, uint32_t>), dim3(Blocks(n)),
                               dim3(256), 0, st, S, src, n, spill, n, out, steps);
    }
    return hipGetLastError();
}

hipError_t pt_launch_trace_rays_stats(const ptd::dscene& S, uint32_t n, const float* origins, const uint32_t* vel,
                                      const float* dur, float4* hit, float2* hc, uint32_t* spill,
                                      unsigned long long* out, uint32_t* steps, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    return LaunchExtendStats(S, ptd::ray_source_arrays{origins, vel, dur, hit, hc}, n, spill, out, steps, st);
}

hipError_t pt_launch_extend_stats(const ptd::dscene& S, const ptd::dslots& L, const ptd::dframe& F, uint32_t* spill,
                                  unsigned long long* out, uint32_t* steps, hipStream_t st)
{
    if (L.n == 0) return hipSuccess;
    return LaunchExtendStats(S, ptd::ray_source_slots{L, F}, L.n, spill, out, steps, st);
}

hipError_t pt_launch_vertex_decode(const uint2* v, uint32_t n, float4* attr, float* vv, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(ptd::vertex_decode_kernel, dim3((n + 255) / 256), dim3(256), 0, st, v, n, attr, vv);
    return hipGetLastError();
}

hipError_t pt_launch_guard(const uint32_t* done, uint32_t words, uint64_t target, uint32_t* flags, hipStream_t st)
{
    hipLaunchKernelGGL(ptd::guard_kernel, dim3(1), dim3(1024), 0, st, done, words, (unsigned long long)target, flags);
    return hipGetLastError();
}

hipError_t pt_launch_tile_order(const ptd::dslots& L, hipStream_t st, uint32_t groups, uint32_t group)
{
    if (!L.order || L.tile_count == 0 || groups == 0 || group >= groups) return hipSuccess;
    hipLaunchKernelGGL(ptd::tile_order_kernel, dim3(1), dim3(1024), 0, st, L.tilecost, L.order, L.tile_count, groups,
                       group, pt_tile_group_start(L.tile_count, groups, group));
    return hipGetLastError();
}

hipError_t pt_launch_atlas_tile(const float4* src, float4* dst, uint32_t w, uint32_t h, uint32_t layers, hipStream_t st)
{
    uint64_t texels = (uint64_t)w * h * layers;
    if (texels == 0) return hipSuccess;
    uint64_t blocks = (texels + 255) / 256;
    hipLaunchKernelGGL(ptd::atlas_tile_kernel, dim3((uint32_t)(blocks < 65536 ? blocks : 65536)), dim3(256), 0, st, src,
                       dst, w, h, texels);
    return hipGetLastError();
}

hipError_t pt_launch_merge_streams(float4* accum, float4* accx, uint32_t width, uint32_t height, uint32_t rank,
                                   uint32_t nranks, uint32_t streams, hipStream_t st)
{
    if (streams <= 1 || width == 0 || height == 0) return hipSuccess;
    hipLaunchKernelGGL(ptd::merge_streams_kernel, dim3(Blocks(width), height < 32768u ? height : 32768u), dim3(256), 0,
                       st, accum, accx, width, height, rank, nranks, streams);
    return hipGetLastError();
}

hipError_t pt_launch_restore_rays(const ptd::dslots& L, const ptd::dframe& F, const float4* rays, uint32_t tile0,
                                  uint32_t tiles, hipStream_t st)
{
    if (tiles == 0) return hipSuccess;
    hipLaunchKernelGGL(ptd::restore_rays_kernel, dim3(tiles), dim3(256), 0, st, L, F, rays, tile0);
    return hipGetLastError();
}

hipError_t pt_launch_grey_check(const ptd::dslots& L, const ptd::dframe& F, uint32_t* count, hipStream_t st)
{
    if (L.n == 0) return hipSuccess;
    hipLaunchKernelGGL(ptd::grey_check_kernel, dim3(Blocks(L.n)), dim3(256), 0, st, L, F, count);
    return hipGetLastError();
}

hipError_t pt_launch_grey_convert(const ptd::dslots& L, const ptd::dframe& F, float* prob1, bool to_grey,
                                  hipStream_t st)
{
    if (L.n == 0) return hipSuccess;
    hipLaunchKernelGGL(ptd::grey_convert_kernel, dim3(Blocks(L.n)), dim3(256), 0, st, L, F, prob1, to_grey);
    return hipGetLastError();
}

hipError_t pt_launch_zero_unowned(float4* accum, uint32_t width, uint32_t height, uint32_t rank, uint32_t nranks,
                                  hipStream_t st)
{
    if (nranks <= 1 || width == 0 || height == 0) return hipSuccess;
    hipLaunchKernelGGL(ptd::zero_unowned_kernel, dim3(Blocks(width), height < 32768u ? height : 32768u), dim3(256), 0, st, accum, width, height,
                       rank, nranks);
    return hipGetLastError();
}

hipError_t pt_launch_extend(const ptd::dscene& S, const ptd::dslots& L, const ptd::dframe& F, uint32_t* spill,
                            hipStream_t st)
{
    return LaunchExtend(S, ptd::ray_source_slots{L, F}, L.n, L.tile_count, spill, st);
}

// Fused rounds (round_kernel): the default extend variant's LDS stack
// without spill, one instantiation per shade material mask and stack entry
// width.  Capacity = the tiles the GPU holds at once (blocks per CU at the
// kernel's occupancy x CUs); a larger partition runs extend + shade.
template <uint32_t MATS, class E>
static const void* RoundKernel() { return reinterpret_cast<const void*>(&ptd::round_kernel<MATS, PT_EXTEND_CAP, E>); }

static const void* RoundKernelFor(uint32_t mats, bool stack16)
{
    constexpr uint32_t D = PT_MATS_DIFFUSE, DS = PT_MATS_DIFFUSE | PT_MATS_SCENE,
                       DM = PT_MATS_DIFFUSE | PT_MATS_METAL | PT_MATS_SCENE, A = PT_MATS_ALL | PT_MATS_SCENE,
                       AO = PT_MATS_ALL | PT_MATS_OPENPBR | PT_MATS_SCENE;
    switch (pt_shade_mats(mats)) {
    case D: return stack16 ? RoundKernel<D, uint16_t>() : RoundKernel<D, uint32_t>();
    case DS: return stack16 ? RoundKernel<DS, uint16_t>() : RoundKernel<DS, uint32_t>();
    case DM: return stack16 ? RoundKernel<DM, uint16_t>() : RoundKernel<DM, uint32_t>();
    case A: return stack16 ? RoundKernel<A, uint16_t>() : RoundKernel<A, uint32_t>();
    default: return stack16 ? RoundKernel<AO, uint16_t>() : RoundKernel<AO, uint32_t>();
    }
}

uint32_t pt_round_capacity(uint32_t scene_mats, bool stack16, uint32_t cu_count)
{
    // Blocks per CU of the round kernel instantiation, cached per (device,
    // shade mask, stack entry width); renderers may be created from several
    // host threads and on several devices.
    static std::mutex mu;
    static std::map<std::tuple<int, uint32_t, bool>, int> per_cu;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    uint32_t m = pt_shade_mats(scene_mats);
    std::lock_guard<std::mutex> lock(mu);
    auto key = std::make_tuple(dev, m, stack16);
    auto it = per_cu.find(key);
    if (it == per_cu.end()) {
        int c = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&c, RoundKernelFor(scene_mats, stack16), 256, 0) != hipSuccess)
            c = 0;
        it = per_cu.emplace(key, c).first;
    }
    return (uint32_t)it->second * cu_count;
}

hipError_t pt_launch_round(const ptd::dscene& S, const ptd::dslots& L, const ptd::dframe& F, const ptd::dparams& P,
                           uint32_t scene_mats, hipStream_t st)
{
    if (L.n == 0 || L.tile_count == 0) return hipSuccess;
    if (L.spill) return hipErrorNotSupported;
    const void* k = RoundKernelFor(scene_mats, S.stack16 != 0);
    void* args[] = {const_cast<ptd::dscene*>(&S), const_cast<ptd::dslots*>(&L), const_cast<ptd::dframe*>(&F),
                    const_cast<ptd::dparams*>(&P)};
    return hipLaunchKernel(k, dim3(L.tile_count), dim3(256), args, 0, st);
}

template <uint32_t MATS, class E>
static const void* RoundsKernel() { return reinterpret_cast<const void*>(&ptd::rounds_kernel<MATS, PT_EXTEND_CAP, E>); }

static const void* RoundsKernelFor(uint32_t mats, bool stack16)
{
    constexpr uint32_t D = PT_MATS_DIFFUSE, DS = PT_MATS_DIFFUSE | PT_MATS_SCENE,
                       DM = PT_MATS_DIFFUSE | PT_MATS_METAL | PT_MATS_SCENE, A = PT_MATS_ALL | PT_MATS_SCENE,
                       AO = PT_MATS_ALL | PT_MATS_OPENPBR | PT_MATS_SCENE;
    switch (pt_shade_mats(mats)) {
    case D: return stack16 ? RoundsKernel<D, uint16_t>() : RoundsKernel<D, uint32_t>();
    case DS: return stack16 ? RoundsKernel<DS, uint16_t>() : RoundsKernel<DS, uint32_t>();
    case DM: return stack16 ? RoundsKernel<DM, uint16_t>() : RoundsKernel<DM, uint32_t>();
    case A: return stack16 ? RoundsKernel<A, uint16_t>() : RoundsKernel<A, uint32_t>();
    default: return stack16 ? RoundsKernel<AO, uint16_t>() : RoundsKernel<AO, uint32_t>();
    }
}

// Round batches need the round kernel's condition: no spilled stack.
bool pt_rounds_available(const ptd::dslots& L)
{
    return !L.spill;
}

hipError_t pt_launch_rounds(const ptd::dscene& S, const ptd::dslots& L, const ptd::dframe& F, const ptd::dparams& P,
                            uint32_t scene_mats, hipStream_t st)
{
    if (L.n == 0 || L.tile_count == 0 || P.rounds == 0) return hipSuccess;
    if (!pt_rounds_available(L)) return hipErrorNotSupported;
    const void* k = RoundsKernelFor(scene_mats, S.stack16 != 0);
    void* args[] = {const_cast<ptd::dscene*>(&S), const_cast<ptd::dslots*>(&L), const_cast<ptd::dframe*>(&F),
                    const_cast<ptd::dparams*>(&P)};
    return hipLaunchKernel(k, dim3(L.tile_count), dim3(256), args, 0, st);
}

// Shade instantiations by material-type mask: the smallest superset of the
// scene's mask is launched.
uint32_t pt_shade_mats(uint32_t scene_mats)
{
    // Diffuse meshes without sky light sampling whose textures lie in the
    // unit square of the atlas (the Viking Room, C3): the lean instantiation,
    // which has no sky lobe and no analytic shapes and wraps texel
    // coordinates with two selects (pt_device.hpp Texel).
    if ((scene_mats & ~(uint32_t)PT_MATS_DIFFUSE) == 0) return PT_MATS_DIFFUSE;
    scene_mats = (scene_mats & ~(uint32_t)PT_MATS_TEXWRAP) | PT_MATS_SCENE;
    if ((scene_mats & ~(uint32_t)(PT_MATS_DIFFUSE | PT_MATS_SCENE)) == 0) return PT_MATS_DIFFUSE | PT_MATS_SCENE;
    if ((scene_mats & ~(uint32_t)(PT_MATS_DIFFUSE | PT_MATS_METAL | PT_MATS_SCENE)) == 0)
        return PT_MATS_DIFFUSE | PT_MATS_METAL | PT_MATS_SCENE;
    if (!(scene_mats & PT_MATS_OPENPBR)) return PT_MATS_ALL | PT_MATS_SCENE;
    return PT_MATS_ALL | PT_MATS_OPENPBR | PT_MATS_SCENE;
}

template <bool COMPACT>
static void LaunchShade(const ptd::dscene& S, const ptd::dslots& L, const ptd::dframe& F, const ptd::dparams& P,
                        uint32_t scene_mats, hipStream_t st)
{
    const uint32_t blocks = L.tile_count;
    switch (pt_shade_mats(scene_mats)) {
    case PT_MATS_DIFFUSE:
        hipLaunchKernelGGL((ptd::shade_kernel<PT_MATS_DIFFUSE, COMPACT>), dim3(blocks), dim3(256), 0, st, S, L, F, P);
        break;
    case PT_MATS_DIFFUSE | PT_MATS_SCENE:
        hipLaunchKernelGGL((ptd::shade_kernel<PT_MATS_DIFFUSE | PT_MATS_SCENE, COMPACT>), dim3(blocks), dim3(256), 0, st,
                           S, L, F, P);
        break;
    case PT_MATS_DIFFUSE | PT_MATS_METAL | PT_MATS_SCENE:
        hipLaunchKernelGGL((ptd::shade_kernel<PT_MATS_DIFFUSE | PT_MATS_METAL | PT_MATS_SCENE, COMPACT>), dim3(blocks),
                           dim3(256), 0, st, S, L, F, P);
        break;
    case PT_MATS_ALL | PT_MATS_SCENE:
        hipLaunchKernelGGL((ptd::shade_kernel<PT_MATS_ALL | PT_MATS_SCENE, COMPACT>), dim3(blocks), dim3(256), 0, st, S,
                           L, F, P);
        break;
    default:
        hipLaunchKernelGGL((ptd::shade_kernel<PT_MATS_ALL | PT_MATS_OPENPBR | PT_MATS_SCENE, COMPACT>), dim3(blocks),
                           dim3(256), 0, st, S, L, F, P);
        break;
    }
}

hipError_t pt_launch_shade(const ptd::dscene& S, const ptd::dslots& L, const ptd::dframe& F, const ptd::dparams& P,
                           uint32_t scene_mats, bool compact, hipStream_t st)
{
    if (L.n == 0 || L.tile_count == 0) return hipSuccess;
    if (compact) LaunchShade<true>(S, L, F, P, scene_mats, st);
    else LaunchShade<false>(S, L, F, P, scene_mats, st);
    return hipGetLastError();
}

template <bool COMPACT>
static void LaunchShadeQ(const ptd::dscene& S, const ptd::dslots& L, const ptd::dframe& F, const ptd::dparams& P,
                         uint32_t scene_mats, const uint32_t* counts, const uint32_t* list, hipStream_t st)
{
    // The shade instantiations of LaunchShade for scenes with more than one
    // material type (pt_class_lists_supported); blocks past the lists return.
    const uint32_t blocks = L.tile_count + ptd::PT_OUTCOME_CLASSES;
    const uint32_t capk = pt_classq_sub_capacity(L.tile_count);
    if (pt_shade_mats(scene_mats) == (PT_MATS_DIFFUSE | PT_MATS_METAL | PT_MATS_SCENE))
        hipLaunchKernelGGL((ptd::shade_classq_kernel<PT_MATS_DIFFUSE | PT_MATS_METAL | PT_MATS_SCENE, COMPACT>),
                           dim3(blocks), dim3(256), 0, st, S, L, F, P, counts, list, capk);
    else
        hipLaunchKernelGGL((ptd::shade_classq_kernel<PT_MATS_ALL | PT_MATS_SCENE, COMPACT>), dim3(blocks), dim3(256), 0,
                           st, S, L, F, P, counts, list, capk);
}

bool pt_class_lists_supported(uint32_t scene_mats)
{
    const uint32_t m = pt_shade_mats(scene_mats);
    return m == (PT_MATS_DIFFUSE | PT_MATS_METAL | PT_MATS_SCENE) || m == (PT_MATS_ALL | PT_MATS_SCENE);
}

hipError_t pt_launch_shade_classq(const ptd::dscene& S, const ptd::dslots& L, const ptd::dframe& F,
                                  const ptd::dparams& P, uint32_t scene_mats, bool compact, uint32_t* counts,
                                  uint32_t* next_counts, uint32_t* list, hipStream_t st, uint32_t tiles_all,
                                  uint32_t groups, uint32_t group)
{
    if (L.n == 0 || L.tile_count == 0) return hipSuccess;
    if (!pt_class_lists_supported(scene_mats)) return hipErrorNotSupported;
    hipLaunchKernelGGL(ptd::class_list_kernel, dim3((L.tile_count + ptd::CQ_TILES - 1) / ptd::CQ_TILES), dim3(256), 0,
                       st, L, S.mat_classes, counts, next_counts, list, pt_classq_sub_capacity(L.tile_count),
                       tiles_all ? tiles_all : L.tile_count, groups, group);
    if (compact) LaunchShadeQ<true>(S, L, F, P, scene_mats, counts, list, st);
    else LaunchShadeQ<false>(S, L, F, P, scene_mats, counts, list, st);
    return hipGetLastError();
}

#if PT_SHADE_STATS
// Experiment build only (tools/shade_stats.py): the launch-summed shade
// branch counters {waves, lanes} x SM_COUNT; reset clears them.
extern "C" int ptShadeStatsRead(unsigned long long* out, int reset)
{
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(ptd::g_shade_stats), sizeof(ptd::g_shade_stats)) != hipSuccess)
        return -1;
    if (reset) {
        unsigned long long z[2 * 32] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(ptd::g_shade_stats), z, sizeof(z)) != hipSuccess) return -1;
    }
    return (int)ptd::SM_COUNT;
}
#endif

hipError_t pt_launch_rcp_check(unsigned long long* mismatches, hipStream_t st)
{
    hipLaunchKernelGGL(ptd::rcp_check_kernel, dim3(8192), dim3(256), 0, st, mismatches);
    return hipGetLastError();
}

hipError_t pt_launch_xdiv_check(uint64_t n, uint32_t seed, unsigned long long* mismatches, hipStream_t st)
{
    hipLaunchKernelGGL(ptd::xdiv_check_kernel, dim3(4096), dim3(256), 0, st, n, seed, mismatches);
    return hipGetLastError();
}

hipError_t pt_launch_trace_rays(const ptd::dscene& S, uint32_t n, const float* origins, const uint32_t* vel,
                                const float* dur, float4* hit, float2* hc, float4* rec, float2* uv, uint32_t* spill,
                                hipStream_t st)
{
    hipError_t e = LaunchExtend(S, ptd::ray_source_arrays{origins, vel, dur, hit, hc}, n, Blocks(n), spill, st);
    if (e != hipSuccess) return e;
    return pt_launch_finalize(S, n, hit, hc, rec, uv, st);
}

hipError_t pt_launch_finalize(const ptd::dscene& S, uint32_t n, const float4* hit, const float2* hc, float4* rec,
                              float2* uv, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(ptd::finalize_kernel, dim3(Blocks(n)), dim3(256), 0, st, S, n, hit, hc, rec, uv);
    return hipGetLastError();
}
