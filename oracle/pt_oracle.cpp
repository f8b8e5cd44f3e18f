// pt_oracle.cpp — CPU oracle (TEST INFRASTRUCTURE; see pt_oracle.h).
//
// Each function below restates the reference GLSL function named in its
// comment, statement by statement, with the GLSL built-ins mapped to
// include/pt_glsl.h.  The per-pixel integrator state is kept in the same
// packed form the reference keeps in its SoA buffers (octahedral snorm16
// velocity / normal / tangent, 16-bit active-shape stack), because that
// quantisation is part of the algorithm's observable behaviour.
#include "pt_oracle.h"
#include "../include/pt_cie.h"
#include "../include/pt_glsl.h"

#include <atomic>
#include <cstring>
#include <thread>
#include <cstdlib>
#include <vector>

namespace {

// --- constants ---------------------------------------------------------------
const uint32_t SHAPE_INDEX_NONE = 0xFFFFFFFFu;       // scene.glsl.inc:7
const uint32_t TEXTURE_INDEX_NONE = 0xFFFFFFFFu;     // scene.glsl.inc:8
const int ACTIVE_SHAPE_LIMIT = 4;                    // basic.glsl.inc:11

struct ray { pt3 Origin; pt3 Velocity; float Duration; };            // common.glsl.inc:23-28
struct medium { uint32_t Priority; pt4 IOR, AbsorptionRate, ScatteringRate; float ScatteringAnisotropy; };
struct hit {                                                          // scene.glsl.inc:102-119
    float Time; uint32_t ShapeIndex; pt3 Position, Normal, TangentX; uint32_t MaterialIndex; pt2 UV;
    pt3 TangentY; uint32_t ShapeType; pt3 PrimitiveCoordinates; uint32_t PrimitiveIndex;
    uint32_t SceneComplexity, MeshComplexity;
};
struct path {                                                         // basic.glsl.inc:13-21
    float NormalizedLambda0; pt4 Throughput, Probability; pt3 Sample; int ImageX, ImageY;
    uint32_t ActiveShapeIndex[4];
};
struct bsdf_parameters { uint32_t MaterialIndex; pt2 TextureUV; pt4 Lambda; pt4 ExteriorIOR; };

// Deep copy of the scene packs.
struct scene_data {
    pt_packed_scene_globals Scene{};
    std::vector<pt_packed_texture> Textures;
    std::vector<uint32_t> MaterialData;
    std::vector<pt_packed_shape> Shapes;
    std::vector<pt_packed_shape_node> ShapeNodes;
    std::vector<pt_packed_mesh_face> MeshFaces;
    std::vector<pt_packed_mesh_vertex> MeshVertices;
    std::vector<pt_packed_mesh_node> MeshNodes;
    std::vector<pt_packed_camera> Cameras;
    std::vector<float> Atlas;
    uint32_t AtlasW = 0, AtlasH = 0, AtlasLayers = 0;

    explicit scene_data(const pt_scene_packs* p)
    {
        if (p->globals) Scene = *p->globals;
        Textures.assign(p->textures, p->textures + p->texture_count);
        MaterialData.assign(p->material_data, p->material_data + p->material_word_count);
        Shapes.assign(p->shapes, p->shapes + p->shape_count);
        ShapeNodes.assign(p->shape_nodes, p->shape_nodes + p->shape_node_count);
        MeshFaces.assign(p->mesh_faces, p->mesh_faces + p->mesh_face_count);
        MeshVertices.assign(p->mesh_vertices, p->mesh_vertices + p->mesh_vertex_count);
        MeshNodes.assign(p->mesh_nodes, p->mesh_nodes + p->mesh_node_count);
        Cameras.assign(p->cameras, p->cameras + p->camera_count);
        AtlasW = p->atlas_width; AtlasH = p->atlas_height; AtlasLayers = p->atlas_layer_count;
        if (p->atlas) Atlas.assign(p->atlas, p->atlas + (size_t)AtlasW * AtlasH * 4 * AtlasLayers);
    }
};

pt3 f3(const float* p) { return v3(p[0], p[1], p[2]); }

// --- common.glsl.inc ---------------------------------------------------------

pt3 TransformPosition(pt3 P, const pt_packed_transform& T) { return mat4_mul_point(T.To, P); }       // :40-43
pt3 TransformVector(pt3 V, const pt_packed_transform& T) { return mat4_mul_vector(T.To, V); }        // :45-48
pt3 TransformNormal(pt3 N, const pt_packed_transform& T) { return normalize(vec_mul_mat4(N, T.From)); } // :50-53
pt3 TransformDirection(pt3 D, const pt_packed_transform& T) { return normalize(TransformVector(D, T)); } // :55-58
ray TransformRay(ray R, const pt_packed_transform& T)                                                // :60-67
{
    ray O; O.Origin = TransformPosition(R.Origin, T); O.Velocity = TransformVector(R.Velocity, T); O.Duration = R.Duration;
    return O;
}
ray InverseTransformRay(ray R, const pt_packed_transform& T)                                         // :84-91
{
    ray O; O.Origin = mat4_mul_point(T.From, R.Origin); O.Velocity = mat4_mul_vector(T.From, R.Velocity);
    O.Duration = R.Duration;
    return O;
}

pt3 SafeNormalize(pt3 V)                                                                             // :93-100
{
    float LenSq = dot(V, V);
    if (LenSq < 1e-12f) return v3(0, 0, 1);
    return V / pt_sqrt(LenSq);
}

pt3 ComputeTangentVector(pt3 Normal)                                                                 // :113-117
{
    pt3 V = pt_abs(Normal.x) < 0.9f ? v3(1, 0, 0) : v3(0, 1, 0);
    return normalize(cross(V, Normal));
}

void ComputeCoordinateFrame(pt3 Z, pt3& X, pt3& Y)                                                   // :120-125
{
    pt3 V = pt_abs(Z.x) < 0.9f ? v3(1, 0, 0) : v3(0, 1, 0);
    X = normalize(cross(V, Z));
    Y = cross(X, Z);
}

pt2 SignNotZero(pt2 V) { return v2(V.x >= 0.0f ? 1.0f : -1.0f, V.y >= 0.0f ? 1.0f : -1.0f); }       // :127-134

uint32_t PackUnitVector(pt3 V)                                                                       // :137-142
{
    pt2 P = v2(V.x, V.y) * (1.0f / (pt_abs(V.x) + pt_abs(V.y) + pt_abs(V.z)));
    if (V.z <= 0.0f) P = v2(1.0f - pt_abs(P.y), 1.0f - pt_abs(P.x)) * SignNotZero(P);
    return pt_pack_snorm16(P.x) | (pt_pack_snorm16(P.y) << 16);
}

pt3 UnpackUnitVector(uint32_t PackedV)                                                               // :145-151
{
    pt2 P = v2(pt_unpack_snorm16(PackedV & 0xFFFFu), pt_unpack_snorm16(PackedV >> 16));
    float Z = 1.0f - pt_abs(P.x) - pt_abs(P.y);
    if (Z < 0.0f) P = v2(1.0f - pt_abs(P.y), 1.0f - pt_abs(P.x)) * SignNotZero(P);
    return normalize(v3(P.x, P.y, Z));
}

// Slab-test division convention (process-wide; oracle_set_slab_division).
// 1 (default, the HIP kernels' convention and SURVEY.md §7/§8(c)'s):
// correctly rounded IEEE (Min - Ray.Origin) / Ray.Velocity.  0: the
// reciprocal form RN((Min - Ray.Origin) * RN(1 / Ray.Velocity)) GPU compilers
// emit for GLSL's 2.5-ULP `/`; kept to measure what that form changes
// (tools/slab_convention.py, tests/test_slab_convention.py).
std::atomic<int> SlabDivisionIEEE{1};

float IntersectBoundingBox(const ray& Ray, float Reach, pt3 Min, pt3 Max)                            // :153-185
{
    pt3 MinT, MaxT;
    if (SlabDivisionIEEE.load(std::memory_order_relaxed)) {
        MinT = (Min - Ray.Origin) / Ray.Velocity;                                                    // :157-158
        MaxT = (Max - Ray.Origin) / Ray.Velocity;
    } else {
        pt3 InverseVelocity = v3(1.0f / Ray.Velocity.x, 1.0f / Ray.Velocity.y, 1.0f / Ray.Velocity.z);
        MinT = (Min - Ray.Origin) * InverseVelocity;
        MaxT = (Max - Ray.Origin) * InverseVelocity;
    }
    pt3 EarlierT = vmin(MinT, MaxT);
    pt3 LaterT = vmax(MinT, MaxT);
    float EntryT = pt_max(pt_max(EarlierT.x, EarlierT.y), EarlierT.z);
    float ExitT = pt_min(pt_min(LaterT.x, LaterT.y), LaterT.z);
    if (ExitT < EntryT) return PT_INFINITY;
    if (ExitT <= 0) return PT_INFINITY;
    if (EntryT >= Reach) return PT_INFINITY;
    return EntryT;
}

struct rng {                                                                                         // :189-203
    uint32_t State;
    float R01() { return pt_random01(&State); }
};

pt2 RandomPointOnDisk(rng& G)                                                                        // :205-210
{
    float R = pt_sqrt(G.R01());
    float Theta = G.R01() * PT_TAU;
    return R * v2(pt_cos(Theta), pt_sin(Theta));
}

pt3 RandomDirection(rng& G)                                                                          // :212-218
{
    float Z = 2 * G.R01() - 1;
    float R = pt_sqrt(1 - Z * Z);
    float Phi = PT_TAU * G.R01();
    return v3(R * pt_cos(Phi), R * pt_sin(Phi), Z);
}

pt3 RandomVonMisesFisher(rng& G, float Kappa)                                                        // :228-239
{
    float Xi = G.R01();
    float Z = 1 + (1 / Kappa) * pt_log(Xi + (1 - Xi) * pt_exp(-2 * Kappa));
    float R = pt_sqrt(1 - Z * Z);
    float Phi = G.R01() * PT_TAU;
    return v3(R * pt_cos(Phi), R * pt_sin(Phi), Z);
}

pt3 RandomVonMisesFisher(rng& G, float Kappa, pt3 Mu)                                                // :241-247
{
    pt3 V = RandomVonMisesFisher(G, Kappa);
    pt3 MuX, MuY;
    ComputeCoordinateFrame(Mu, MuX, MuY);
    return SafeNormalize(V.x * MuX + V.y * MuY + V.z * Mu);
}

float VonMisesFisherPDF(float Kappa, pt3 Mu, pt3 Direction)                                          // :249-254
{
    if (Kappa < PT_EPSILON) return 1.0f / (4 * PT_PI);
    float C = Kappa / (2 * PT_PI * (1 - pt_exp(-2 * Kappa)));
    return C * pt_exp(Kappa * (dot(Mu, Direction) - 1.0f));
}

pt3 SampleDirectionHG(float Anisotropy, float U1, float U2)                                          // :259-276
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

pt2 GGXRoughnessAlpha(float Roughness, float Anisotropy)                                             // :281-288
{
    float R = Roughness;
    float S = 1 - Anisotropy;
    float AlphaX = R * R * pt_sqrt(2 / (1 + S * S));
    float AlphaY = S * AlphaX;
    return v2(AlphaX, AlphaY);
}

float GGXSmithG1(pt3 Direction, pt2 RoughnessAlpha)                                                  // :294-301
{
    pt3 DirectionSq = Direction * Direction;
    if (DirectionSq.z < PT_EPSILON) return 0.0f;
    pt2 RoughnessAlphaSq = RoughnessAlpha * RoughnessAlpha;
    float AlphaSqByTanThetaSq = dot(RoughnessAlphaSq, v2(DirectionSq.x, DirectionSq.y)) / DirectionSq.z;
    return 2.0f / (1.0f + pt_sqrt(1.0f + AlphaSqByTanThetaSq));
}

pt3 GGXVisibleNormal(pt3 Direction, pt2 RoughnessAlpha, float U1, float U2)                          // :306-346
{
    pt3 Vz = SafeNormalize(v3(RoughnessAlpha.x * Direction.x, RoughnessAlpha.y * Direction.y, Direction.z));
    float LengthSq = dot(v2(Vz.x, Vz.y), v2(Vz.x, Vz.y));
    pt3 Vx = LengthSq > 0 ? v3(-Vz.y, Vz.x, 0) / pt_sqrt(LengthSq) : v3(1, 0, 0);
    pt3 Vy = cross(Vz, Vx);
    float R = pt_sqrt(U1);
    float Phi = PT_TAU * U2;
    float S = 0.5f * (1.0f + Vz.z);
    float Tx = R * pt_cos(Phi);
    float Ty = (1.0f - S) * pt_sqrt(1.0f - Tx * Tx) + S * R * pt_sin(Phi);
    float Tz = pt_sqrt(pt_max(0.0f, 1.0f - Tx * Tx - Ty * Ty));
    pt3 Normal = Tx * Vx + Ty * Vy + Tz * Vz;
    return SafeNormalize(v3(RoughnessAlpha.x * Normal.x, RoughnessAlpha.y * Normal.y, pt_max(0.0f, Normal.z)));
}

float GGXDistribution(pt3 Normal, pt2 RoughnessAlpha)                                                // :349-354
{
    pt2 A = v2(1.0f / RoughnessAlpha.x, 1.0f / RoughnessAlpha.y);
    float B = dot(Normal * Normal, v3(A.x * A.x, A.y * A.y, 1.0f));
    return 1.0f / (PT_PI * RoughnessAlpha.x * RoughnessAlpha.y * B * B);
}

pt4 CauchyEmpiricalIOR(float BaseIOR, float AbbeNumber, pt4 Lambda)                                  // :360-371
{
    const float LC = 656.3f, Ld = 587.6f, LF = 486.1f;
    float B = (BaseIOR - 1) / (AbbeNumber * (1.0f / (LF * LF) - 1.0f / (LC * LC)));
    float A = BaseIOR - B / (Ld * Ld);
    return A + B / (Lambda * Lambda);
}

float ComputeCosThetaRefracted(float Eta, float CosTheta)                                            // :379-383
{
    float Cos2ThetaRefracted = 1 - Eta * Eta * (1 - CosTheta * CosTheta);
    return -pt_sign(CosTheta) * pt_sqrt(pt_max(Cos2ThetaRefracted, 0.0f));
}

pt4 ComputeCosThetaRefracted(pt4 Eta, pt4 CosTheta)                                                  // :386-390
{
    pt4 C2 = 1 - Eta * Eta * (1 - CosTheta * CosTheta);
    return -vsign(CosTheta) * vsqrt(vmax(C2, 0.0f));
}

float FresnelDielectric(float Eta, float CosTheta1, float CosTheta2)                                 // :396-403
{
    float Ks = Eta * CosTheta1;
    float SqrtRs = (Ks + CosTheta2) / (Ks - CosTheta2);
    float Kp = Eta * CosTheta2;
    float SqrtRp = (Kp + CosTheta1) / (Kp - CosTheta1);
    return 0.5f * (SqrtRs * SqrtRs + SqrtRp * SqrtRp);
}

pt4 FresnelDielectric(pt4 Eta, pt4 CosTheta1, pt4 CosTheta2)                                         // :406-413
{
    pt4 Ks = Eta * CosTheta1;
    pt4 SqrtRs = (Ks + CosTheta2) / (Ks - CosTheta2);
    pt4 Kp = Eta * CosTheta2;
    pt4 SqrtRp = (Kp + CosTheta1) / (Kp - CosTheta1);
    return 0.5f * (SqrtRs * SqrtRs + SqrtRp * SqrtRp);
}

pt4 FresnelDielectric(pt4 Eta, pt4 CosTheta1)                                                        // :416-420
{
    pt4 CosTheta2 = ComputeCosThetaRefracted(Eta, CosTheta1);
    return FresnelDielectric(Eta, CosTheta1, CosTheta2);
}

// pow(x, 5) and pow(x, 6) for the constant exponents used below.
float Pow5(float x) { float x2 = x * x; return (x2 * x2) * x; }
float Pow6(float x) { float x2 = x * x; return (x2 * x2) * x2; }

pt4 SchlickFresnelMetal(pt4 Base, pt4 Specular, float CosTheta)                                      // :425-436
{
    const float CosThetaMax = 1 / 7.0f;
    pt4 FSchlick = Base + (1 - Base) * Pow5(1.0f - CosTheta);
    pt4 FSchlickMax = Base + (1 - Base) * Pow5(1 - CosThetaMax);
    pt4 FMax = Specular * FSchlickMax;
    const float Denominator = CosThetaMax * Pow6(1 - CosThetaMax);
    float Nominator = CosTheta * Pow6(1.0f - CosTheta);
    return FSchlick - (Nominator / Denominator) * (FSchlickMax - FMax);
}

// --- spectrum.glsl.inc -------------------------------------------------------

pt3 SampleStandardObserver(float Lambda)                                                             // :10-34
{
    pt3 Result;
    {
        float T1 = (Lambda - 442.0f) * (Lambda < 442.0f ? 0.0624f : 0.0374f);
        float T2 = (Lambda - 599.8f) * (Lambda < 599.8f ? 0.0264f : 0.0323f);
        float T3 = (Lambda - 501.1f) * (Lambda < 501.1f ? 0.0490f : 0.0382f);
        Result.x = 0.362f * pt_exp(-0.5f * T1 * T1) + 1.056f * pt_exp(-0.5f * T2 * T2) - 0.065f * pt_exp(-0.5f * T3 * T3);
    }
    {
        float T1 = (Lambda - 568.8f) * (Lambda < 568.8f ? 0.0213f : 0.0247f);
        float T2 = (Lambda - 530.9f) * (Lambda < 530.9f ? 0.0613f : 0.0322f);
        Result.y = 0.821f * pt_exp(-0.5f * T1 * T1) + 0.286f * pt_exp(-0.5f * T2 * T2);
    }
    {
        float T1 = (Lambda - 437.0f) * (Lambda < 437.0f ? 0.0845f : 0.0278f);
        float T2 = (Lambda - 459.0f) * (Lambda < 459.0f ? 0.0385f : 0.0725f);
        Result.z = 1.217f * pt_exp(-0.5f * T1 * T1) + 0.681f * pt_exp(-0.5f * T2 * T2);
    }
    return Result;
}

float SampleParametricSpectrum(pt3 Beta, float Lambda)                                               // :169-173
{
    float X = (Beta.x * Lambda + Beta.y) * Lambda + Beta.z;
    return 0.5f + X / (2.0f * pt_sqrt(1.0f + X * X));
}

pt4 SampleParametricSpectrum(pt3 Beta, pt4 L)                                                        // :176-180
{
    return v4(SampleParametricSpectrum(Beta, L.x), SampleParametricSpectrum(Beta, L.y),
              SampleParametricSpectrum(Beta, L.z), SampleParametricSpectrum(Beta, L.w));
}

pt4 SampleParametricSpectrum(pt4 BetaAndIntensity, pt4 L)                                            // :189-192
{
    return BetaAndIntensity.w * SampleParametricSpectrum(v3(BetaAndIntensity.x, BetaAndIntensity.y, BetaAndIntensity.z), L);
}

// --- the integrator context ----------------------------------------------------

struct context {
    const scene_data& S;
    rng G;

    explicit context(const scene_data& s) : S(s) { G.State = 0; }

    // scene.glsl.inc:181-205; textureLod(level 0) with the REPEAT samplers of
    // src/core/vulkan.cpp:1669-1716, filtered in software (Vulkan formula).
    pt4 Texel(uint32_t Layer, int X, int Y) const
    {
        int W = (int)S.AtlasW, H = (int)S.AtlasH;
        X %= W; if (X < 0) X += W;
        Y %= H; if (Y < 0) Y += H;
        if (Layer >= S.AtlasLayers) Layer = S.AtlasLayers ? S.AtlasLayers - 1 : 0;
        if (S.AtlasLayers == 0) return v4s(0);
        const float* T = &S.Atlas[(((size_t)Layer * H + Y) * W + X) * 4];
        return v4(T[0], T[1], T[2], T[3]);
    }

    pt4 SampleTexture(uint32_t Index, pt2 UV) const
    {
        const pt_packed_texture& T = S.Textures[Index];
        float U = pt_mix(T.AtlasPlacementMinimum[0], T.AtlasPlacementMaximum[0], pt_fract(UV.x));
        float V = pt_mix(T.AtlasPlacementMinimum[1], T.AtlasPlacementMaximum[1], pt_fract(UV.y));
        float W = (float)S.AtlasW, H = (float)S.AtlasH;
        if (T.Flags & PT_TEXTURE_FLAG_FILTER_NEAREST) {
            return Texel(T.AtlasImageIndex, (int)pt_floor(U * W), (int)pt_floor(V * H));
        }
        float Us = U * W - 0.5f, Vs = V * H - 0.5f;
        float Fi = pt_floor(Us), Fj = pt_floor(Vs);
        float A = Us - Fi, B = Vs - Fj;
        int I0 = (int)Fi, J0 = (int)Fj;
        pt4 T00 = Texel(T.AtlasImageIndex, I0, J0), T10 = Texel(T.AtlasImageIndex, I0 + 1, J0);
        pt4 T01 = Texel(T.AtlasImageIndex, I0, J0 + 1), T11 = Texel(T.AtlasImageIndex, I0 + 1, J0 + 1);
        return ((1 - A) * (1 - B)) * T00 + (A * (1 - B)) * T10 + ((1 - A) * B) * T01 + (A * B) * T11;
    }

    pt4 SampleSkyboxSpectrum(pt3 Direction) const                                                     // :209-221
    {
        if (S.Scene.SkyboxTextureIndex == TEXTURE_INDEX_NONE) return v4(0, 0, 100, 1);
        float Phi = pt_atan2(Direction.y, Direction.x);
        float Theta = pt_asin(Direction.z);
        float U = 0.5f + Phi / PT_TAU;
        float V = 0.5f + Theta / PT_PI;
        return SampleTexture(S.Scene.SkyboxTextureIndex, v2(U, V));
    }

    pt4 SampleSkyboxRadiance(pt3 Direction, pt4 Lambda) const                                         // :225-229
    {
        pt4 Spectrum = SampleSkyboxSpectrum(Direction);
        return SampleParametricSpectrum(Spectrum, Lambda) * S.Scene.SkyboxBrightness;
    }

    uint32_t MaterialType(uint32_t M) const { return S.MaterialData[32 * M]; }                      // :231-234
    uint32_t MaterialUint(uint32_t M, uint32_t A) const { return S.MaterialData[32 * M + A]; }       // :236-239
    float MaterialFloat(uint32_t M, uint32_t A) const { return pt_u2f(MaterialUint(M, A)); }         // :241-244
    pt3 MaterialVec3(uint32_t M, uint32_t A) const                                                   // :246-252
    {
        return v3(MaterialFloat(M, A + 0), MaterialFloat(M, A + 1), MaterialFloat(M, A + 2));
    }

    pt4 MaterialTexturableReflectance(uint32_t M, uint32_t A, pt4 Lambda, pt2 UV) const              // :276-290
    {
        pt3 Beta = MaterialVec3(M, A + 0);
        pt4 Value = SampleParametricSpectrum(Beta, Lambda);
        uint32_t TextureIndex = MaterialUint(M, A + 3);
        if (TextureIndex != TEXTURE_INDEX_NONE) {
            pt4 Tx = SampleTexture(TextureIndex, UV);
            Value = Value * SampleParametricSpectrum(v3(Tx.x, Tx.y, Tx.z), Lambda);
        }
        return Value;
    }

    float MaterialTexturableValue(uint32_t M, uint32_t A, pt2 UV) const                              // :292-302
    {
        float Value = MaterialFloat(M, A + 0);
        uint32_t TextureIndex = MaterialUint(M, A + 1);
        if (TextureIndex != TEXTURE_INDEX_NONE) Value *= SampleTexture(TextureIndex, UV).x;
        return Value;
    }

    // --- traversal ------------------------------------------------------------

    void IntersectMeshFace(const ray& Ray, uint32_t MeshFaceIndex, hit& Hit) const                   // :304-334
    {
        const pt_packed_mesh_face& Face = S.MeshFaces[MeshFaceIndex];
        pt3 P0 = f3(Face.Position0), P1 = f3(Face.Position1), P2 = f3(Face.Position2);
        pt3 Edge1 = P1 - P0;
        pt3 Edge2 = P2 - P0;
        pt3 RayCrossEdge2 = cross(Ray.Velocity, Edge2);
        float Det = dot(Edge1, RayCrossEdge2);
        if (pt_abs(Det) < PT_EPSILON) return;
        float InvDet = 1.0f / Det;
        pt3 Sv = Ray.Origin - P0;
        float U = InvDet * dot(Sv, RayCrossEdge2);
        if (U < 0 || U > 1) return;
        pt3 SCrossEdge1 = cross(Sv, Edge1);
        float V = InvDet * dot(Ray.Velocity, SCrossEdge1);
        if (V < 0 || U + V > 1) return;
        float T = InvDet * dot(Edge2, SCrossEdge1);
        if (T < 0 || T > Hit.Time) return;
        Hit.Time = T;
        Hit.ShapeType = PT_SHAPE_TYPE_MESH_INSTANCE;
        Hit.ShapeIndex = 0xFFFFFFFEu;
        Hit.PrimitiveIndex = MeshFaceIndex;
        Hit.PrimitiveCoordinates = v3(1 - U - V, U, V);
    }

    // Stack[32] as in the reference; a push beyond 32 entries (UB there) is dropped.
    void IntersectMeshNode(const ray& Ray, uint32_t MeshNodeIndex, hit& Hit) const                   // :336-399
    {
        uint32_t Stack[32];
        uint32_t Depth = 0;
        auto Push = [&](uint32_t v) { if (Depth < 32) Stack[Depth++] = v; };
        pt_packed_mesh_node Node = S.MeshNodes[MeshNodeIndex];
        while (true) {
            Hit.MeshComplexity++;
            if (Node.FaceEndIndex > 0) {
                for (uint32_t FaceIndex = Node.FaceBeginOrNodeIndex; FaceIndex < Node.FaceEndIndex; FaceIndex++)
                    IntersectMeshFace(Ray, FaceIndex, Hit);
            } else {
                uint32_t Index = Node.FaceBeginOrNodeIndex;
                Node = S.MeshNodes[Index];
                float Time = IntersectBoundingBox(Ray, Hit.Time, f3(Node.Minimum), f3(Node.Maximum));
                uint32_t IndexB = Index + 1;
                pt_packed_mesh_node NodeB = S.MeshNodes[IndexB];
                float TimeB = IntersectBoundingBox(Ray, Hit.Time, f3(NodeB.Minimum), f3(NodeB.Maximum));
                if (Time > TimeB) {
                    if (Time < PT_INFINITY) Push(Index);
                    Node = NodeB;
                    continue;
                }
                if (TimeB < PT_INFINITY) { Push(IndexB); continue; }
                if (Time < PT_INFINITY) continue;
            }
            if (Depth == 0) break;
            Node = S.MeshNodes[Stack[--Depth]];
        }
    }

    void IntersectShape(ray Ray, uint32_t ShapeIndex, hit& Hit) const                                // :401-466
    {
        const pt_packed_shape& Shape = S.Shapes[ShapeIndex];
        Ray = InverseTransformRay(Ray, Shape.Transform);
        if (Shape.Type == PT_SHAPE_TYPE_MESH_INSTANCE) {
            IntersectMeshNode(Ray, Shape.MeshRootNodeIndex, Hit);
            if (Hit.ShapeIndex == 0xFFFFFFFEu) Hit.ShapeIndex = ShapeIndex;
        } else if (Shape.Type == PT_SHAPE_TYPE_PLANE) {
            float T = -Ray.Origin.z / Ray.Velocity.z;
            if (T < 0 || T > Hit.Time) return;
            Hit.Time = T;
            Hit.ShapeType = PT_SHAPE_TYPE_PLANE;
            Hit.ShapeIndex = ShapeIndex;
            Hit.PrimitiveIndex = 0;
            Hit.PrimitiveCoordinates = Ray.Origin + Ray.Velocity * T;
        } else if (Shape.Type == PT_SHAPE_TYPE_SPHERE) {
            float V = dot(Ray.Velocity, Ray.Velocity);
            float P = dot(Ray.Origin, Ray.Velocity);
            float Q = dot(Ray.Origin, Ray.Origin) - 1.0f;
            float D2 = P * P - Q * V;
            if (D2 < 0) return;
            float D = pt_sqrt(D2);
            if (D < P) return;
            float S0 = -P - D;
            float S1 = -P + D;
            float Sv = S0 < 0 ? S1 : S0;
            if (Sv < 0 || Sv > V * Hit.Time) return;
            Hit.Time = Sv / V;
            Hit.ShapeType = PT_SHAPE_TYPE_SPHERE;
            Hit.ShapeIndex = ShapeIndex;
            Hit.PrimitiveIndex = 0;
            Hit.PrimitiveCoordinates = Ray.Origin + Ray.Velocity * Hit.Time;
        } else if (Shape.Type == PT_SHAPE_TYPE_CUBE) {
            pt3 Minimum = (v3s(-1) - Ray.Origin) / Ray.Velocity;
            pt3 Maximum = (v3s(+1) - Ray.Origin) / Ray.Velocity;
            pt3 Earlier = vmin(Minimum, Maximum);
            pt3 Later = vmax(Minimum, Maximum);
            float T0 = pt_max(pt_max(Earlier.x, Earlier.y), Earlier.z);
            float T1 = pt_min(pt_min(Later.x, Later.y), Later.z);
            if (T1 < T0) return;
            if (T1 <= 0) return;
            float T = T0 < 0 ? T1 : T0;
            if (T >= Hit.Time) return;
            Hit.Time = T;
            Hit.ShapeType = PT_SHAPE_TYPE_CUBE;
            Hit.ShapeIndex = ShapeIndex;
            Hit.PrimitiveIndex = 0;
            Hit.PrimitiveCoordinates = Ray.Origin + Ray.Velocity * T;
        }
    }

    void Intersect(const ray& Ray, hit& Hit) const                                                   // :468-520
    {
        if (S.Scene.ShapeCount == 0) return;
        uint32_t Stack[32];
        uint32_t Depth = 0;
        auto Push = [&](uint32_t v) { if (Depth < 32) Stack[Depth++] = v; };
        pt_packed_shape_node NodeA = S.ShapeNodes[0];
        pt_packed_shape_node NodeB;
        while (true) {
            Hit.SceneComplexity++;
            if (NodeA.ChildNodeIndices == 0) {
                IntersectShape(Ray, NodeA.ShapeIndex, Hit);
            } else {
                uint32_t IndexA = NodeA.ChildNodeIndices & 0xFFFF;
                uint32_t IndexB = NodeA.ChildNodeIndices >> 16;
                NodeA = S.ShapeNodes[IndexA];
                NodeB = S.ShapeNodes[IndexB];
                float TimeA = IntersectBoundingBox(Ray, Hit.Time, f3(NodeA.Minimum), f3(NodeA.Maximum));
                float TimeB = IntersectBoundingBox(Ray, Hit.Time, f3(NodeB.Minimum), f3(NodeB.Maximum));
                if (TimeA > TimeB) {
                    if (TimeA < PT_INFINITY) Push(IndexA);
                    NodeA = NodeB;
                    continue;
                }
                if (TimeB < PT_INFINITY) { Push(IndexB); continue; }
                if (TimeA < PT_INFINITY) continue;
            }
            if (Depth == 0) break;
            NodeA = S.ShapeNodes[Stack[--Depth]];
        }
    }

    hit Trace(const ray& Ray) const                                                                  // :522-611
    {
        hit Hit{};
        Hit.ShapeIndex = SHAPE_INDEX_NONE;
        Hit.Time = Ray.Duration;
        Hit.MeshComplexity = 0;
        Hit.SceneComplexity = 0;
        Intersect(Ray, Hit);
        if (Hit.ShapeIndex == SHAPE_INDEX_NONE) return Hit;
        const pt_packed_shape& Shape = S.Shapes[Hit.ShapeIndex];
        Hit.MaterialIndex = Shape.MaterialIndex;
        if (Hit.ShapeType == PT_SHAPE_TYPE_MESH_INSTANCE) {
            const pt_packed_mesh_face& Face = S.MeshFaces[Hit.PrimitiveIndex];
            const pt_packed_mesh_vertex& V0 = S.MeshVertices[Face.VertexIndex0];
            const pt_packed_mesh_vertex& V1 = S.MeshVertices[Face.VertexIndex1];
            const pt_packed_mesh_vertex& V2 = S.MeshVertices[Face.VertexIndex2];
            pt3 C = Hit.PrimitiveCoordinates;
            pt3 Normal = SafeNormalize(UnpackUnitVector(V0.PackedNormal) * C.x + UnpackUnitVector(V1.PackedNormal) * C.y +
                                       UnpackUnitVector(V2.PackedNormal) * C.z);
            Hit.Normal = TransformNormal(Normal, Shape.Transform);
            Hit.TangentX = ComputeTangentVector(Hit.Normal);
            pt2 UV0 = v2(pt_half_to_float(V0.PackedUV & 0xFFFF), pt_half_to_float(V0.PackedUV >> 16));
            pt2 UV1 = v2(pt_half_to_float(V1.PackedUV & 0xFFFF), pt_half_to_float(V1.PackedUV >> 16));
            pt2 UV2 = v2(pt_half_to_float(V2.PackedUV & 0xFFFF), pt_half_to_float(V2.PackedUV >> 16));
            Hit.UV = UV0 * C.x + UV1 * C.y + UV2 * C.z;
        } else if (Hit.ShapeType == PT_SHAPE_TYPE_PLANE) {
            Hit.Normal = TransformNormal(v3(0, 0, 1), Shape.Transform);
            Hit.TangentX = TransformDirection(v3(1, 0, 0), Shape.Transform);
            Hit.UV = v2(pt_fract(Hit.PrimitiveCoordinates.x), pt_fract(Hit.PrimitiveCoordinates.y));
        } else if (Hit.ShapeType == PT_SHAPE_TYPE_SPHERE) {
            pt3 P = Hit.PrimitiveCoordinates;
            float U = (pt_atan2(P.y, P.x) + PT_PI) / PT_TAU;
            float V = (P.z + 1.0f) / 2.0f;
            Hit.Normal = TransformNormal(P, Shape.Transform);
            Hit.TangentX = TransformDirection(cross(P, v3(-P.y, P.x, 0)), Shape.Transform);
            Hit.UV = v2(U, V);
        } else if (Hit.ShapeType == PT_SHAPE_TYPE_CUBE) {
            pt3 P = Hit.PrimitiveCoordinates;
            pt3 Q = vabs(P);
            pt3 Normal, TangentX;
            if (Q.x >= Q.y && Q.x >= Q.z) {
                float Sg = pt_sign(P.x);
                Normal = v3(Sg, 0, 0); TangentX = v3(0, Sg, 0);
                Hit.UV = 0.5f * (v2(1.0f + P.y, 1.0f + P.z));
            } else if (Q.y >= Q.x && Q.y >= Q.z) {
                float Sg = pt_sign(P.y);
                Normal = v3(0, Sg, 0); TangentX = v3(0, 0, Sg);
                Hit.UV = 0.5f * (v2(1.0f + P.x, 1.0f + P.z));
            } else {
                float Sg = pt_sign(P.z);
                Normal = v3(0, 0, Sg); TangentX = v3(Sg, 0, 0);
                Hit.UV = 0.5f * (v2(1.0f + P.x, 1.0f + P.y));
            }
            Hit.Normal = TransformNormal(Normal, Shape.Transform);
            Hit.TangentX = TransformDirection(TangentX, Shape.Transform);
        }
        return Hit;
    }

    ray GenerateCameraRay(const pt_packed_camera& Camera, pt2 NSP)                                   // :613-655
    {
        ray Ray{};
        Ray.Duration = PT_HIT_TIME_LIMIT;
        if (Camera.Model == PT_CAMERA_MODEL_PINHOLE) {
            pt3 SensorPosition = v3(-Camera.SensorSize[0] * (NSP.x - 0.5f), -Camera.SensorSize[1] * (0.5f - NSP.y),
                                    Camera.SensorDistance);
            pt2 D = Camera.ApertureRadius * RandomPointOnDisk(G);
            Ray.Origin = v3(D.x, D.y, 0);
            Ray.Velocity = normalize(Ray.Origin - SensorPosition);
        } else if (Camera.Model == PT_CAMERA_MODEL_THIN_LENS) {
            pt3 SensorPosition = v3(-Camera.SensorSize[0] * (NSP.x - 0.5f), -Camera.SensorSize[1] * (0.5f - NSP.y),
                                    Camera.SensorDistance);
            pt3 ObjectPosition = -SensorPosition * Camera.FocalLength / (SensorPosition.z - Camera.FocalLength);
            pt2 D = Camera.ApertureRadius * RandomPointOnDisk(G);
            Ray.Origin = v3(D.x, D.y, 0);
            Ray.Velocity = normalize(ObjectPosition - Ray.Origin);
        } else if (Camera.Model == PT_CAMERA_MODEL_360) {
            float Phi = (NSP.x - 0.5f) * PT_TAU;
            float Theta = (0.5f - NSP.y) * PT_PI;
            Ray.Origin = v3(0, 0, 0);
            Ray.Velocity = v3(pt_cos(Theta) * pt_sin(Phi), pt_sin(Theta), -pt_cos(Theta) * pt_cos(Phi));
        }
        return TransformRay(Ray, Camera.Transform);
    }

    // --- materials ----------------------------------------------------------------

    // basic_diffuse.glsl.inc:19-50
    bool BasicDiffuse_EvaluateBSDF(const bsdf_parameters& P, pt3 In, pt3 Out, pt4& Throughput, pt4& Probability)
    {
        (void)Out;
        pt4 Reflectance = MaterialTexturableReflectance(P.MaterialIndex, PT_BASIC_DIFFUSE_BASE_SPECTRUM, P.Lambda, P.TextureUV);
        Probability = v4s(In.z / PT_PI);
        Throughput = Probability * Reflectance;
        return true;
    }
    bool BasicDiffuse_SampleBSDF(const bsdf_parameters& P, pt3 In, pt3& Out, pt4& Throughput, pt4& Probability)
    {
        Out = SafeNormalize(RandomDirection(G) + v3(0, 0, 1));
        return BasicDiffuse_EvaluateBSDF(P, In, Out, Throughput, Probability);
    }

    // basic_metal.glsl.inc:6-26
    void BasicMetal_GetParameters(const bsdf_parameters& P, pt4& Base, pt4& Specular, pt2& Alpha, bool& Rough)
    {
        Base = MaterialTexturableReflectance(P.MaterialIndex, PT_BASIC_METAL_BASE_SPECTRUM, P.Lambda, P.TextureUV);
        Specular = MaterialTexturableReflectance(P.MaterialIndex, PT_BASIC_METAL_SPECULAR_SPECTRUM, P.Lambda, P.TextureUV);
        Alpha = GGXRoughnessAlpha(MaterialTexturableValue(P.MaterialIndex, PT_BASIC_METAL_ROUGHNESS, P.TextureUV),
                                  MaterialTexturableValue(P.MaterialIndex, PT_BASIC_METAL_ROUGHNESS_ANISOTROPY, P.TextureUV));
        Rough = Alpha.x * Alpha.y > PT_EPSILON;
    }
    bool BasicMetal_HasDiracBSDF(const bsdf_parameters& P)                                           // :38-41
    {
        return MaterialTexturableValue(P.MaterialIndex, PT_BASIC_METAL_ROUGHNESS, P.TextureUV) < 1e-3f;
    }
    bool BasicMetal_EvaluateBSDF(const bsdf_parameters& P, pt3 In, pt3 Out, pt4& Throughput, pt4& Probability) // :44-83
    {
        pt4 Base, Specular; pt2 Alpha; bool Rough;
        BasicMetal_GetParameters(P, Base, Specular, Alpha, Rough);
        if (In.z <= 0.0f || Out.z <= 0.0f || !Rough) return false;
        pt3 Half = SafeNormalize(In + Out);
        float Gm = GGXSmithG1(In, Alpha);
        float D = GGXDistribution(Half, Alpha);
        Probability = v4s(Gm * D / (4 * In.z));
        float Gs = GGXSmithG1(Out, Alpha);
        pt4 F = SchlickFresnelMetal(Base, Specular, dot(In, Half));
        Throughput = Probability * Gs * F;
        return true;
    }
    bool BasicMetal_SampleBSDF(const bsdf_parameters& P, pt3 In, pt3& Out, pt4& Throughput, pt4& Probability) // :86-141
    {
        pt4 Base, Specular; pt2 Alpha; bool Rough;
        BasicMetal_GetParameters(P, Base, Specular, Alpha, Rough);
        if (In.z <= 0.0f) return false;
        float NormalU1 = G.R01();
        float NormalU2 = G.R01();
        pt3 Normal = GGXVisibleNormal(In, Alpha, NormalU1, NormalU2);
        float CosThetaIn = pt_min(dot(Normal, In), 1.0f);
        Out = 2 * CosThetaIn * Normal - In;
        if (Out.z <= 0.0f) return false;
        Probability = v4s(1.0f);
        if (Rough) {
            float Gm = GGXSmithG1(In, Alpha);
            float D = GGXDistribution(Normal, Alpha);
            Probability = Probability * v4s(Gm * D / (4 * In.z));
        }
        float Gs = GGXSmithG1(Out, Alpha);
        pt4 F = SchlickFresnelMetal(Base, Specular, CosThetaIn);
        Throughput = Probability * Gs * F;
        return true;
    }

    // basic_translucent.glsl.inc:10-48
    void BasicTranslucent_GetParameters(const bsdf_parameters& P, pt3 In, pt4& RelativeIOR, pt2& Alpha, bool& Rough)
    {
        pt4 InteriorIOR = CauchyEmpiricalIOR(MaterialFloat(P.MaterialIndex, PT_BASIC_TRANSLUCENT_IOR),
                                             MaterialFloat(P.MaterialIndex, PT_BASIC_TRANSLUCENT_ABBE_NUMBER), P.Lambda);
        if (In.z < 0.0f) RelativeIOR = InteriorIOR / P.ExteriorIOR;
        else RelativeIOR = P.ExteriorIOR / InteriorIOR;
        Alpha = GGXRoughnessAlpha(MaterialTexturableValue(P.MaterialIndex, PT_BASIC_TRANSLUCENT_ROUGHNESS, P.TextureUV),
                                  MaterialTexturableValue(P.MaterialIndex, PT_BASIC_TRANSLUCENT_ROUGHNESS_ANISOTROPY, P.TextureUV));
        Rough = Alpha.x * Alpha.y > PT_EPSILON;
    }
    bool BasicTranslucent_LoadMedium(uint32_t M, pt4 Lambda, medium& Medium)                          // :55-82
    {
        Medium.IOR = CauchyEmpiricalIOR(MaterialFloat(M, PT_BASIC_TRANSLUCENT_IOR),
                                        MaterialFloat(M, PT_BASIC_TRANSLUCENT_ABBE_NUMBER), Lambda);
        float TransmissionDepth = MaterialFloat(M, PT_BASIC_TRANSLUCENT_TRANSMISSION_DEPTH);
        if (TransmissionDepth > 0.0f) {
            pt4 ExtinctionRate = -vlog(SampleParametricSpectrum(MaterialVec3(M, PT_BASIC_TRANSLUCENT_TRANSMISSION_SPECTRUM), Lambda)) / TransmissionDepth;
            pt4 ScatteringRate = SampleParametricSpectrum(MaterialVec3(M, PT_BASIC_TRANSLUCENT_SCATTERING_SPECTRUM), Lambda) / TransmissionDepth;
            Medium.AbsorptionRate = vmax(ExtinctionRate - ScatteringRate, 0.0f);
            Medium.ScatteringRate = ScatteringRate;
            Medium.ScatteringAnisotropy = MaterialFloat(M, PT_BASIC_TRANSLUCENT_SCATTERING_ANISOTROPY);
        } else {
            Medium.AbsorptionRate = v4s(0.0f);
            Medium.ScatteringRate = v4s(0.0f);
            Medium.ScatteringAnisotropy = 0.0f;
        }
        return true;
    }
    bool BasicTranslucent_HasDiracBSDF(const bsdf_parameters& P)                                     // :84-87
    {
        return MaterialTexturableValue(P.MaterialIndex, PT_BASIC_TRANSLUCENT_ROUGHNESS, P.TextureUV) < 1e-3f;
    }
    bool BasicTranslucent_EvaluateBSDF(const bsdf_parameters& P, pt3 In, pt3 Out, pt4& Throughput, pt4& Probability) // :90-169
    {
        pt4 RelativeIOR; pt2 Alpha; bool Rough;
        BasicTranslucent_GetParameters(P, In, RelativeIOR, Alpha, Rough);
        if (!Rough) { Probability = v4s(0.0f); Throughput = v4s(0.0f); return true; }
        float Gm = GGXSmithG1(In, Alpha);
        if (In.z * Out.z > 0) {
            pt3 Half = SafeNormalize(Out + In);
            float CosThetaIn = dot(Half, In);
            pt4 F = FresnelDielectric(RelativeIOR, v4s(CosThetaIn));
            float D = GGXDistribution(Half, Alpha);
            Probability = F * Gm * D / (4 * In.z);
        } else {
            pt3 Half1 = SafeNormalize(Out + In * RelativeIOR.x);
            pt3 Half2 = SafeNormalize(Out + In * RelativeIOR.y);
            pt3 Half3 = SafeNormalize(Out + In * RelativeIOR.z);
            pt3 Half4 = SafeNormalize(Out + In * RelativeIOR.w);
            pt4 CosThetaIn = v4(dot(In, Half1), dot(In, Half2), dot(In, Half3), dot(In, Half4));
            pt4 CosThetaOut = v4(dot(Out, Half1), dot(Out, Half2), dot(Out, Half3), dot(Out, Half4));
            pt4 F = FresnelDielectric(RelativeIOR, CosThetaIn, CosThetaOut);
            pt4 D = v4s(0.0f);
            if (CosThetaIn.x * CosThetaOut.x < 0.0f) D.x = GGXDistribution(Half1, Alpha);
            if (CosThetaIn.y * CosThetaOut.y < 0.0f) D.y = GGXDistribution(Half2, Alpha);
            if (CosThetaIn.z * CosThetaOut.z < 0.0f) D.z = GGXDistribution(Half3, Alpha);
            if (CosThetaIn.w * CosThetaOut.w < 0.0f) D.w = GGXDistribution(Half4, Alpha);
            pt4 Sq = CosThetaIn * RelativeIOR + CosThetaOut;
            pt4 J = vabs(CosThetaOut) / (Sq * Sq);
            Probability = D * (1 - F) * Gm * J * vabs(CosThetaIn / In.z);
        }
        float Gs = GGXSmithG1(Out, Alpha);
        Throughput = Probability * Gs;
        return true;
    }
    bool BasicTranslucent_SampleBSDF(const bsdf_parameters& P, pt3 In, pt3& Out, pt4& Throughput, pt4& Probability) // :172-339
    {
        pt4 RelativeIOR; pt2 Alpha; bool Rough;
        BasicTranslucent_GetParameters(P, In, RelativeIOR, Alpha, Rough);
        float NormalU1 = G.R01();
        float NormalU2 = G.R01();
        pt3 Normal = GGXVisibleNormal(In * pt_sign(In.z), Alpha, NormalU1, NormalU2);
        float CosThetaIn = pt_clamp(dot(Normal, In), -1.0f, +1.0f);
        float CosThetaRefracted = ComputeCosThetaRefracted(RelativeIOR.x, CosThetaIn);
        float Reflectance = FresnelDielectric(RelativeIOR.x, CosThetaIn, CosThetaRefracted);
        if (G.R01() < Reflectance) {
            Out = 2 * CosThetaIn * Normal - In;
            if (Out.z * In.z <= 0) return false;
            pt4 F = FresnelDielectric(RelativeIOR, v4s(CosThetaIn));
            Probability = F;
            if (Rough) {
                float Gm = GGXSmithG1(In, Alpha);
                float D = GGXDistribution(Normal, Alpha);
                Probability = Probability * (Gm * D / (4 * pt_abs(In.z)));
            }
            float Gs = GGXSmithG1(Out, Alpha);
            Throughput = Probability * Gs;
            return true;
        }
        Out = (CosThetaRefracted + RelativeIOR.x * CosThetaIn) * Normal - RelativeIOR.x * In;
        if (Out.z * In.z >= 0) return false;
        if (Rough) {
            pt3 Normal2 = SafeNormalize(Out + In * RelativeIOR.y);
            pt3 Normal3 = SafeNormalize(Out + In * RelativeIOR.z);
            pt3 Normal4 = SafeNormalize(Out + In * RelativeIOR.w);
            pt4 CosThetaIn4 = v4(CosThetaIn, dot(In, Normal2), dot(In, Normal3), dot(In, Normal4));
            pt4 CosThetaOut4 = v4(CosThetaRefracted, dot(Out, Normal2), dot(Out, Normal3), dot(Out, Normal4));
            pt4 F = FresnelDielectric(RelativeIOR, CosThetaIn4, CosThetaOut4);
            pt4 D = v4s(0.0f);
            D.x = GGXDistribution(Normal, Alpha);
            if (CosThetaIn4.y * CosThetaOut4.y < 0.0f) D.y = GGXDistribution(Normal2, Alpha);
            if (CosThetaIn4.z * CosThetaOut4.z < 0.0f) D.z = GGXDistribution(Normal3, Alpha);
            if (CosThetaIn4.w * CosThetaOut4.w < 0.0f) D.w = GGXDistribution(Normal4, Alpha);
            float Gm = GGXSmithG1(In, Alpha);
            pt4 Sq = CosThetaIn4 * RelativeIOR + CosThetaOut4;
            pt4 J = vabs(CosThetaOut4) / (Sq * Sq);
            Probability = D * (1 - F) * Gm * J * vabs(CosThetaIn4 / In.z);
        } else {
            Probability = v4(1 - Reflectance, 0, 0, 0);
        }
        float Gs = GGXSmithG1(Out, Alpha);
        Throughput = Probability * Gs;
        return true;
    }

    // --- openpbr.glsl.inc (opt-in: the reference never compiles it) ---------------

    struct openpbr_parameters {                                                                     // :30-47
        uint32_t LayerBounceLimit;
        bool BaseIsMetal, BaseIsTranslucent, CoatIsPresent;
        pt4 BaseReflectance;
        float BaseDiffuseRoughness;
        pt4 CoatRelativeIOR, CoatTransmittance;
        pt2 CoatRoughnessAlpha;
        float SpecularWeight;
        pt4 SpecularRelativeIOR, SpecularReflectance;
        pt2 SpecularRoughnessAlpha;
        // Emission (:46, :142-152) is never read by OpenPBR_Sample: omitted.
    };

    openpbr_parameters OpenPBR_Parameters(uint32_t MI, pt2 TextureUV, pt4 Lambda, pt4 ExteriorIOR)  // :66-158
    {
        openpbr_parameters Parameters;
        Parameters.CoatIsPresent = G.R01() < MaterialFloat(MI, PT_OPENPBR_COAT_WEIGHT);
        Parameters.BaseIsMetal = G.R01() < MaterialFloat(MI, PT_OPENPBR_BASE_METALNESS);
        Parameters.BaseIsTranslucent =
            !Parameters.BaseIsMetal && G.R01() < MaterialFloat(MI, PT_OPENPBR_TRANSMISSION_WEIGHT);
        Parameters.BaseReflectance = MaterialFloat(MI, PT_OPENPBR_BASE_WEIGHT) *
                                     SampleParametricSpectrum(MaterialVec3(MI, PT_OPENPBR_BASE_SPECTRUM), Lambda);
        Parameters.BaseDiffuseRoughness = MaterialFloat(MI, PT_OPENPBR_BASE_DIFFUSE_ROUGHNESS);
        uint32_t BaseSpectrumTextureIndex = MaterialUint(MI, PT_OPENPBR_BASE_SPECTRUM_TEXTURE_INDEX);
        if (BaseSpectrumTextureIndex != TEXTURE_INDEX_NONE) {
            pt4 Value = SampleTexture(BaseSpectrumTextureIndex, TextureUV);
            Parameters.BaseReflectance =
                Parameters.BaseReflectance * SampleParametricSpectrum(v3(Value.x, Value.y, Value.z), Lambda);
        }
        // (unused without a coat; set so that the struct is fully defined)
        Parameters.CoatRelativeIOR = v4s(1.0f);
        Parameters.CoatTransmittance = v4s(1.0f);
        Parameters.CoatRoughnessAlpha = v2(0.0f, 0.0f);
        if (Parameters.CoatIsPresent) {
            Parameters.CoatRelativeIOR = ExteriorIOR / MaterialFloat(MI, PT_OPENPBR_COAT_IOR);
            Parameters.CoatTransmittance = SampleParametricSpectrum(MaterialVec3(MI, PT_OPENPBR_COAT_COLOR_SPECTRUM), Lambda);
            Parameters.CoatRoughnessAlpha = GGXRoughnessAlpha(MaterialFloat(MI, PT_OPENPBR_COAT_ROUGHNESS),
                                                              MaterialFloat(MI, PT_OPENPBR_COAT_ROUGHNESS_ANISOTROPY));
        }
        Parameters.SpecularWeight = MaterialFloat(MI, PT_OPENPBR_SPECULAR_WEIGHT);
        Parameters.SpecularReflectance = SampleParametricSpectrum(MaterialVec3(MI, PT_OPENPBR_SPECULAR_SPECTRUM), Lambda);
        pt4 SpecularIOR = CauchyEmpiricalIOR(MaterialFloat(MI, PT_OPENPBR_SPECULAR_IOR),
                                             MaterialFloat(MI, PT_OPENPBR_TRANSMISSION_DISPERSION_ABBE_NUMBER), Lambda);
        if (Parameters.CoatIsPresent)
            Parameters.SpecularRelativeIOR = MaterialFloat(MI, PT_OPENPBR_COAT_IOR) / SpecularIOR;
        else
            Parameters.SpecularRelativeIOR = ExteriorIOR / SpecularIOR;
        float SpecularRoughness = MaterialFloat(MI, PT_OPENPBR_SPECULAR_ROUGHNESS);
        uint32_t SpecularRoughnessTextureIndex = MaterialUint(MI, PT_OPENPBR_SPECULAR_ROUGHNESS_TEXTURE_INDEX);
        if (SpecularRoughnessTextureIndex != TEXTURE_INDEX_NONE) {
            pt4 Value = SampleTexture(SpecularRoughnessTextureIndex, TextureUV);
            SpecularRoughness *= Value.x;
        }
        Parameters.SpecularRoughnessAlpha =
            GGXRoughnessAlpha(SpecularRoughness, MaterialFloat(MI, PT_OPENPBR_SPECULAR_ROUGHNESS_ANISOTROPY));
        Parameters.LayerBounceLimit = MaterialUint(MI, PT_OPENPBR_LAYER_BOUNCE_LIMIT);
        return Parameters;
    }

    void OpenPBR_Medium(uint32_t MI, pt4 Lambda, medium& Medium)                                    // :160-191
    {
        Medium.IOR = CauchyEmpiricalIOR(MaterialFloat(MI, PT_OPENPBR_SPECULAR_IOR),
                                        MaterialFloat(MI, PT_OPENPBR_TRANSMISSION_DISPERSION_ABBE_NUMBER), Lambda);
        float TransmissionDepth = MaterialFloat(MI, PT_OPENPBR_TRANSMISSION_DEPTH);
        if (TransmissionDepth > 0.0f) {
            pt4 ExtinctionRate =
                -vlog(SampleParametricSpectrum(MaterialVec3(MI, PT_OPENPBR_TRANSMISSION_SPECTRUM), Lambda)) / TransmissionDepth;
            pt4 ScatteringRate =
                SampleParametricSpectrum(MaterialVec3(MI, PT_OPENPBR_TRANSMISSION_SCATTER_SPECTRUM), Lambda) / TransmissionDepth;
            Medium.AbsorptionRate = vmax(ExtinctionRate - ScatteringRate, 0.0f);
            Medium.ScatteringRate = ScatteringRate;
            Medium.ScatteringAnisotropy = MaterialFloat(MI, PT_OPENPBR_TRANSMISSION_SCATTER_ANISOTROPY);
        } else {
            Medium.AbsorptionRate = v4s(0.0f);
            Medium.ScatteringRate = v4s(0.0f);
            Medium.ScatteringAnisotropy = 0.0f;
        }
    }

    void OpenPBR_CoatSample(const openpbr_parameters& Parameters, pt3 Out, pt3& In, pt4& PathThroughput,  // :194-283
                            pt4& PathDensity)
    {
        if (!Parameters.CoatIsPresent) { In = -Out; return; }
        float NormalU1 = G.R01();
        float NormalU2 = G.R01();
        pt3 Normal = GGXVisibleNormal(Out * pt_sign(Out.z), Parameters.CoatRoughnessAlpha, NormalU1, NormalU2);
        float Cosine = dot(Normal, Out);
        pt4 RelativeIOR = Parameters.CoatRelativeIOR;
        if (Out.z < 0) RelativeIOR = 1.0f / RelativeIOR;
        float RefractedCosineSquared = 1 - RelativeIOR.x * RelativeIOR.x * (1 - Cosine * Cosine);
        float RefractedCosine = -pt_sign(Out.z) * pt_sqrt(pt_max(RefractedCosineSquared, 0.0f));
        // :227 passes (RefractedCosine, Cosine, RelativeIOR.x) to
        // FresnelDielectric(Eta, CosTheta1, CosTheta2); restated in signature
        // order, as the base layer calls it (:346).
        float Reflectance = FresnelDielectric(RelativeIOR.x, Cosine, RefractedCosine);
        if (G.R01() < Reflectance) {
            In = 2 * Cosine * Normal - Out;
            if (In.z * Out.z <= 0) { PathDensity = v4s(0.0f); return; }
            PathThroughput = PathThroughput * GGXSmithG1(In, Parameters.CoatRoughnessAlpha);
            if (Out.z < 0) {
                float Exponent = -(0.5f / Out.z + 0.5f / In.z);
                PathThroughput = PathThroughput * vpow(Parameters.CoatTransmittance, Exponent);
            }
        } else {
            In = (RelativeIOR.x * Cosine + RefractedCosine) * Normal - RelativeIOR.x * Out;
            if (In.z * Out.z > 0) { PathDensity = v4s(0.0f); return; }
            PathThroughput = PathThroughput * GGXSmithG1(In, Parameters.CoatRoughnessAlpha);
            if (Out.z < 0)
                PathThroughput = PathThroughput * vpow(Parameters.CoatTransmittance, -0.5f / Out.z);
            else
                PathThroughput = PathThroughput * vpow(Parameters.CoatTransmittance, -0.5f / In.z);
        }
    }

    void OpenPBR_BaseSpecularSample(const openpbr_parameters& Parameters, pt3 Out, pt3& In,           // :286-435
                                    pt4& PathThroughput, pt4& PathDensity)
    {
        float NormalU1 = G.R01();
        float NormalU2 = G.R01();
        pt3 Normal = GGXVisibleNormal(Out * pt_sign(Out.z), Parameters.SpecularRoughnessAlpha, NormalU1, NormalU2);
        float Cosine = dot(Normal, Out);
        if (Parameters.BaseIsMetal) {
            In = 2 * Cosine * Normal - Out;
            if (Out.z * In.z <= 0) { PathDensity = v4s(0.0f); return; }
            float Shadowing = GGXSmithG1(Out, Parameters.SpecularRoughnessAlpha);
            pt4 Fresnel = Parameters.SpecularWeight *
                          SchlickFresnelMetal(Parameters.BaseReflectance, Parameters.SpecularReflectance, pt_abs(Cosine));
            PathThroughput = PathThroughput * (Fresnel * Shadowing);
        } else {
            pt4 RelativeIOR = Parameters.SpecularRelativeIOR;
            if (Out.z < 0) RelativeIOR = 1.0f / RelativeIOR;
            if (Parameters.SpecularWeight < 1.0f) {
                pt4 R = pt_sqrt(Parameters.SpecularWeight) * (1.0f - RelativeIOR) / (1.0f + RelativeIOR);
                RelativeIOR = (1.0f - R) / (1.0f + R);
            }
            float RefractedCosine = ComputeCosThetaRefracted(RelativeIOR.x, Cosine);
            float Reflectance = FresnelDielectric(RelativeIOR.x, Cosine, RefractedCosine);
            if (G.R01() < Reflectance) {
                In = 2 * Cosine * Normal - Out;
                if (In.z * Out.z <= 0) { PathDensity = v4s(0.0f); return; }
                if (Out.z > 0) PathThroughput = PathThroughput * Parameters.SpecularReflectance;
                PathThroughput = PathThroughput * GGXSmithG1(In, Parameters.SpecularRoughnessAlpha);
            } else {
                In = (RelativeIOR.x * Cosine + RefractedCosine) * Normal - RelativeIOR.x * Out;
                if (In.z * Out.z > 0) { PathDensity = v4s(0.0f); return; }
                float Shadowing = GGXSmithG1(In, Parameters.SpecularRoughnessAlpha);
                if (length(Parameters.SpecularRoughnessAlpha) > PT_EPSILON) {
                    pt4 Fresnel = v4s(0.0f);   // :390-391 "TODO: This is broken for now!"
                    pt3 Normal2 = SafeNormalize(In + Out * RelativeIOR.y);
                    pt3 Normal3 = SafeNormalize(In + Out * RelativeIOR.z);
                    pt3 Normal4 = SafeNormalize(In + Out * RelativeIOR.w);
                    pt4 Density = v4s(0.0f);
                    Density.x = GGXDistribution(Normal, Parameters.SpecularRoughnessAlpha);
                    if (dot(In, Normal2) * dot(Out, Normal2) < 0.0f)
                        Density.y = GGXDistribution(Normal2, Parameters.SpecularRoughnessAlpha);
                    if (dot(In, Normal3) * dot(Out, Normal3) < 0.0f)
                        Density.z = GGXDistribution(Normal3, Parameters.SpecularRoughnessAlpha);
                    if (dot(In, Normal4) * dot(Out, Normal4) < 0.0f)
                        Density.w = GGXDistribution(Normal4, Parameters.SpecularRoughnessAlpha);
                    Density = Density / pt_max(PT_EPSILON, max4(Density));
                    PathThroughput = PathThroughput * (Density * Fresnel * Shadowing);
                    PathDensity = PathDensity * (Density * Fresnel);
                } else {
                    PathThroughput = PathThroughput * v4(Shadowing, 0, 0, 0);
                    PathDensity = PathDensity * v4(1, 0, 0, 0);
                }
            }
        }
    }

    void OpenPBR_BaseDiffuseSample(const openpbr_parameters& Parameters, pt3 Out, pt3& In,            // :438-461
                                   pt4& PathThroughput)
    {
        if (Parameters.BaseIsTranslucent) { In = -Out; return; }
        In = SafeNormalize(RandomDirection(G) + v3(0, 0, 1));
        float S_ = dot(In, Out) - In.z * Out.z;
        float T_ = S_ > 0 ? pt_max(In.z, Out.z) : 1.0f;
        float SigmaSq = Parameters.BaseDiffuseRoughness * Parameters.BaseDiffuseRoughness;
        pt4 A = (1 - 0.5f * SigmaSq / (SigmaSq + 0.33f)) + 0.17f * Parameters.BaseReflectance * SigmaSq / (SigmaSq + 0.13f);
        float B = 0.45f * SigmaSq / (SigmaSq + 0.09f);
        PathThroughput = PathThroughput * (Parameters.BaseReflectance * (B * S_ / T_ + A));
    }

    bool OpenPBR_Sample(const openpbr_parameters& Parameters, pt3 Out, pt3& In, pt4& Throughput,       // :463-515
                        pt4& InPDF)
    {
        const int LAYER_EXTERNAL = -1, LAYER_COAT = 0, LAYER_BASE_SPECULAR = 1, LAYER_BASE_DIFFUSE = 2;
        int Layer;
        if (Out.z > 0) Layer = Parameters.CoatIsPresent ? LAYER_COAT : LAYER_BASE_SPECULAR;
        else Layer = LAYER_BASE_SPECULAR;
        Throughput = v4s(1.0f);
        InPDF = v4s(1.0f);
        In = -Out;   // the reference leaves In unassigned when LayerBounceLimit is 0
        for (uint32_t I = 0; I < Parameters.LayerBounceLimit; I++) {
            if (Layer == LAYER_COAT) {
                OpenPBR_CoatSample(Parameters, Out, In, Throughput, InPDF);
                Layer = In.z < 0 ? LAYER_BASE_SPECULAR : LAYER_EXTERNAL;
            } else if (Layer == LAYER_BASE_SPECULAR) {
                OpenPBR_BaseSpecularSample(Parameters, Out, In, Throughput, InPDF);
                Layer = In.z < 0 ? LAYER_BASE_DIFFUSE : LAYER_COAT;
            } else if (Layer == LAYER_BASE_DIFFUSE) {
                OpenPBR_BaseDiffuseSample(Parameters, Out, In, Throughput);
                Layer = In.z < 0 ? LAYER_EXTERNAL : LAYER_BASE_SPECULAR;
            } else if (Layer == LAYER_EXTERNAL) {
                break;
            }
            if (max4(InPDF) < PT_EPSILON) return false;
            Out = -In;
        }
        return true;
    }

    // Dispatch (scene.glsl.inc:687-762).  OpenPBR / unknown types are not
    // compiled into the reference kernels: Sample/Evaluate return false,
    // HasDirac false; LoadMedium leaves the medium as the vacuum (the
    // reference's `out` parameter is undefined there).  With OpenPBR shading
    // enabled (the renderer's opt-in), OpenPBR is a sampling-only BSDF:
    // HasDirac true (no skybox light sampling), SampleBSDF = OpenPBR_Parameters
    // + OpenPBR_Sample, LoadMedium = OpenPBR_Medium.
    bool OpenPBR = false;

    bool MaterialLoadMedium(uint32_t M, pt4 Lambda, medium& Medium)
    {
        Medium.IOR = v4s(1.0f); Medium.AbsorptionRate = v4s(0.0f); Medium.ScatteringRate = v4s(0.0f);
        Medium.ScatteringAnisotropy = 0.0f;
        uint32_t Type = MaterialType(M);
        if (Type == PT_MATERIAL_TYPE_BASIC_TRANSLUCENT) return BasicTranslucent_LoadMedium(M, Lambda, Medium);
        if (Type == PT_MATERIAL_TYPE_OPENPBR && OpenPBR) { OpenPBR_Medium(M, Lambda, Medium); return true; }
        return false;
    }
    bool MaterialHasDiracBSDF(const bsdf_parameters& P)
    {
        uint32_t Type = MaterialType(P.MaterialIndex);
        if (Type == PT_MATERIAL_TYPE_BASIC_DIFFUSE) return false;
        if (Type == PT_MATERIAL_TYPE_BASIC_METAL) return BasicMetal_HasDiracBSDF(P);
        if (Type == PT_MATERIAL_TYPE_BASIC_TRANSLUCENT) return BasicTranslucent_HasDiracBSDF(P);
        if (Type == PT_MATERIAL_TYPE_OPENPBR) return OpenPBR;
        return false;
    }
    bool MaterialEvaluateBSDF(const bsdf_parameters& P, pt3 In, pt3 Out, pt4& T, pt4& Pr)
    {
        uint32_t Type = MaterialType(P.MaterialIndex);
        if (Type == PT_MATERIAL_TYPE_BASIC_DIFFUSE) return BasicDiffuse_EvaluateBSDF(P, In, Out, T, Pr);
        if (Type == PT_MATERIAL_TYPE_BASIC_METAL) return BasicMetal_EvaluateBSDF(P, In, Out, T, Pr);
        if (Type == PT_MATERIAL_TYPE_BASIC_TRANSLUCENT) return BasicTranslucent_EvaluateBSDF(P, In, Out, T, Pr);
        return false;
    }
    bool MaterialSampleBSDF(const bsdf_parameters& P, pt3 In, pt3& Out, pt4& T, pt4& Pr)
    {
        uint32_t Type = MaterialType(P.MaterialIndex);
        if (Type == PT_MATERIAL_TYPE_BASIC_DIFFUSE) return BasicDiffuse_SampleBSDF(P, In, Out, T, Pr);
        if (Type == PT_MATERIAL_TYPE_BASIC_METAL) return BasicMetal_SampleBSDF(P, In, Out, T, Pr);
        if (Type == PT_MATERIAL_TYPE_BASIC_TRANSLUCENT) return BasicTranslucent_SampleBSDF(P, In, Out, T, Pr);
        if (Type == PT_MATERIAL_TYPE_OPENPBR && OpenPBR) {
            openpbr_parameters Q = OpenPBR_Parameters(P.MaterialIndex, P.TextureUV, P.Lambda, P.ExteriorIOR);
            return OpenPBR_Sample(Q, In, Out, T, Pr);
        }
        return false;
    }

    // --- basic_scatter.glsl ----------------------------------------------------------

    medium ResolveMedium(uint32_t ShapeIndex, pt4 Lambda)                                            // :44-64
    {
        medium Medium;
        if (ShapeIndex == SHAPE_INDEX_NONE) {
            Medium.Priority = 0xFFFFFFFFu;
            Medium.IOR = v4s(1.0f);
            Medium.AbsorptionRate = v4s(0.0f);
            Medium.ScatteringRate = v4s(S.Scene.SceneScatterRate);
            Medium.ScatteringAnisotropy = 0.0f;
        } else {
            const pt_packed_shape& Shape = S.Shapes[ShapeIndex];
            MaterialLoadMedium(Shape.MaterialIndex, Lambda, Medium);
            Medium.Priority = ShapeIndex;
        }
        return Medium;
    }

    bool SampleSurfaceIntegrand(const hit& Hit, const bsdf_parameters& Parameters, pt3 Out, pt3& In,  // :68-109
                                pt4& Throughput, pt4& Probability)
    {
        float LightProbability = MaterialHasDiracBSDF(Parameters) ? 0.0f : S.Scene.SkyboxSamplingProbability;
        pt4 MaterialPDF = v4s(0.0f);
        pt3 SMD = f3(S.Scene.SkyboxMeanDirection);
        pt3 SkyboxMeanDirection = v3(dot(SMD, Hit.TangentX), dot(SMD, Hit.TangentY), dot(SMD, Hit.Normal));
        if (G.R01() < LightProbability) {
            In = RandomVonMisesFisher(G, S.Scene.SkyboxConcentration, SkyboxMeanDirection);
            if (In.z < 0.0f) return false;
            if (!MaterialEvaluateBSDF(Parameters, Out, In, Throughput, MaterialPDF)) return false;
        } else {
            if (!MaterialSampleBSDF(Parameters, Out, In, Throughput, MaterialPDF)) return false;
        }
        pt4 SkyboxPDF = v4s(VonMisesFisherPDF(S.Scene.SkyboxConcentration, SkyboxMeanDirection, In));
        Probability = LightProbability * SkyboxPDF + (1 - LightProbability) * MaterialPDF;
        return true;
    }

    pt4 ClusterLambda(float L0)                                                                      // :116-122
    {
        return v4(pt_mix(PT_CIE_LAMBDA_MIN, PT_CIE_LAMBDA_MAX, L0),
                  pt_mix(PT_CIE_LAMBDA_MIN, PT_CIE_LAMBDA_MAX, pt_fract(L0 + 0.25f)),
                  pt_mix(PT_CIE_LAMBDA_MIN, PT_CIE_LAMBDA_MAX, pt_fract(L0 + 0.50f)),
                  pt_mix(PT_CIE_LAMBDA_MIN, PT_CIE_LAMBDA_MAX, pt_fract(L0 + 0.75f)));
    }

    bool Scatter(path& Path, ray& Ray, const hit& Hit)                                               // :114-310
    {
        pt4 Lambda = ClusterLambda(Path.NormalizedLambda0);

        uint32_t ActiveShapeIndex = SHAPE_INDEX_NONE;
        for (int I = 0; I < ACTIVE_SHAPE_LIMIT; I++) ActiveShapeIndex = pt_umin(ActiveShapeIndex, Path.ActiveShapeIndex[I]);

        medium Medium = ResolveMedium(ActiveShapeIndex, Lambda);

        Path.Throughput = Path.Throughput * vexp(-Medium.AbsorptionRate * Hit.Time);

        float ScatteringTime = PT_HIT_TIME_LIMIT;
        if (Medium.ScatteringRate.x > 0.0f) ScatteringTime = -pt_log(G.R01()) / Medium.ScatteringRate.x;

        if (Hit.Time >= ScatteringTime) {
            if (ScatteringTime < PT_HIT_TIME_LIMIT) {
                Ray.Origin = Ray.Origin + Ray.Velocity * ScatteringTime;
                pt3 X, Y, Z = Ray.Velocity;
                ComputeCoordinateFrame(Z, X, Y);
                float U1 = G.R01();
                float U2 = G.R01();
                pt3 Scattered = SampleDirectionHG(Medium.ScatteringAnisotropy, U1, U2);
                pt4 Density = Medium.ScatteringRate * vexp(-Medium.ScatteringRate * ScatteringTime);
                Density = Density / pt_max(PT_EPSILON, max4(Density));
                Path.Throughput = Path.Throughput * Density;
                Path.Probability = Path.Probability * Density;
                Ray.Velocity = normalize(X * Scattered.x + Y * Scattered.y + Z * Scattered.z);
                Ray.Duration = PT_HIT_TIME_LIMIT;
            } else {
                pt4 Emission = SampleSkyboxRadiance(Ray.Velocity, Lambda);
                float ClusterPDF = Path.Probability.x + Path.Probability.y + Path.Probability.z + Path.Probability.w;
                pt3 O0 = SampleStandardObserver(Lambda.x), O1 = SampleStandardObserver(Lambda.y);
                pt3 O2 = SampleStandardObserver(Lambda.z), O3 = SampleStandardObserver(Lambda.w);
                pt4 E = Emission * Path.Throughput;
                pt3 XYZ = O0 * E.x + O1 * E.y + O2 * E.z + O3 * E.w;   // mat4x3 * vec4
                Path.Sample = Path.Sample + XYZ / ClusterPDF;
                Path.Probability = v4s(0.0f);
            }
            return max4(Path.Probability) > PT_EPSILON;
        }

        pt3 In;
        pt3 Out = -v3(dot(Ray.Velocity, Hit.TangentX), dot(Ray.Velocity, Hit.TangentY), dot(Ray.Velocity, Hit.Normal));

        bool IsRealSurface = true;
        pt4 ExteriorIOR = v4s(1.0f);
        uint32_t ShapePriority = Hit.ShapeIndex;

        if (Out.z > 0) {
            IsRealSurface = Medium.Priority > ShapePriority;
            if (IsRealSurface) ExteriorIOR = Medium.IOR;
        } else {
            IsRealSurface = Medium.Priority == ShapePriority;
            if (IsRealSurface) {
                uint32_t ExteriorShapeIndex = SHAPE_INDEX_NONE;
                for (int I = 0; I < ACTIVE_SHAPE_LIMIT; I++) {
                    if (Path.ActiveShapeIndex[I] == ActiveShapeIndex) continue;
                    ExteriorShapeIndex = pt_umin(ExteriorShapeIndex, Path.ActiveShapeIndex[I]);
                }
                medium Exterior = ResolveMedium(ExteriorShapeIndex, Lambda);
                ExteriorIOR = Exterior.IOR;
            }
        }

        if (IsRealSurface) {
            bsdf_parameters Parameters;
            Parameters.MaterialIndex = Hit.MaterialIndex;
            Parameters.TextureUV = Hit.UV;
            Parameters.Lambda = Lambda;
            Parameters.ExteriorIOR = ExteriorIOR;
            pt4 Throughput, Probability;
            if (!SampleSurfaceIntegrand(Hit, Parameters, Out, In, Throughput, Probability)) return false;
            float Scale = 1.0f / pt_max(PT_EPSILON, max4(Probability));
            Path.Throughput = Path.Throughput * (Throughput * Scale);
            Path.Probability = Path.Probability * (Probability * Scale);
        } else {
            In = -Out;
        }

        if (In.z * Out.z < 0) {
            if (Out.z > 0) {
                for (int I = 0; I < ACTIVE_SHAPE_LIMIT; I++)
                    if (Path.ActiveShapeIndex[I] == SHAPE_INDEX_NONE) { Path.ActiveShapeIndex[I] = Hit.ShapeIndex; break; }
            } else {
                for (int I = 0; I < ACTIVE_SHAPE_LIMIT; I++)
                    if (Path.ActiveShapeIndex[I] == Hit.ShapeIndex) { Path.ActiveShapeIndex[I] = SHAPE_INDEX_NONE; break; }
            }
        }

        if (G.R01() < PathTerminationProbability) return false;
        Path.Probability = Path.Probability * (1.0f - PathTerminationProbability);

        Ray.Velocity = In.x * Hit.TangentX + In.y * Hit.TangentY + In.z * Hit.Normal;
        Ray.Origin = Hit.Position + 1e-3f * Ray.Velocity;
        Ray.Duration = PT_HIT_TIME_LIMIT;
        return max4(Path.Probability) > PT_EPSILON;
    }

    float PathTerminationProbability = 0.0f;
};

// Per-pixel SoA state in the reference's packed form.
struct pixel_state {
    float OriginX, OriginY, OriginZ;
    uint32_t PackedVelocity;
    pt_hit_record Hit;
    float Lambda0;
    float Throughput[4], Probability[4], Sample[3];
    uint32_t Active01, Active23;
};

}  // namespace

struct oracle_renderer {
    scene_data Scene;
    uint32_t W, H, Rank, NRanks;
    int Threads;
    pt_basic_renderer_params Params{};
    bool OpenPBR = false;                  // oracle_set_openpbr
    std::vector<uint32_t> Pixels;          // owned pixel indices (y*W+x)
    std::vector<pixel_state> State;        // parallel to Pixels
    std::vector<float> Accum;              // W*H*4
    uint64_t Rays = 0, Samples = 0;

    oracle_renderer(const pt_scene_packs* p, uint32_t w, uint32_t h, uint32_t rank, uint32_t nranks, int threads)
        : Scene(p), W(w), H(h), Rank(rank), NRanks(nranks ? nranks : 1), Threads(threads)
    {
        for (uint32_t y = 0; y < H; y++)
            if ((y / 16) % NRanks == Rank)
                for (uint32_t x = 0; x < W; x++) Pixels.push_back(y * W + x);
        State.resize(Pixels.size());
        Accum.assign((size_t)W * H * 4, 0.0f);
        // threads = 0: OMP_NUM_THREADS when set (the GPU box's CPU share),
        // else the hardware concurrency, at most 64 either way.
        if (Threads <= 0) {
            const char* e = std::getenv("OMP_NUM_THREADS");
            Threads = e ? std::atoi(e) : 0;
        }
        if (Threads <= 0) Threads = (int)std::thread::hardware_concurrency();
        Threads = std::max(1, std::min(Threads, 64));
    }

    template <class F>
    void ParallelFor(size_t n, F&& f)
    {
        int T = std::min<int>(Threads, (int)((n + 1023) / 1024));
        if (T <= 1) { for (size_t i = 0; i < n; i++) f(i); return; }
        std::atomic<size_t> next{0};
        auto worker = [&]() {
            for (;;) {
                size_t b = next.fetch_add(4096);
                if (b >= n) break;
                size_t e = std::min(n, b + 4096);
                for (size_t i = b; i < e; i++) f(i);
            }
        };
        std::vector<std::thread> pool;
        for (int t = 0; t < T; t++) pool.emplace_back(worker);
        for (auto& t : pool) t.join();
    }

    // basic_trace.glsl:7-16 (every slot is traced; the reference's
    // W*H/256 dispatch defect K8 is not reproduced).
    void TracePhase()
    {
        ParallelFor(Pixels.size(), [&](size_t i) {
            context C(Scene);
            pixel_state& P = State[i];
            ray Ray;
            Ray.Origin = v3(P.OriginX, P.OriginY, P.OriginZ);
            Ray.Velocity = UnpackUnitVector(P.PackedVelocity);
            Ray.Duration = PT_HIT_TIME_LIMIT;
            hit Hit = C.Trace(Ray);
            // StoreTraceHit (basic.glsl.inc:142-157)
            if (Hit.ShapeIndex == SHAPE_INDEX_NONE) { P.Hit.shape_material = 0xFFFFFFFFu; return; }
            P.Hit.shape_material = (Hit.ShapeIndex << 16) | Hit.MaterialIndex;
            P.Hit.time = Hit.Time;
            P.Hit.packed_normal = PackUnitVector(Hit.Normal);
            P.Hit.packed_tangent = PackUnitVector(Hit.TangentX);
            P.Hit.u = Hit.UV.x;
            P.Hit.v = Hit.UV.y;
        });
        Rays += Pixels.size();
    }

    static void StoreTraceRay(pixel_state& P, const ray& Ray)                                         // basic.glsl.inc:133-140
    {
        P.OriginX = Ray.Origin.x; P.OriginY = Ray.Origin.y; P.OriginZ = Ray.Origin.z;
        P.PackedVelocity = PackUnitVector(Ray.Velocity);
    }

    static void StorePathVertexData(pixel_state& P, const path& Path)                                 // basic.glsl.inc:200-216
    {
        P.Throughput[0] = Path.Throughput.x; P.Throughput[1] = Path.Throughput.y;
        P.Throughput[2] = Path.Throughput.z; P.Throughput[3] = Path.Throughput.w;
        P.Probability[0] = Path.Probability.x; P.Probability[1] = Path.Probability.y;
        P.Probability[2] = Path.Probability.z; P.Probability[3] = Path.Probability.w;
        P.Sample[0] = Path.Sample.x; P.Sample[1] = Path.Sample.y; P.Sample[2] = Path.Sample.z;
        P.Active01 = (Path.ActiveShapeIndex[1] << 16) | Path.ActiveShapeIndex[0];
        P.Active23 = (Path.ActiveShapeIndex[3] << 16) | Path.ActiveShapeIndex[2];
    }

    // GenerateNewPath (basic_scatter.glsl:7-42)
    void GenerateNewPath(context& C, pixel_state& P, int X, int Y)
    {
        pt2 SamplePosition = v2((float)X, (float)Y);
        if (Params.RenderFlags & PT_RENDER_FLAG_SAMPLE_JITTER) {
            float JX = C.G.R01();
            float JY = C.G.R01();
            SamplePosition = SamplePosition + v2(JX, JY);
        } else {
            SamplePosition = SamplePosition + v2(0.5f, 0.5f);
        }
        pt2 NSP = SamplePosition / v2((float)W, (float)H);
        const pt_packed_camera& Camera = Scene.Cameras[Params.CameraIndex];
        ray Ray = C.GenerateCameraRay(Camera, NSP);
        StoreTraceRay(P, Ray);
        path Path;
        Path.NormalizedLambda0 = C.G.R01();
        Path.Throughput = v4s(1.0f);
        Path.Probability = v4s(1.0f);
        Path.Sample = v3s(0.0f);
        for (int I = 0; I < 4; I++) Path.ActiveShapeIndex[I] = SHAPE_INDEX_NONE;
        P.Lambda0 = Path.NormalizedLambda0;
        StorePathVertexData(P, Path);
    }

    // basic_scatter.glsl:312-360
    void ScatterPhase(uint32_t Seed, bool Restart)
    {
        std::atomic<uint64_t> done{0};
        ParallelFor(Pixels.size(), [&](size_t i) {
            context C(Scene);
            C.PathTerminationProbability = Params.PathTerminationProbability;
            C.OpenPBR = OpenPBR;
            uint32_t pix = Pixels[i];
            int X = (int)(pix % W), Y = (int)(pix / W);
            C.G.State = pt_seed((uint32_t)X, (uint32_t)Y, Seed);
            pixel_state& P = State[i];
            float* A = &Accum[(size_t)pix * 4];
            if (Restart) {
                GenerateNewPath(C, P, X, Y);
                A[0] = A[1] = A[2] = A[3] = 0.0f;
                return;
            }
            // LoadPath (basic.glsl.inc:159-198)
            path Path;
            Path.ImageX = X; Path.ImageY = Y;
            Path.NormalizedLambda0 = P.Lambda0;
            Path.Throughput = v4(P.Throughput[0], P.Throughput[1], P.Throughput[2], P.Throughput[3]);
            Path.Probability = v4(P.Probability[0], P.Probability[1], P.Probability[2], P.Probability[3]);
            Path.Sample = v3(P.Sample[0], P.Sample[1], P.Sample[2]);
            Path.ActiveShapeIndex[0] = P.Active01 & 0xFFFF;
            Path.ActiveShapeIndex[1] = P.Active01 >> 16;
            Path.ActiveShapeIndex[2] = P.Active23 & 0xFFFF;
            Path.ActiveShapeIndex[3] = P.Active23 >> 16;
            for (int I = 0; I < 4; I++)
                if (Path.ActiveShapeIndex[I] == 0xFFFF) Path.ActiveShapeIndex[I] = SHAPE_INDEX_NONE;
            // LoadTraceResult (basic.glsl.inc:99-131)
            ray Ray;
            hit Hit{};
            Ray.Origin = v3(P.OriginX, P.OriginY, P.OriginZ);
            Ray.Velocity = UnpackUnitVector(P.PackedVelocity);
            Ray.Duration = PT_HIT_TIME_LIMIT;
            if (P.Hit.shape_material == 0xFFFFFFFFu) {
                Hit.ShapeIndex = SHAPE_INDEX_NONE;
                Hit.Time = PT_HIT_TIME_LIMIT;
            } else {
                Hit.ShapeIndex = P.Hit.shape_material >> 16;
                Hit.MaterialIndex = P.Hit.shape_material & 0xFFFF;
                Hit.Time = P.Hit.time;
                Hit.Normal = UnpackUnitVector(P.Hit.packed_normal);
                Hit.TangentX = UnpackUnitVector(P.Hit.packed_tangent);
                Hit.TangentY = cross(Hit.Normal, Hit.TangentX);
                Hit.UV = v2(P.Hit.u, P.Hit.v);
                Hit.Position = Ray.Origin + Hit.Time * Ray.Velocity;
            }
            if (C.Scatter(Path, Ray, Hit)) {
                StoreTraceRay(P, Ray);
                StorePathVertexData(P, Path);
            } else {
                float V0 = Path.Sample.x, V1 = Path.Sample.y, V2 = Path.Sample.z, V3 = 1.0f;
                if (Params.RenderFlags & PT_RENDER_FLAG_ACCUMULATE) { V0 += A[0]; V1 += A[1]; V2 += A[2]; V3 += A[3]; }
                A[0] = V0; A[1] = V1; A[2] = V2; A[3] = V3;
                GenerateNewPath(C, P, X, Y);
                done.fetch_add(1, std::memory_order_relaxed);
            }
        });
        Samples += done.load();
    }
};

extern "C" {

oracle_renderer* oracle_create(const pt_scene_packs* packs, uint32_t width, uint32_t height, uint32_t rank,
                               uint32_t nranks, int threads)
{
    if (!packs || width == 0 || height == 0) return nullptr;
    return new oracle_renderer(packs, width, height, rank, nranks, threads);
}

void oracle_destroy(oracle_renderer* r) { delete r; }
pt_basic_renderer_params* oracle_params(oracle_renderer* r) { return &r->Params; }
void oracle_set_openpbr(oracle_renderer* r, int enable) { r->OpenPBR = enable != 0; }
// Worker threads of the following rounds (1..64; the CPU baseline's scaling runs).
void oracle_set_threads(oracle_renderer* r, int threads) { r->Threads = std::max(1, std::min(threads, 64)); }
void oracle_set_slab_division(int ieee) { SlabDivisionIEEE.store(ieee != 0); }
int oracle_slab_division(void) { return SlabDivisionIEEE.load(); }
float oracle_intersect_bounding_box(const float origin[3], const float velocity[3], float reach, const float mn[3],
                                    const float mx[3])
{
    ray R;
    R.Origin = v3(origin[0], origin[1], origin[2]);
    R.Velocity = v3(velocity[0], velocity[1], velocity[2]);
    R.Duration = reach;
    return IntersectBoundingBox(R, reach, v3(mn[0], mn[1], mn[2]), v3(mx[0], mx[1], mx[2]));
}

// ResetBasicRenderer (basic.cpp:285-304): one scatter dispatch, Restart=1,
// seeded with the current FrameIndex.
void oracle_reset(oracle_renderer* r) { r->ScatterPhase(r->Params.FrameIndex, true); }

// RunBasicRenderer (basic.cpp:306-332): ++FrameIndex, then Rounds x
// (trace, scatter) all with that seed.
void oracle_run(oracle_renderer* r, uint32_t rounds)
{
    r->Params.FrameIndex += 1;
    for (uint32_t i = 0; i < rounds; i++) {
        r->TracePhase();
        r->ScatterPhase(r->Params.FrameIndex, false);
    }
}

void oracle_read_accum(oracle_renderer* r, float* rgba) { std::memcpy(rgba, r->Accum.data(), r->Accum.size() * 4); }

void oracle_read_state(oracle_renderer* r, pt_pixel_state* out)
{
    for (size_t i = 0; i < r->Pixels.size(); i++) {
        const pixel_state& P = r->State[i];
        pt_pixel_state& O = out[r->Pixels[i]];
        O.origin[0] = P.OriginX; O.origin[1] = P.OriginY; O.origin[2] = P.OriginZ;
        O.packed_velocity = P.PackedVelocity;
        O.hit = P.Hit;
        O.lambda0 = P.Lambda0;
        std::memcpy(O.throughput, P.Throughput, 16);
        std::memcpy(O.probability, P.Probability, 16);
        std::memcpy(O.sample, P.Sample, 12);
        O.active01 = P.Active01;
        O.active23 = P.Active23;
    }
}

void oracle_counters(oracle_renderer* r, uint64_t* rays, uint64_t* samples)
{
    if (rays) *rays = r->Rays;
    if (samples) *samples = r->Samples;
}

void oracle_trace_rays(const pt_scene_packs* packs, uint32_t n, const float* origins, const uint32_t* vel,
                       const float* durations, pt_hit_record* out)
{
    scene_data S(packs);
    context C(S);
    for (uint32_t i = 0; i < n; i++) {
        ray Ray;
        Ray.Origin = v3(origins[3 * i], origins[3 * i + 1], origins[3 * i + 2]);
        Ray.Velocity = UnpackUnitVector(vel[i]);
        Ray.Duration = durations[i];
        hit Hit = C.Trace(Ray);
        pt_hit_record& O = out[i];
        std::memset(&O, 0, sizeof(O));
        if (Hit.ShapeIndex == SHAPE_INDEX_NONE) { O.shape_material = 0xFFFFFFFFu; continue; }
        O.shape_material = (Hit.ShapeIndex << 16) | Hit.MaterialIndex;
        O.time = Hit.Time;
        O.packed_normal = PackUnitVector(Hit.Normal);
        O.packed_tangent = PackUnitVector(Hit.TangentX);
        O.u = Hit.UV.x;
        O.v = Hit.UV.y;
    }
}

// --- resolve.glsl (RenderSampleBuffer) -----------------------------------------

namespace {

float Luminance(pt3 C) { return dot(C, v3(0.2126f, 0.7152f, 0.0722f)); }                       // resolve.glsl:61-64

pt3 Mat3TimesVec3(const float (&M)[3][3], pt3 V)   // GLSL mat3 * vec3, M[column][row]
{
    return v3(M[0][0] * V.x + M[1][0] * V.y + M[2][0] * V.z,
              M[0][1] * V.x + M[1][1] * V.y + M[2][1] * V.z,
              M[0][2] * V.x + M[1][2] * V.y + M[2][2] * V.z);
}

pt3 ToneMapReinhard(pt3 Color, float WhiteLevel)                                                // :66-73
{
    float OldL = Luminance(Color);
    float MaxL = WhiteLevel;
    float N = OldL * (1.0f + (OldL / (MaxL * MaxL)));
    float NewL = N / (1.0f + OldL);
    return Color * NewL / OldL;
}

pt3 ToneMapHablePartial(pt3 X)                                                                  // :75-80
{
    float A = 0.15f, B = 0.50f, C = 0.10f;
    float D = 0.20f, E = 0.02f, F = 0.30f;
    return ((X * (A * X + v3s(C * B)) + v3s(D * E)) / (X * (A * X + v3s(B)) + v3s(D * F))) - v3s(E / F);
}

pt3 ToneMapHable(pt3 Color)                                                                     // :82-89
{
    float ExposureBias = 2.0f;
    pt3 Current = ToneMapHablePartial(Color * ExposureBias);
    pt3 W = v3s(11.2f);
    pt3 WhiteScale = v3s(1.0f) / ToneMapHablePartial(W);
    return Current * WhiteScale;
}

const float ACES_INPUT_MATRIX[3][3] = {{0.59719f, 0.07600f, 0.02840f},                          // :91-96
                                       {0.35458f, 0.90834f, 0.13383f},
                                       {0.04823f, 0.01566f, 0.83777f}};
const float ACES_OUTPUT_MATRIX[3][3] = {{1.60475f, -0.10208f, -0.00327f},                       // :98-103
                                        {-0.53108f, 1.10813f, -0.07276f},
                                        {-0.07367f, -0.00605f, 1.07602f}};
const float CIE_XYZ_TO_SRGB[3][3] = {{+3.2406f, -0.9689f, +0.0557f},                            // spectrum.glsl.inc:50-55
                                     {-1.5372f, +1.8758f, -0.2040f},
                                     {-0.4986f, +0.0415f, +1.0570f}};

pt3 ToneMapACES(pt3 Color)                                                                      // :105-111
{
    pt3 V = Mat3TimesVec3(ACES_INPUT_MATRIX, Color);
    pt3 A = V * (V + v3s(0.0245786f)) - v3s(0.000090537f);
    pt3 B = V * (0.983729f * V + v3s(0.4329510f)) + v3s(0.238081f);
    return Mat3TimesVec3(ACES_OUTPUT_MATRIX, A / B);
}

// sRGB transfer + UNORM8 quantisation of a B8G8R8A8_SRGB store (vulkan.cpp:1407)
// under the build's convention (pt_exp/pt_log power, round half up).
uint8_t EncodeSRGB8(float C)
{
    C = pt_clamp(C, 0.0f, 1.0f);
    float E = C <= 0.0031308f ? 12.92f * C : 1.055f * pt_exp(pt_log(C) * (1.0f / 2.4f)) - 0.055f;
    return (uint8_t)(uint32_t)(pt_clamp(E, 0.0f, 1.0f) * 255.0f + 0.5f);
}

}  // namespace

void oracle_resolve(const float* accum, uint32_t n, const pt_resolve_parameters* P, float* out, uint8_t* out8)
{
    for (uint32_t i = 0; i < n; i++) {                                                          // main, :113-130
        const float* Value = accum + 4 * (size_t)i;
        pt3 Color = v3s(0.0f);
        if (Value[3] > 0)
            Color = Mat3TimesVec3(CIE_XYZ_TO_SRGB, P->Brightness * v3(Value[0], Value[1], Value[2]) / Value[3]);
        if (P->ToneMappingMode == PT_TONE_MAPPING_CLAMP)
            Color = v3(pt_clamp(Color.x, 0.0f, 1.0f), pt_clamp(Color.y, 0.0f, 1.0f), pt_clamp(Color.z, 0.0f, 1.0f));
        if (P->ToneMappingMode == PT_TONE_MAPPING_REINHARD) Color = ToneMapReinhard(Color, P->ToneMappingWhiteLevel);
        if (P->ToneMappingMode == PT_TONE_MAPPING_HABLE) Color = ToneMapHable(Color);
        if (P->ToneMappingMode == PT_TONE_MAPPING_ACES) Color = ToneMapACES(Color);
        float* O = out + 4 * (size_t)i;
        O[0] = Color.x; O[1] = Color.y; O[2] = Color.z; O[3] = 1.0f;
        uint8_t* O8 = out8 + 4 * (size_t)i;
        O8[0] = EncodeSRGB8(Color.x); O8[1] = EncodeSRGB8(Color.y); O8[2] = EncodeSRGB8(Color.z); O8[3] = 255;
    }
}

// --- preview_render.glsl (RenderPreview) ----------------------------------------

namespace {

const float D65[PT_CIE_D65_COUNT] = {PT_CIE_D65_VALUES};                                         // spectrum.glsl.inc:56-157

float SampleIlluminantD65(float NormalizedLambda)                                               // :159-164
{
    float Offset = NormalizedLambda * 470;
    int Index = (int)Offset;
    Index = Index < 0 ? 0 : (Index > 469 ? 469 : Index);
    return pt_mix(D65[Index], D65[Index + 1], Offset - (float)Index);
}

float SampleParametricSpectrumI(pt4 BetaAndIntensity, float Lambda)                            // :183-186
{
    return BetaAndIntensity.w * SampleParametricSpectrum(v3(BetaAndIntensity.x, BetaAndIntensity.y, BetaAndIntensity.z), Lambda);
}

pt3 ObserveParametricSpectrumUnderD65(pt4 BetaAndIntensity)                                     // :194-208
{
    const int SampleCount = 16;
    const float DeltaLambda = (PT_CIE_LAMBDA_MAX - PT_CIE_LAMBDA_MIN) / SampleCount;
    pt3 Color = v3s(0);
    for (int I = 0; I < SampleCount; I++) {
        float NormalizedLambda = (float)I / (float)(SampleCount - 1);
        float D = SampleIlluminantD65(NormalizedLambda) / PT_CIE_D65_NORMALIZATION;
        float Lambda = pt_mix(PT_CIE_LAMBDA_MIN, PT_CIE_LAMBDA_MAX, NormalizedLambda);
        Color = Color + SampleParametricSpectrumI(BetaAndIntensity, Lambda) * D * SampleStandardObserver(Lambda) * DeltaLambda;
    }
    return Color;
}

pt3 ObserveBetaUnderD65(pt3 Beta) { return ObserveParametricSpectrumUnderD65(v4(Beta.x, Beta.y, Beta.z, 1)); }   // :210-213

const float PREVIEW_COLORS[20][3] = {                                                           // preview_render.glsl:16-38
    {0.902f, 0.098f, 0.294f}, {0.235f, 0.706f, 0.294f}, {1.000f, 0.882f, 0.098f}, {0.263f, 0.388f, 0.847f},
    {0.961f, 0.510f, 0.192f}, {0.569f, 0.118f, 0.706f}, {0.275f, 0.941f, 0.941f}, {0.941f, 0.196f, 0.902f},
    {0.737f, 0.965f, 0.047f}, {0.980f, 0.745f, 0.745f}, {0.000f, 0.502f, 0.502f}, {0.902f, 0.745f, 1.000f},
    {0.604f, 0.388f, 0.141f}, {1.000f, 0.980f, 0.784f}, {0.502f, 0.000f, 0.000f}, {0.667f, 1.000f, 0.765f},
    {0.502f, 0.502f, 0.000f}, {1.000f, 0.847f, 0.694f}, {0.000f, 0.000f, 0.459f}, {0.502f, 0.502f, 0.502f}};

pt3 PreviewColor(uint32_t I) { return v3(PREVIEW_COLORS[I % 20][0], PREVIEW_COLORS[I % 20][1], PREVIEW_COLORS[I % 20][2]); }

struct preview_context {
    const context& C;

    pt3 MaterialColor(uint32_t M, uint32_t A) const                                             // scene.glsl.inc:254-258
    {
        return ObserveBetaUnderD65(C.MaterialVec3(M, A));
    }

    pt3 MaterialTexturableColor(uint32_t M, uint32_t A, pt2 UV) const                           // :260-274
    {
        pt3 Color = ObserveBetaUnderD65(C.MaterialVec3(M, A + 0));
        uint32_t TextureIndex = C.MaterialUint(M, A + 3);
        if (TextureIndex != TEXTURE_INDEX_NONE) {
            pt4 T = C.SampleTexture(TextureIndex, UV);
            Color = Color * ObserveBetaUnderD65(v3(T.x, T.y, T.z));
        }
        return Color;
    }

    pt3 MaterialBaseColor(uint32_t M, pt2 UV) const                                             // :696-701 + *_BaseColor
    {
        uint32_t Type = C.MaterialType(M);
        if (Type == PT_MATERIAL_TYPE_BASIC_DIFFUSE) return MaterialTexturableColor(M, PT_BASIC_DIFFUSE_BASE_SPECTRUM, UV);
        if (Type == PT_MATERIAL_TYPE_BASIC_METAL) return MaterialTexturableColor(M, PT_BASIC_METAL_BASE_SPECTRUM, UV);
        if (Type == PT_MATERIAL_TYPE_BASIC_TRANSLUCENT) return MaterialColor(M, PT_BASIC_TRANSLUCENT_TRANSMISSION_SPECTRUM);
        return v3s(0);
    }
};

}  // namespace

void oracle_preview(const pt_scene_packs* packs, const pt_preview_parameters* P, float* rgba, pt_preview_aov* aov,
                    uint32_t* hit_shape_index)
{
    scene_data S(packs);
    context C(S);
    preview_context PC{C};
    const uint32_t W = P->RenderSizeX, H = P->RenderSizeY;
    for (uint32_t Py = 0; Py < H; Py++)
        for (uint32_t Px = 0; Px < W; Px++) {                                                   // main, :96-178
            // ScreenXY interpolated at the pixel centre of a W x H viewport
            pt2 ScreenXY = v2(((float)Px + 0.5f) / (float)W, ((float)Py + 0.5f) / (float)H);
            float AspectRatio = (float)W / (float)H;
            float NearX = (ScreenXY.x - 0.5f) * AspectRatio;
            float NearY = 0.5f - ScreenXY.y;
            ray Ray;
            Ray.Origin = v3s(0);
            Ray.Velocity = normalize(v3(NearX, NearY, -1.0f));
            Ray.Duration = PT_HIT_TIME_LIMIT;
            Ray = TransformRay(Ray, P->CameraTransform);
            hit Hit = C.Trace(Ray);
            pt3 Color = v3s(0);
            bool Miss = Hit.ShapeIndex == SHAPE_INDEX_NONE;
            switch (P->RenderMode) {
            case PT_PREVIEW_RENDER_MODE_BASE_COLOR:
            case PT_PREVIEW_RENDER_MODE_BASE_COLOR_SHADED:
                if (Miss) {
                    Color = Mat3TimesVec3(CIE_XYZ_TO_SRGB, ObserveParametricSpectrumUnderD65(C.SampleSkyboxSpectrum(Ray.Velocity)));
                } else {
                    Color = Mat3TimesVec3(CIE_XYZ_TO_SRGB, PC.MaterialBaseColor(Hit.MaterialIndex, Hit.UV));
                    if (P->RenderMode == PT_PREVIEW_RENDER_MODE_BASE_COLOR_SHADED)
                        Color = Color * dot(Hit.Normal, -Ray.Velocity);
                }
                break;
            case PT_PREVIEW_RENDER_MODE_NORMAL:
                Color = Miss ? 0.5f * (v3s(1) - Ray.Velocity) : 0.5f * (Hit.Normal + v3s(1));
                break;
            case PT_PREVIEW_RENDER_MODE_MATERIAL_INDEX:
                if (!Miss) Color = PreviewColor(Hit.MaterialIndex);
                break;
            case PT_PREVIEW_RENDER_MODE_PRIMITIVE_INDEX:
                if (!Miss) Color = PreviewColor(Hit.PrimitiveIndex);
                break;
            case PT_PREVIEW_RENDER_MODE_MESH_COMPLEXITY:
                Color = v3(0, 1, 0) * (float)Hit.MeshComplexity / 256.0f;
                break;
            case PT_PREVIEW_RENDER_MODE_SCENE_COMPLEXITY:
                Color = v3(0, 1, 0) * (float)Hit.SceneComplexity / 256.0f;
                break;
            }
            if (Hit.ShapeIndex == P->SelectedShapeIndex) Color = Color * v3(1.0f, 0.5f, 0.5f);
            Color = Color * P->Brightness;
            if (hit_shape_index && Px == P->MouseX && Py == P->MouseY) *hit_shape_index = Hit.ShapeIndex;
            size_t i = (size_t)Py * W + Px;
            if (rgba) { rgba[4 * i] = Color.x; rgba[4 * i + 1] = Color.y; rgba[4 * i + 2] = Color.z; rgba[4 * i + 3] = 1.0f; }
            if (aov) {
                pt_preview_aov& A = aov[i];
                std::memset(&A, 0, sizeof(A));
                A.shape_index = Hit.ShapeIndex;
                A.mesh_complexity = Hit.MeshComplexity;
                A.scene_complexity = Hit.SceneComplexity;
                if (!Miss) {
                    A.time = Hit.Time;
                    A.material_index = Hit.MaterialIndex;
                    A.primitive_index = Hit.PrimitiveIndex;
                    A.normal[0] = Hit.Normal.x; A.normal[1] = Hit.Normal.y; A.normal[2] = Hit.Normal.z;
                    A.u = Hit.UV.x; A.v = Hit.UV.y;
                }
            }
        }
}

float oracle_fp_exp(float x) { return pt_exp(x); }
float oracle_fp_log(float x) { return pt_log(x); }
float oracle_fp_sin(float x) { return pt_sin(x); }
float oracle_fp_cos(float x) { return pt_cos(x); }
float oracle_fp_atan2(float y, float x) { return pt_atan2(y, x); }
float oracle_fp_asin(float x) { return pt_asin(x); }
uint32_t oracle_pcg(uint32_t* state) { return pt_random(state); }
uint32_t oracle_pack_unit_vector(const float v[3]) { return PackUnitVector(v3(v[0], v[1], v[2])); }
float oracle_unpack_snorm16(uint32_t bits) { return pt_unpack_snorm16(bits); }
void oracle_unpack_unit_vector(uint32_t packed, float out[3])
{
    pt3 v = UnpackUnitVector(packed);
    out[0] = v.x; out[1] = v.y; out[2] = v.z;
}
void oracle_sample_observer(float lambda, float out[3])
{
    pt3 v = SampleStandardObserver(lambda);
    out[0] = v.x; out[1] = v.y; out[2] = v.z;
}

}  // extern "C"
