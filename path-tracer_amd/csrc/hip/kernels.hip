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
// t = s/256, so a 64-lane wave holds a 16x4 pixel block (coherent primary
// rays) and a renderer can own an arbitrary set of 16-row bands.
#include "pt_device.hpp"
#include "kernels.hpp"

namespace ptd {

// --- traversal stack: LDS columns + global spill ----------------------------

template <bool SPILL>
struct tstack {
    uint32_t* lds;        // &smem[tid]; entry i at lds[i * 256]
    uint32_t* spill;      // &spill[slot]; entry i (>= PT_LDS_STACK) at spill[(i - CAP) * stride]
    uint32_t stride;
    PT_DEV void put(uint32_t i, uint32_t v)
    {
        if (!SPILL || i < PT_LDS_STACK) lds[i * 256] = v;
        else spill[(i - PT_LDS_STACK) * stride] = v;
    }
    PT_DEV uint32_t get(uint32_t i) const
    {
        if (!SPILL || i < PT_LDS_STACK) return lds[i * 256];
        return spill[(i - PT_LDS_STACK) * stride];
    }
};

struct thit {
    float Time;
    uint32_t ShapeIndex;
    uint32_t ShapeType;
    uint32_t PrimitiveIndex;
    pt3 Coords;
};

// IntersectMeshFace (scene.glsl.inc:304-334)
PT_DEV void IntersectMeshFace(const dscene& S, pt3 O, pt3 V, uint32_t F, thit& H)
{
    float4 a = S.mesh_faces[3 * F + 0], b = S.mesh_faces[3 * F + 1], c = S.mesh_faces[3 * F + 2];
    pt3 P0 = xyz(a), P1 = xyz(b), P2 = xyz(c);
    pt3 Edge1 = P1 - P0;
    pt3 Edge2 = P2 - P0;
    pt3 RCE2 = cross(V, Edge2);
    float Det = dot(Edge1, RCE2);
    if (pt_abs(Det) < PT_EPSILON) return;
    float InvDet = 1.0f / Det;
    pt3 Sv = O - P0;
    float U = InvDet * dot(Sv, RCE2);
    if (U < 0 || U > 1) return;
    pt3 SCE1 = cross(Sv, Edge1);
    float W = InvDet * dot(V, SCE1);
    if (W < 0 || U + W > 1) return;
    float T = InvDet * dot(Edge2, SCE1);
    if (T < 0 || T > H.Time) return;
    H.Time = T;
    H.ShapeType = PT_SHAPE_TYPE_MESH_INSTANCE;
    H.ShapeIndex = 0xFFFFFFFEu;
    H.PrimitiveIndex = F;
    H.Coords = v3(1 - U - W, U, W);
}

// IntersectMeshNode (scene.glsl.inc:336-399); BLAS entries are stacked above
// the TLAS entries (base), 32 per level like the reference's Stack[32].
template <bool SPILL>
PT_DEV void IntersectMeshNode(const dscene& S, pt3 O, pt3 V, uint32_t Root, thit& H, tstack<SPILL>& st, uint32_t base)
{
    uint32_t Depth = 0;
    float4 n0 = S.mesh_nodes[2 * Root], n1 = S.mesh_nodes[2 * Root + 1];
    while (true) {
        uint32_t Begin = __float_as_uint(n0.w), End = __float_as_uint(n1.w);
        if (End > 0) {
            for (uint32_t F = Begin; F < End; F++) IntersectMeshFace(S, O, V, F, H);
        } else {
            uint32_t Index = Begin;
            n0 = S.mesh_nodes[2 * Index]; n1 = S.mesh_nodes[2 * Index + 1];
            float TimeA = IntersectBoundingBox(O, V, H.Time, n0, n1);
            float4 m0 = S.mesh_nodes[2 * Index + 2], m1 = S.mesh_nodes[2 * Index + 3];
            float TimeB = IntersectBoundingBox(O, V, H.Time, m0, m1);
            if (TimeA > TimeB) {
                if (TimeA < PT_INFINITY && Depth < 32) st.put(base + Depth++, Index);
                n0 = m0; n1 = m1;
                continue;
            }
            if (TimeB < PT_INFINITY) {
                if (Depth < 32) st.put(base + Depth++, Index + 1);
                continue;
            }
            if (TimeA < PT_INFINITY) continue;
        }
        if (Depth == 0) break;
        uint32_t I = st.get(base + --Depth);
        n0 = S.mesh_nodes[2 * I]; n1 = S.mesh_nodes[2 * I + 1];
    }
}

// IntersectShape (scene.glsl.inc:401-466)
template <bool SPILL>
PT_DEV void IntersectShape(const dscene& S, pt3 WO, pt3 WV, uint32_t ShapeIndex, thit& H, tstack<SPILL>& st, uint32_t base)
{
    const pt_packed_shape* Shape = &S.shapes[ShapeIndex];
    const float* From = Shape->Transform.From;
    pt3 O = mat4_mul_point(From, WO);
    pt3 V = mat4_mul_vector(From, WV);
    int32_t Type = Shape->Type;
    if (Type == PT_SHAPE_TYPE_MESH_INSTANCE) {
        IntersectMeshNode<SPILL>(S, O, V, Shape->MeshRootNodeIndex, H, st, base);
        if (H.ShapeIndex == 0xFFFFFFFEu) H.ShapeIndex = ShapeIndex;
    } else if (Type == PT_SHAPE_TYPE_PLANE) {
        float T = -O.z / V.z;
        if (T < 0 || T > H.Time) return;
        H.Time = T;
        H.ShapeType = PT_SHAPE_TYPE_PLANE;
        H.ShapeIndex = ShapeIndex;
        H.PrimitiveIndex = 0;
        H.Coords = O + V * T;
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
        if (Sv < 0 || Sv > Vv * H.Time) return;
        H.Time = Sv / Vv;
        H.ShapeType = PT_SHAPE_TYPE_SPHERE;
        H.ShapeIndex = ShapeIndex;
        H.PrimitiveIndex = 0;
        H.Coords = O + V * H.Time;
    } else if (Type == PT_SHAPE_TYPE_CUBE) {
        pt3 Mn = (v3s(-1) - O) / V;
        pt3 Mx = (v3s(+1) - O) / V;
        pt3 E = vmin(Mn, Mx);
        pt3 L = vmax(Mn, Mx);
        float T0 = pt_max(pt_max(E.x, E.y), E.z);
        float T1 = pt_min(pt_min(L.x, L.y), L.z);
        if (T1 < T0) return;
        if (T1 <= 0) return;
        float T = T0 < 0 ? T1 : T0;
        if (T >= H.Time) return;
        H.Time = T;
        H.ShapeType = PT_SHAPE_TYPE_CUBE;
        H.ShapeIndex = ShapeIndex;
        H.PrimitiveIndex = 0;
        H.Coords = O + V * T;
    }
}

// Trace (scene.glsl.inc:468-611) -> packed hit record.
template <bool SPILL>
PT_DEV void TraceRecord(const dscene& S, pt3 O, pt3 V, float Duration, tstack<SPILL>& st, float4& rec, float2& uv,
                        bool& isHit)
{
    thit H;
    H.ShapeIndex = SHAPE_INDEX_NONE;
    H.Time = Duration;
    H.ShapeType = 0;
    H.PrimitiveIndex = 0;
    H.Coords = v3s(0);
    if (S.g.ShapeCount != 0) {
        uint32_t Depth = 0;
        float4 a0 = S.shape_nodes[0], a1 = S.shape_nodes[1];
        while (true) {
            uint32_t Children = __float_as_uint(a0.w);
            if (Children == 0) {
                IntersectShape<SPILL>(S, O, V, __float_as_uint(a1.w), H, st, Depth);
            } else {
                uint32_t IA = Children & 0xFFFF, IB = Children >> 16;
                a0 = S.shape_nodes[2 * IA]; a1 = S.shape_nodes[2 * IA + 1];
                float4 b0 = S.shape_nodes[2 * IB], b1 = S.shape_nodes[2 * IB + 1];
                float TA = IntersectBoundingBox(O, V, H.Time, a0, a1);
                float TB = IntersectBoundingBox(O, V, H.Time, b0, b1);
                if (TA > TB) {
                    if (TA < PT_INFINITY && Depth < 32) st.put(Depth++, IA);
                    a0 = b0; a1 = b1;
                    continue;
                }
                if (TB < PT_INFINITY) {
                    if (Depth < 32) st.put(Depth++, IB);
                    continue;
                }
                if (TA < PT_INFINITY) continue;
            }
            if (Depth == 0) break;
            uint32_t I = st.get(--Depth);
            a0 = S.shape_nodes[2 * I]; a1 = S.shape_nodes[2 * I + 1];
        }
    }
    isHit = H.ShapeIndex != SHAPE_INDEX_NONE;
    if (!isHit) return;

    const pt_packed_shape* Shape = &S.shapes[H.ShapeIndex];
    uint32_t MaterialIndex = Shape->MaterialIndex;
    const float* To = Shape->Transform.To;
    const float* From = Shape->Transform.From;
    pt3 Normal, TangentX;
    pt2 UV;
    if (H.ShapeType == PT_SHAPE_TYPE_MESH_INSTANCE) {
        float4 f0 = S.mesh_faces[3 * H.PrimitiveIndex + 0];
        float4 f1 = S.mesh_faces[3 * H.PrimitiveIndex + 1];
        float4 f2 = S.mesh_faces[3 * H.PrimitiveIndex + 2];
        uint2 V0 = S.mesh_vertices[__float_as_uint(f0.w)];
        uint2 V1 = S.mesh_vertices[__float_as_uint(f1.w)];
        uint2 V2 = S.mesh_vertices[__float_as_uint(f2.w)];
        pt3 C = H.Coords;
        pt3 N = SafeNormalize(UnpackUnitVector(V0.x) * C.x + UnpackUnitVector(V1.x) * C.y + UnpackUnitVector(V2.x) * C.z);
        Normal = TransformNormal(N, From);
        TangentX = ComputeTangentVector(Normal);
        pt2 UV0 = v2(pt_half_to_float(V0.y & 0xFFFF), pt_half_to_float(V0.y >> 16));
        pt2 UV1 = v2(pt_half_to_float(V1.y & 0xFFFF), pt_half_to_float(V1.y >> 16));
        pt2 UV2 = v2(pt_half_to_float(V2.y & 0xFFFF), pt_half_to_float(V2.y >> 16));
        UV = UV0 * C.x + UV1 * C.y + UV2 * C.z;
    } else if (H.ShapeType == PT_SHAPE_TYPE_PLANE) {
        Normal = TransformNormal(v3(0, 0, 1), From);
        TangentX = TransformDirection(v3(1, 0, 0), To);
        UV = v2(pt_fract(H.Coords.x), pt_fract(H.Coords.y));
    } else if (H.ShapeType == PT_SHAPE_TYPE_SPHERE) {
        pt3 P = H.Coords;
        float U = (pt_atan2(P.y, P.x) + PT_PI) / PT_TAU;
        float W = (P.z + 1.0f) / 2.0f;
        Normal = TransformNormal(P, From);
        TangentX = TransformDirection(cross(P, v3(-P.y, P.x, 0)), To);
        UV = v2(U, W);
    } else {
        pt3 P = H.Coords;
        pt3 Q = vabs(P);
        pt3 N, T;
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
        Normal = TransformNormal(N, From);
        TangentX = TransformDirection(T, To);
    }
    // StoreTraceHit (basic.glsl.inc:142-157)
    rec.x = H.Time;
    rec.y = __uint_as_float((H.ShapeIndex << 16) | MaterialIndex);
    rec.z = __uint_as_float(PackUnitVector(Normal));
    rec.w = __uint_as_float(PackUnitVector(TangentX));
    uv = make_float2(UV.x, UV.y);
}

// --- slot / pixel mapping ---------------------------------------------------

PT_DEV bool SlotPixel(const dframe& F, uint32_t s, uint32_t& x, uint32_t& y)
{
    uint32_t t = s >> 8, l = s & 255u;
    uint32_t k = t / F.tiles_x;
    uint32_t tx = t - k * F.tiles_x;
    uint32_t band = F.rank + k * F.nranks;
    x = tx * 16 + (l & 15u);
    y = band * 16 + (l >> 4);
    return x < F.width && y < F.height;
}

// --- materials ---------------------------------------------------------------

struct bsdf_parameters { uint32_t MaterialIndex; pt2 TextureUV; pt4 Lambda; pt4 ExteriorIOR; };

PT_DEV bool Diffuse_Evaluate(const dscene& S, const bsdf_parameters& P, pt3 In, pt4& T, pt4& Pr)
{
    pt4 R = MaterialTexturableReflectance(S, P.MaterialIndex, PT_BASIC_DIFFUSE_BASE_SPECTRUM, P.Lambda, P.TextureUV);
    Pr = v4s(In.z / PT_PI);
    T = Pr * R;
    return true;
}

PT_DEV void Metal_GetParameters(const dscene& S, const bsdf_parameters& P, pt4& Base, pt4& Spec, pt2& A, bool& Rough)
{
    Base = MaterialTexturableReflectance(S, P.MaterialIndex, PT_BASIC_METAL_BASE_SPECTRUM, P.Lambda, P.TextureUV);
    Spec = MaterialTexturableReflectance(S, P.MaterialIndex, PT_BASIC_METAL_SPECULAR_SPECTRUM, P.Lambda, P.TextureUV);
    A = GGXRoughnessAlpha(MaterialTexturableValue(S, P.MaterialIndex, PT_BASIC_METAL_ROUGHNESS, P.TextureUV),
                          MaterialTexturableValue(S, P.MaterialIndex, PT_BASIC_METAL_ROUGHNESS_ANISOTROPY, P.TextureUV));
    Rough = A.x * A.y > PT_EPSILON;
}

PT_DEV bool Metal_Evaluate(const dscene& S, const bsdf_parameters& P, pt3 In, pt3 Out, pt4& T, pt4& Pr)
{
    pt4 Base, Spec; pt2 A; bool Rough;
    Metal_GetParameters(S, P, Base, Spec, A, Rough);
    if (In.z <= 0.0f || Out.z <= 0.0f || !Rough) return false;
    pt3 Half = SafeNormalize(In + Out);
    float Gm = GGXSmithG1(In, A);
    float D = GGXDistribution(Half, A);
    Pr = v4s(Gm * D / (4 * In.z));
    float Gs = GGXSmithG1(Out, A);
    pt4 F = SchlickFresnelMetal(Base, Spec, dot(In, Half));
    T = Pr * Gs * F;
    return true;
}

PT_DEV bool Metal_Sample(const dscene& S, rng& G, const bsdf_parameters& P, pt3 In, pt3& Out, pt4& T, pt4& Pr)
{
    pt4 Base, Spec; pt2 A; bool Rough;
    Metal_GetParameters(S, P, Base, Spec, A, Rough);
    if (In.z <= 0.0f) return false;
    float U1 = G.R01();
    float U2 = G.R01();
    pt3 N = GGXVisibleNormal(In, A, U1, U2);
    float CosThetaIn = pt_min(dot(N, In), 1.0f);
    Out = 2 * CosThetaIn * N - In;
    if (Out.z <= 0.0f) return false;
    Pr = v4s(1.0f);
    if (Rough) {
        float Gm = GGXSmithG1(In, A);
        float D = GGXDistribution(N, A);
        Pr = Pr * v4s(Gm * D / (4 * In.z));
    }
    float Gs = GGXSmithG1(Out, A);
    pt4 F = SchlickFresnelMetal(Base, Spec, CosThetaIn);
    T = Pr * Gs * F;
    return true;
}

PT_DEV void Translucent_GetParameters(const dscene& S, const bsdf_parameters& P, pt3 In, pt4& RelIOR, pt2& A, bool& Rough)
{
    pt4 Interior = CauchyEmpiricalIOR(MFloat(S, P.MaterialIndex, PT_BASIC_TRANSLUCENT_IOR),
                                      MFloat(S, P.MaterialIndex, PT_BASIC_TRANSLUCENT_ABBE_NUMBER), P.Lambda);
    if (In.z < 0.0f) RelIOR = Interior / P.ExteriorIOR;
    else RelIOR = P.ExteriorIOR / Interior;
    A = GGXRoughnessAlpha(MaterialTexturableValue(S, P.MaterialIndex, PT_BASIC_TRANSLUCENT_ROUGHNESS, P.TextureUV),
                          MaterialTexturableValue(S, P.MaterialIndex, PT_BASIC_TRANSLUCENT_ROUGHNESS_ANISOTROPY, P.TextureUV));
    Rough = A.x * A.y > PT_EPSILON;
}

PT_DEV bool Translucent_Evaluate(const dscene& S, const bsdf_parameters& P, pt3 In, pt3 Out, pt4& T, pt4& Pr)
{
    pt4 RelIOR; pt2 A; bool Rough;
    Translucent_GetParameters(S, P, In, RelIOR, A, Rough);
    if (!Rough) { Pr = v4s(0.0f); T = v4s(0.0f); return true; }
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

PT_DEV bool Translucent_Sample(const dscene& S, rng& G, const bsdf_parameters& P, pt3 In, pt3& Out, pt4& T, pt4& Pr)
{
    pt4 RelIOR; pt2 A; bool Rough;
    Translucent_GetParameters(S, P, In, RelIOR, A, Rough);
    float U1 = G.R01();
    float U2 = G.R01();
    pt3 N = GGXVisibleNormal(In * pt_sign(In.z), A, U1, U2);
    float CosThetaIn = pt_clamp(dot(N, In), -1.0f, +1.0f);
    float CosThetaRefracted = ComputeCosThetaRefracted(RelIOR.x, CosThetaIn);
    float Reflectance = FresnelDielectric(RelIOR.x, CosThetaIn, CosThetaRefracted);
    if (G.R01() < Reflectance) {
        Out = 2 * CosThetaIn * N - In;
        if (Out.z * In.z <= 0) return false;
        pt4 F = FresnelDielectric(RelIOR, v4s(CosThetaIn));
        Pr = F;
        if (Rough) {
            float Gm = GGXSmithG1(In, A);
            float D = GGXDistribution(N, A);
            Pr = Pr * (Gm * D / (4 * pt_abs(In.z)));
        }
        float Gs = GGXSmithG1(Out, A);
        T = Pr * Gs;
        return true;
    }
    Out = (CosThetaRefracted + RelIOR.x * CosThetaIn) * N - RelIOR.x * In;
    if (Out.z * In.z >= 0) return false;
    if (Rough) {
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

PT_DEV void LoadMedium(const dscene& S, uint32_t M, pt4 Lambda, medium& Md)
{
    Md.IOR = v4s(1.0f); Md.AbsorptionRate = v4s(0.0f); Md.ScatteringRate = v4s(0.0f); Md.ScatteringAnisotropy = 0.0f;
    if (MUint(S, M, 0) != PT_MATERIAL_TYPE_BASIC_TRANSLUCENT) return;
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
        LoadMedium(S, S.shapes[ShapeIndex].MaterialIndex, Lambda, Md);
        Md.Priority = ShapeIndex;
    }
    return Md;
}

PT_DEV bool HasDirac(const dscene& S, const bsdf_parameters& P, uint32_t Type)
{
    if (Type == PT_MATERIAL_TYPE_BASIC_METAL)
        return MaterialTexturableValue(S, P.MaterialIndex, PT_BASIC_METAL_ROUGHNESS, P.TextureUV) < 1e-3f;
    if (Type == PT_MATERIAL_TYPE_BASIC_TRANSLUCENT)
        return MaterialTexturableValue(S, P.MaterialIndex, PT_BASIC_TRANSLUCENT_ROUGHNESS, P.TextureUV) < 1e-3f;
    return false;
}

// SampleSurfaceIntegrand (basic_scatter.glsl:68-109)
PT_DEV bool SampleSurfaceIntegrand(const dscene& S, rng& G, pt3 Nrm, pt3 TX, pt3 TY, const bsdf_parameters& P, pt3 Out,
                                   pt3& In, pt4& Throughput, pt4& Probability)
{
    uint32_t Type = MUint(S, P.MaterialIndex, 0);
    float LightProbability = HasDirac(S, P, Type) ? 0.0f : S.g.SkyboxSamplingProbability;
    pt4 MaterialPDF = v4s(0.0f);
    pt3 SMD = v3(S.g.SkyboxMeanDirection[0], S.g.SkyboxMeanDirection[1], S.g.SkyboxMeanDirection[2]);
    pt3 Mu = v3(dot(SMD, TX), dot(SMD, TY), dot(SMD, Nrm));
    bool ok;
    if (G.R01() < LightProbability) {
        In = RandomVonMisesFisher(G, S.g.SkyboxConcentration, Mu);
        if (In.z < 0.0f) return false;
        // MaterialEvaluateBSDF(Parameters, Out, In, ...)
        if (Type == PT_MATERIAL_TYPE_BASIC_DIFFUSE) ok = Diffuse_Evaluate(S, P, Out, Throughput, MaterialPDF);
        else if (Type == PT_MATERIAL_TYPE_BASIC_METAL) ok = Metal_Evaluate(S, P, Out, In, Throughput, MaterialPDF);
        else if (Type == PT_MATERIAL_TYPE_BASIC_TRANSLUCENT) ok = Translucent_Evaluate(S, P, Out, In, Throughput, MaterialPDF);
        else ok = false;
        if (!ok) return false;
    } else {
        // MaterialSampleBSDF(Parameters, Out, In, ...)
        if (Type == PT_MATERIAL_TYPE_BASIC_DIFFUSE) {
            In = SafeNormalize(RandomDirection(G) + v3(0, 0, 1));
            ok = Diffuse_Evaluate(S, P, Out, Throughput, MaterialPDF);
        } else if (Type == PT_MATERIAL_TYPE_BASIC_METAL) {
            ok = Metal_Sample(S, G, P, Out, In, Throughput, MaterialPDF);
        } else if (Type == PT_MATERIAL_TYPE_BASIC_TRANSLUCENT) {
            ok = Translucent_Sample(S, G, P, Out, In, Throughput, MaterialPDF);
        } else {
            ok = false;
        }
        if (!ok) return false;
    }
    pt4 SkyboxPDF = v4s(VonMisesFisherPDF(S.g.SkyboxConcentration, Mu, In));
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

PT_DEV void StorePathVertex(const dslots& L, uint32_t s, const path& P)
{
    L.thr[s] = make_float4(P.Throughput.x, P.Throughput.y, P.Throughput.z, P.Throughput.w);
    L.prob[s] = make_float4(P.Probability.x, P.Probability.y, P.Probability.z, P.Probability.w);
    L.smp[s] = make_float4(P.Sample.x, P.Sample.y, P.Sample.z, P.Lambda0);
    L.act[s] = make_uint2((P.Active[1] << 16) | P.Active[0], (P.Active[3] << 16) | P.Active[2]);
}

PT_DEV void StoreRay(const dslots& L, uint32_t s, pt3 O, pt3 V)
{
    L.ray[s] = make_float4(O.x, O.y, O.z, __uint_as_float(PackUnitVector(V)));
}

// GenerateNewPath (basic_scatter.glsl:7-42) + GenerateCameraRay (scene.glsl.inc:613-655)
PT_DEV void GenerateNewPath(const dscene& S, const dslots& L, const dframe& F, const dparams& Pm, rng& G, uint32_t s,
                            uint32_t x, uint32_t y)
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
    StoreRay(L, s, mat4_mul_point(To, O), mat4_mul_vector(To, V));
    path P;
    P.Lambda0 = G.R01();
    P.Throughput = v4s(1.0f);
    P.Probability = v4s(1.0f);
    P.Sample = v3s(0.0f);
    P.Active[0] = P.Active[1] = P.Active[2] = P.Active[3] = SHAPE_INDEX_NONE;
    StorePathVertex(L, s, P);
}

// Scatter (basic_scatter.glsl:114-310).  Returns true if an extension ray was
// produced (written to O, V).
PT_DEV bool Scatter(const dscene& S, rng& G, float PTP, path& Path, pt3& O, pt3& V, uint32_t HitShape,
                    uint32_t HitMaterial, float HitTime, uint32_t PN, uint32_t PT, pt2 UV)
{
    float L0 = Path.Lambda0;
    pt4 Lambda = v4(pt_mix(PT_CIE_LAMBDA_MIN, PT_CIE_LAMBDA_MAX, L0),
                    pt_mix(PT_CIE_LAMBDA_MIN, PT_CIE_LAMBDA_MAX, pt_fract(L0 + 0.25f)),
                    pt_mix(PT_CIE_LAMBDA_MIN, PT_CIE_LAMBDA_MAX, pt_fract(L0 + 0.50f)),
                    pt_mix(PT_CIE_LAMBDA_MIN, PT_CIE_LAMBDA_MAX, pt_fract(L0 + 0.75f)));

    uint32_t Active = SHAPE_INDEX_NONE;
    for (int I = 0; I < 4; I++) Active = pt_umin(Active, Path.Active[I]);

    medium Md = ResolveMedium(S, Active, Lambda);
    Path.Throughput = Path.Throughput * vexp(-Md.AbsorptionRate * HitTime);

    float ScatteringTime = PT_HIT_TIME_LIMIT;
    if (Md.ScatteringRate.x > 0.0f) ScatteringTime = -pt_log(G.R01()) / Md.ScatteringRate.x;

    if (HitTime >= ScatteringTime) {
        if (ScatteringTime < PT_HIT_TIME_LIMIT) {
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
            pt4 Emission = SampleSkyboxRadiance(S, V, Lambda);
            float ClusterPDF = Path.Probability.x + Path.Probability.y + Path.Probability.z + Path.Probability.w;
            pt4 E = Emission * Path.Throughput;
            pt3 XYZ = SampleStandardObserver(Lambda.x) * E.x + SampleStandardObserver(Lambda.y) * E.y +
                      SampleStandardObserver(Lambda.z) * E.z + SampleStandardObserver(Lambda.w) * E.w;
            Path.Sample = Path.Sample + XYZ / ClusterPDF;
            Path.Probability = v4s(0.0f);
        }
        return max4(Path.Probability) > PT_EPSILON;
    }

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
            uint32_t Ext = SHAPE_INDEX_NONE;
            for (int I = 0; I < 4; I++) {
                if (Path.Active[I] == Active) continue;
                Ext = pt_umin(Ext, Path.Active[I]);
            }
            ExteriorIOR = ResolveMedium(S, Ext, Lambda).IOR;
        }
    }

    pt3 In;
    if (IsReal) {
        bsdf_parameters P;
        P.MaterialIndex = HitMaterial;
        P.TextureUV = UV;
        P.Lambda = Lambda;
        P.ExteriorIOR = ExteriorIOR;
        pt4 T, Pr;
        if (!SampleSurfaceIntegrand(S, G, Nrm, TX, TY, P, Out, In, T, Pr)) return false;
        float Scale = 1.0f / pt_max(PT_EPSILON, max4(Pr));
        Path.Throughput = Path.Throughput * (T * Scale);
        Path.Probability = Path.Probability * (Pr * Scale);
    } else {
        In = -Out;
    }

    if (In.z * Out.z < 0) {
        if (Out.z > 0) {
            for (int I = 0; I < 4; I++)
                if (Path.Active[I] == SHAPE_INDEX_NONE) { Path.Active[I] = HitShape; break; }
        } else {
            for (int I = 0; I < 4; I++)
                if (Path.Active[I] == HitShape) { Path.Active[I] = SHAPE_INDEX_NONE; break; }
        }
    }

    if (G.R01() < PTP) return false;
    Path.Probability = Path.Probability * (1.0f - PTP);

    V = In.x * TX + In.y * TY + In.z * Nrm;
    O = Position + 1e-3f * V;
    return max4(Path.Probability) > PT_EPSILON;
}

// --- kernels -------------------------------------------------------------------

__global__ __launch_bounds__(256) void raygen_kernel(dscene S, dslots L, dframe F, dparams Pm)
{
    uint32_t s = blockIdx.x * 256 + threadIdx.x;
    if (s >= L.n) return;
    uint32_t x, y;
    if (!SlotPixel(F, s, x, y)) return;
    rng G;
    G.State = pt_seed(x, y, Pm.seed);
    GenerateNewPath(S, L, F, Pm, G, s, x, y);
    F.accum[(size_t)y * F.width + x] = make_float4(0, 0, 0, 0);
}

template <bool SPILL>
__global__ __launch_bounds__(256) void extend_kernel(dscene S, dslots L, dframe F)
{
    __shared__ uint32_t smem[PT_LDS_STACK * 256];
    uint32_t s = blockIdx.x * 256 + threadIdx.x;
    if (s >= L.n) return;
    uint32_t x, y;
    if (!SlotPixel(F, s, x, y)) return;
    float4 r = L.ray[s];
    pt3 O = v3(r.x, r.y, r.z);
    pt3 V = UnpackUnitVector(__float_as_uint(r.w));
    tstack<SPILL> st;
    st.lds = &smem[threadIdx.x];
    st.spill = L.spill + s;
    st.stride = L.n;
    float4 rec;
    float2 uv;
    bool isHit;
    TraceRecord<SPILL>(S, O, V, PT_HIT_TIME_LIMIT, st, rec, uv, isHit);
    if (isHit) {
        L.hit[s] = rec;
        L.uv[s] = uv;
    } else {
        reinterpret_cast<uint32_t*>(&L.hit[s])[1] = 0xFFFFFFFFu;
    }
}

__global__ __launch_bounds__(256) void shade_kernel(dscene S, dslots L, dframe F, dparams Pm)
{
    uint32_t s = blockIdx.x * 256 + threadIdx.x;
    if (s >= L.n) return;
    uint32_t x, y;
    if (!SlotPixel(F, s, x, y)) return;
    rng G;
    G.State = pt_seed(x, y, Pm.seed);

    // LoadPath (basic.glsl.inc:159-198)
    path P;
    float4 thr = L.thr[s], prob = L.prob[s], smp = L.smp[s];
    uint2 act = L.act[s];
    P.Throughput = v4(thr.x, thr.y, thr.z, thr.w);
    P.Probability = v4(prob.x, prob.y, prob.z, prob.w);
    P.Sample = v3(smp.x, smp.y, smp.z);
    P.Lambda0 = smp.w;
    P.Active[0] = act.x & 0xFFFF; P.Active[1] = act.x >> 16;
    P.Active[2] = act.y & 0xFFFF; P.Active[3] = act.y >> 16;
    for (int I = 0; I < 4; I++)
        if (P.Active[I] == 0xFFFF) P.Active[I] = SHAPE_INDEX_NONE;

    // LoadTraceResult (basic.glsl.inc:99-131)
    float4 r = L.ray[s];
    pt3 O = v3(r.x, r.y, r.z);
    pt3 V = UnpackUnitVector(__float_as_uint(r.w));
    float4 h = L.hit[s];
    uint32_t sm = __float_as_uint(h.y);
    uint32_t HitShape = SHAPE_INDEX_NONE, HitMaterial = 0;
    float HitTime = PT_HIT_TIME_LIMIT;
    uint32_t PN = 0, PTg = 0;
    pt2 UV = v2(0, 0);
    if (sm != 0xFFFFFFFFu) {
        HitShape = sm >> 16;
        HitMaterial = sm & 0xFFFF;
        HitTime = h.x;
        PN = __float_as_uint(h.z);
        PTg = __float_as_uint(h.w);
        float2 uv = L.uv[s];
        UV = v2(uv.x, uv.y);
    }

    if (Scatter(S, G, Pm.termination_probability, P, O, V, HitShape, HitMaterial, HitTime, PN, PTg, UV)) {
        StoreRay(L, s, O, V);
        StorePathVertex(L, s, P);
    } else {
        float4* A = &F.accum[(size_t)y * F.width + x];
        float4 Val = make_float4(P.Sample.x, P.Sample.y, P.Sample.z, 1.0f);
        if (Pm.render_flags & PT_RENDER_FLAG_ACCUMULATE) {
            float4 Old = *A;
            Val.x = Val.x + Old.x; Val.y = Val.y + Old.y; Val.z = Val.z + Old.z; Val.w = Val.w + Old.w;
        }
        *A = Val;
        GenerateNewPath(S, L, F, Pm, G, s, x, y);
    }
}

template <bool SPILL>
__global__ __launch_bounds__(256) void trace_rays_kernel(dscene S, uint32_t n, const float* origins,
                                                         const uint32_t* vel, const float* dur, float4* out_rec,
                                                         float2* out_uv, uint32_t* spill)
{
    __shared__ uint32_t smem[PT_LDS_STACK * 256];
    uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    pt3 O = v3(origins[3 * i], origins[3 * i + 1], origins[3 * i + 2]);
    pt3 V = UnpackUnitVector(vel[i]);
    tstack<SPILL> st;
    st.lds = &smem[threadIdx.x];
    st.spill = spill + i;
    st.stride = n;
    float4 rec;
    float2 uv;
    bool isHit;
    TraceRecord<SPILL>(S, O, V, dur[i], st, rec, uv, isHit);
    if (!isHit) {
        rec = make_float4(0, __uint_as_float(0xFFFFFFFFu), 0, 0);
        uv = make_float2(0, 0);
    }
    out_rec[i] = rec;
    out_uv[i] = uv;
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

hipError_t pt_launch_extend(const ptd::dscene& S, const ptd::dslots& L, const ptd::dframe& F, bool spill,
                            hipStream_t st)
{
    if (L.n == 0) return hipSuccess;
    if (spill) hipLaunchKernelGGL(ptd::extend_kernel<true>, dim3(Blocks(L.n)), dim3(256), 0, st, S, L, F);
    else hipLaunchKernelGGL(ptd::extend_kernel<false>, dim3(Blocks(L.n)), dim3(256), 0, st, S, L, F);
    return hipGetLastError();
}

hipError_t pt_launch_shade(const ptd::dscene& S, const ptd::dslots& L, const ptd::dframe& F, const ptd::dparams& P,
                           hipStream_t st)
{
    if (L.n == 0) return hipSuccess;
    hipLaunchKernelGGL(ptd::shade_kernel, dim3(Blocks(L.n)), dim3(256), 0, st, S, L, F, P);
    return hipGetLastError();
}

hipError_t pt_launch_trace_rays(const ptd::dscene& S, uint32_t n, const float* origins, const uint32_t* vel,
                                const float* dur, float4* rec, float2* uv, uint32_t* spill, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    if (spill) hipLaunchKernelGGL(ptd::trace_rays_kernel<true>, dim3(Blocks(n)), dim3(256), 0, st, S, n, origins, vel, dur, rec, uv, spill);
    else hipLaunchKernelGGL(ptd::trace_rays_kernel<false>, dim3(Blocks(n)), dim3(256), 0, st, S, n, origins, vel, dur, rec, uv, spill);
    return hipGetLastError();
}
