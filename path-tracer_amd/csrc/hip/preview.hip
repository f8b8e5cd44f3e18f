// preview.hip — RenderPreview (src/application/preview_render.cpp:118-181,
// preview_render.glsl:96-178): one primary ray per pixel through the same
// Trace() as the extend kernel (traverse.hpp), coloured by one of the seven
// preview modes (base colour, shaded, normal, material / primitive ID, mesh /
// scene BVH complexity), with the selected-shape tint, the mouse pick query,
// and per-pixel primary-hit AOVs.
//
// The fragment shader's interpolated ScreenXY is the pixel centre of a
// RenderSizeX x RenderSizeY viewport.  Pixels are mapped in 16x16 tiles
// (256-thread blocks) so a wave traces a 16x4 coherent block.
#include "pt_device.hpp"
#include "traverse.hpp"
#include "kernels.hpp"
#include "../../../include/pt_cie.h"

namespace ptd {

__constant__ float kD65[PT_CIE_D65_COUNT] = {PT_CIE_D65_VALUES};

__constant__ float kPreviewColors[20][3] = {                           // preview_render.glsl:16-38
    {0.902f, 0.098f, 0.294f}, {0.235f, 0.706f, 0.294f}, {1.000f, 0.882f, 0.098f}, {0.263f, 0.388f, 0.847f},
    {0.961f, 0.510f, 0.192f}, {0.569f, 0.118f, 0.706f}, {0.275f, 0.941f, 0.941f}, {0.941f, 0.196f, 0.902f},
    {0.737f, 0.965f, 0.047f}, {0.980f, 0.745f, 0.745f}, {0.000f, 0.502f, 0.502f}, {0.902f, 0.745f, 1.000f},
    {0.604f, 0.388f, 0.141f}, {1.000f, 0.980f, 0.784f}, {0.502f, 0.000f, 0.000f}, {0.667f, 1.000f, 0.765f},
    {0.502f, 0.502f, 0.000f}, {1.000f, 0.847f, 0.694f}, {0.000f, 0.000f, 0.459f}, {0.502f, 0.502f, 0.502f}};

PT_DEV float SampleIlluminantD65(float NormalizedLambda)              // spectrum.glsl.inc:159-164
{
    float Offset = NormalizedLambda * 470;
    int Index = (int)Offset;
    Index = Index < 0 ? 0 : (Index > 469 ? 469 : Index);
    return pt_mix(kD65[Index], kD65[Index + 1], Offset - (float)Index);
}

// ObserveParametricSpectrumUnderD65 (spectrum.glsl.inc:194-208), 16 samples.
// Everything but the spectrum itself -- each sample's wavelength, D65 weight
// and CIE observer value -- depends on the sample index only, so
// observe_table_kernel evaluates the 16 samples once per preview context and
// every observation reads them (uniform index: scalar loads): the same
// functions on the same operands give the same bits, and the 7 exponentials
// of each observer value leave the per-pixel path.
constexpr int OBSERVE_SAMPLES = 16;
struct observe_table {
    float D[OBSERVE_SAMPLES], Lambda[OBSERVE_SAMPLES];
    pt3 Obs[OBSERVE_SAMPLES];
};

static_assert(sizeof(observe_table) == PT_OBSERVE_TABLE_FLOATS * 4, "observe_table size");

__global__ void observe_table_kernel(observe_table* T)
{
    const int I = (int)threadIdx.x;
    if (I >= OBSERVE_SAMPLES) return;
    float NormalizedLambda = (float)I / (float)(OBSERVE_SAMPLES - 1);
    T->D[I] = SampleIlluminantD65(NormalizedLambda) / PT_CIE_D65_NORMALIZATION;
    T->Lambda[I] = pt_mix(PT_CIE_LAMBDA_MIN, PT_CIE_LAMBDA_MAX, NormalizedLambda);
    T->Obs[I] = SampleStandardObserver(T->Lambda[I]);
}

PT_DEV pt3 ObserveUnderD65(const observe_table& T, pt4 BetaAndIntensity)
{
    const float DeltaLambda = (PT_CIE_LAMBDA_MAX - PT_CIE_LAMBDA_MIN) / OBSERVE_SAMPLES;
    pt3 Color = v3s(0);
    pt3 Beta = v3(BetaAndIntensity.x, BetaAndIntensity.y, BetaAndIntensity.z);
    for (int I = 0; I < OBSERVE_SAMPLES; I++) {
        float Sp = BetaAndIntensity.w * SampleParametricSpectrum(Beta, T.Lambda[I]);
        Color = Color + Sp * T.D[I] * T.Obs[I] * DeltaLambda;
    }
    return Color;
}

PT_DEV pt3 ObserveUnderD65(const observe_table& T, pt3 Beta) { return ObserveUnderD65(T, v4(Beta.x, Beta.y, Beta.z, 1)); }

// MaterialBaseColor (scene.glsl.inc:254-274,696-701 + *_BaseColor)
PT_DEV pt3 MaterialBaseColor(const dscene& S, const observe_table& Tb, uint32_t M, pt2 UV)
{
    uint32_t Type = MUint(S, M, 0);
    uint32_t A;
    if (Type == PT_MATERIAL_TYPE_BASIC_DIFFUSE) A = PT_BASIC_DIFFUSE_BASE_SPECTRUM;
    else if (Type == PT_MATERIAL_TYPE_BASIC_METAL) A = PT_BASIC_METAL_BASE_SPECTRUM;
    else if (Type == PT_MATERIAL_TYPE_BASIC_TRANSLUCENT) return ObserveUnderD65(Tb, MVec3(S, M, PT_BASIC_TRANSLUCENT_TRANSMISSION_SPECTRUM));
    else return v3s(0);
    pt3 Color = ObserveUnderD65(Tb, MVec3(S, M, A));
    uint32_t TextureIndex = MUint(S, M, A + 3);
    if (TextureIndex != TEXTURE_INDEX_NONE) {
        pt4 T = SampleTexture(S, TextureIndex, UV);
        Color = Color * ObserveUnderD65(Tb, v3(T.x, T.y, T.z));
    }
    return Color;
}

PT_DEV pt3 XYZToSRGB(pt3 V)                                            // CIE_XYZ_TO_SRGB * V (spectrum.glsl.inc:50-55)
{
    return v3(+3.2406f * V.x + -1.5372f * V.y + -0.4986f * V.z,
              -0.9689f * V.x + +1.8758f * V.y + +0.0415f * V.z,
              +0.0557f * V.x + -0.2040f * V.y + +1.0570f * V.z);
}

struct preview_args {
    pt_packed_transform cam;
    uint32_t mode;
    float brightness;
    uint32_t selected;
    uint32_t w, h, mx, my;
    uint32_t tiles_x;
};

// The pixel's primary ray (preview_render.glsl:98-106); also the ray source
// LaneStep reloads after a BLAS.
struct ray_source_preview {
    const preview_args* P;
    PT_DEV bool pixel(uint32_t i, uint32_t& x, uint32_t& y) const
    {
        uint32_t t = i >> 8, l = i & 255u;
        uint32_t ty = t / P->tiles_x;
        x = (t - ty * P->tiles_x) * 16 + (l & 15u);
        y = ty * 16 + (l >> 4);
        return x < P->w && y < P->h;
    }
    PT_DEV bool load(uint32_t i, pt3& O, pt3& V, float& D) const
    {
        uint32_t x, y;
        pixel(i, x, y);
        float SX = ((float)x + 0.5f) / (float)P->w, SY = ((float)y + 0.5f) / (float)P->h;
        float AspectRatio = (float)P->w / (float)P->h;
        pt3 V0 = normalize(v3((SX - 0.5f) * AspectRatio, 0.5f - SY, -1.0f));
        O = mat4_mul_point(P->cam.To, v3s(0));          // TransformRay (common.glsl.inc:60-67)
        V = mat4_mul_vector(P->cam.To, V0);
        D = PT_HIT_TIME_LIMIT;
        return true;
    }
};

template <int CAP>
__global__ __launch_bounds__(256) void preview_kernel(dscene S, preview_args P, uint32_t* spill, uint32_t spill_stride,
                                                      float4* __restrict__ out, pt_preview_aov* __restrict__ aov,
                                                      uint32_t* __restrict__ query,
                                                      const observe_table* __restrict__ observe)
{
    __shared__ uint32_t smem[CAP * 256];
    const observe_table& Tb = *observe;
    uint32_t i = blockIdx.x * 256 + threadIdx.x;
    ray_source_preview src{&P};
    uint32_t x, y;
    if (!src.pixel(i, x, y)) return;
    tstack<true, CAP> st;
    st.lds = &smem[threadIdx.x];
    st.spill = spill ? spill + i : nullptr;
    st.stride = spill_stride;

    pt3 O, V;
    float D;
    src.load(i, O, V, D);
    lane_state Ln;
    LaneBegin(S, Ln, O, V, D);
    complexity_stats cx;
    if (S.g.ShapeCount != 0)
        while (!LaneStep<true, CAP>(S, Ln, st, src, i, cx)) {}

    bool Miss = Ln.Shape == SHAPE_INDEX_NONE;
    uint32_t Material = 0;
    pt3 N = v3s(0), TX;
    pt2 UV = v2(0, 0);
    if (!Miss) HitAttributes(S, Ln.Shape, Ln.Prim, Ln.C, Material, N, TX, UV);

    pt3 Color = v3s(0);
    switch (P.mode) {                                                  // preview_render.glsl:110-162
    case PT_PREVIEW_RENDER_MODE_BASE_COLOR:
    case PT_PREVIEW_RENDER_MODE_BASE_COLOR_SHADED:
        if (Miss) {
            Color = XYZToSRGB(ObserveUnderD65(Tb, SampleSkyboxSpectrum(S, V)));
        } else {
            Color = XYZToSRGB(MaterialBaseColor(S, Tb, Material, UV));
            if (P.mode == PT_PREVIEW_RENDER_MODE_BASE_COLOR_SHADED) Color = Color * dot(N, -V);
        }
        break;
    case PT_PREVIEW_RENDER_MODE_NORMAL:
        Color = Miss ? 0.5f * (v3s(1) - V) : 0.5f * (N + v3s(1));
        break;
    case PT_PREVIEW_RENDER_MODE_MATERIAL_INDEX:
        if (!Miss) Color = v3(kPreviewColors[Material % 20][0], kPreviewColors[Material % 20][1], kPreviewColors[Material % 20][2]);
        break;
    case PT_PREVIEW_RENDER_MODE_PRIMITIVE_INDEX:
        if (!Miss) Color = v3(kPreviewColors[Ln.Prim % 20][0], kPreviewColors[Ln.Prim % 20][1], kPreviewColors[Ln.Prim % 20][2]);
        break;
    case PT_PREVIEW_RENDER_MODE_MESH_COMPLEXITY:
        Color = v3(0, 1, 0) * (float)cx.mesh / 256.0f;
        break;
    case PT_PREVIEW_RENDER_MODE_SCENE_COMPLEXITY:
        Color = v3(0, 1, 0) * (float)cx.scene / 256.0f;
        break;
    }
    if (Ln.Shape == P.selected) Color = Color * v3(1.0f, 0.5f, 0.5f);
    Color = Color * P.brightness;
    if (x == P.mx && y == P.my) *query = Ln.Shape;

    size_t p = (size_t)y * P.w + x;
    out[p] = make_float4(Color.x, Color.y, Color.z, 1.0f);
    pt_preview_aov A;
    A.time = Miss ? 0.0f : Ln.Time;
    A.shape_index = Ln.Shape;
    A.material_index = Material;
    A.primitive_index = Miss ? 0u : Ln.Prim;
    A.mesh_complexity = cx.mesh;
    A.scene_complexity = cx.scene;
    A.normal[0] = N.x; A.normal[1] = N.y; A.normal[2] = N.z;
    A.u = UV.x; A.v = UV.y;
    A.reserved = 0;
    aov[p] = A;
}

}  // namespace ptd

hipError_t pt_launch_observe_table(float* table, hipStream_t st)
{
    hipLaunchKernelGGL(ptd::observe_table_kernel, dim3(1), dim3(64), 0, st,
                       reinterpret_cast<ptd::observe_table*>(table));
    return hipGetLastError();
}

hipError_t pt_launch_preview(const ptd::dscene& S, const pt_preview_parameters* p, uint32_t* spill, float4* out,
                             pt_preview_aov* aov, uint32_t* query, const float* observe_table, hipStream_t st)
{
    ptd::preview_args P;
    P.cam = p->CameraTransform;
    P.mode = p->RenderMode;
    P.brightness = p->Brightness;
    P.selected = p->SelectedShapeIndex;
    P.w = p->RenderSizeX;
    P.h = p->RenderSizeY;
    P.mx = p->MouseX;
    P.my = p->MouseY;
    P.tiles_x = (P.w + 15) / 16;
    uint32_t tiles = P.tiles_x * ((P.h + 15) / 16);
    if (tiles == 0) return hipSuccess;
    hipLaunchKernelGGL(ptd::preview_kernel<20>, dim3(tiles), dim3(256), 0, st, S, P, spill, tiles * 256, out, aov, query,
                       reinterpret_cast<const ptd::observe_table*>(observe_table));
    return hipGetLastError();
}

uint32_t pt_preview_stack_cap() { return 20; }
