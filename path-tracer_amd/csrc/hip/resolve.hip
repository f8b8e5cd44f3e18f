// resolve.hip — RenderSampleBuffer (src/integrator/integrator.cpp:105-159,
// resolve.glsl:60-130) as a compute kernel: CIE XYZ sum / count -> linear
// sRGB (CIE_XYZ_TO_SRGB, spectrum.glsl.inc:50-55) x Brightness -> tone map
// (Clamp / Reinhard / Hable / ACES).  Writes the fragment shader's OutColor
// (rgba32f, alpha 1) and its encoding in a B8G8R8A8_SRGB swapchain image
// (vulkan.cpp:1407; stored here as R,G,B,A bytes).
//
// The reference samples the accumulator with a texture fetch at the pixel
// centre of a same-sized viewport, i.e. the texel itself; this kernel reads
// the texel directly.  Arithmetic follows include/pt_fp.h (IEEE f32, no
// contraction, left-to-right matrix products).  The 8-bit encoding uses the
// sRGB transfer function with pt_exp/pt_log for the 1/2.4 power and rounds
// to nearest (the swapchain's hardware conversion is driver-defined).
//
// HBM-bound: 16 B read + 16 B + 4 B written per pixel.
#include "pt_device.hpp"
#include "kernels.hpp"

namespace ptd {

struct resolve_args {
    float brightness;
    uint32_t mode;
    float white;
};

PT_DEV pt3 Mat3MulRows(const float m[9], pt3 v)   // GLSL mat3 (column-major) * vec3
{
    return v3(m[0] * v.x + m[3] * v.y + m[6] * v.z,
              m[1] * v.x + m[4] * v.y + m[7] * v.z,
              m[2] * v.x + m[5] * v.y + m[8] * v.z);
}

PT_DEV pt3 HablePartial(pt3 X)                     // resolve.glsl:80-85
{
    const float A = 0.15f, B = 0.50f, C = 0.10f, D = 0.20f, E = 0.02f, F = 0.30f;
    pt3 Num = X * (A * X + v3s(C * B)) + v3s(D * E);
    pt3 Den = X * (A * X + v3s(B)) + v3s(D * F);
    return Num / Den - v3s(E / F);
}

PT_DEV pt3 ResolvePixel(float4 Value, const resolve_args& P)
{
    // resolve.glsl:112-128
    const float XYZ_TO_SRGB[9] = {+3.2406f, -0.9689f, +0.0557f, -1.5372f, +1.8758f, -0.2040f,
                                  -0.4986f, +0.0415f, +1.0570f};
    pt3 Color = v3s(0.0f);
    if (Value.w > 0) Color = Mat3MulRows(XYZ_TO_SRGB, (P.brightness * v3(Value.x, Value.y, Value.z)) / Value.w);
    if (P.mode == PT_TONE_MAPPING_CLAMP) {
        Color = v3(pt_clamp(Color.x, 0, 1), pt_clamp(Color.y, 0, 1), pt_clamp(Color.z, 0, 1));
    } else if (P.mode == PT_TONE_MAPPING_REINHARD) {             // resolve.glsl:66-73
        float OldL = Color.x * 0.2126f + Color.y * 0.7152f + Color.z * 0.0722f;
        float MaxL = P.white;
        float N = OldL * (1.0f + (OldL / (MaxL * MaxL)));
        float NewL = N / (1.0f + OldL);
        Color = Color * NewL / OldL;
    } else if (P.mode == PT_TONE_MAPPING_HABLE) {                // resolve.glsl:87-94
        pt3 Current = HablePartial(Color * 2.0f);
        pt3 WhiteScale = v3s(1.0f) / HablePartial(v3s(11.2f));
        Color = Current * WhiteScale;
    } else if (P.mode == PT_TONE_MAPPING_ACES) {                 // resolve.glsl:96-110
        const float IN[9] = {0.59719f, 0.07600f, 0.02840f, 0.35458f, 0.90834f, 0.13383f,
                             0.04823f, 0.01566f, 0.83777f};
        const float OUT[9] = {1.60475f, -0.10208f, -0.00327f, -0.53108f, 1.10813f, -0.07276f,
                              -0.07367f, -0.00605f, 1.07602f};
        pt3 V = Mat3MulRows(IN, Color);
        pt3 A = V * (V + v3s(0.0245786f)) - v3s(0.000090537f);
        pt3 B = V * (0.983729f * V + v3s(0.4329510f)) + v3s(0.238081f);
        Color = Mat3MulRows(OUT, A / B);
    }
    return Color;
}

PT_DEV uint32_t EncodeSRGB8(float c)
{
    c = pt_clamp(c, 0.0f, 1.0f);               // UNORM store clamps; NaN -> 0
    float e = c <= 0.0031308f ? 12.92f * c : 1.055f * pt_exp(pt_log(c) * (1.0f / 2.4f)) - 0.055f;
    float q = pt_clamp(e, 0.0f, 1.0f) * 255.0f;
    return (uint32_t)(q + 0.5f);
}

__global__ __launch_bounds__(256) void resolve_kernel(const float4* __restrict__ accum, uint32_t n, resolve_args P,
                                                      float4* __restrict__ out, uint32_t* __restrict__ out8)
{
    uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    pt3 C = ResolvePixel(accum[i], P);
    out[i] = make_float4(C.x, C.y, C.z, 1.0f);
    out8[i] = EncodeSRGB8(C.x) | (EncodeSRGB8(C.y) << 8) | (EncodeSRGB8(C.z) << 16) | (255u << 24);
}

}  // namespace ptd

hipError_t pt_launch_resolve(const float4* accum, uint32_t n, float brightness, uint32_t mode, float white, float4* out,
                             uint32_t* out8, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    ptd::resolve_args P{brightness, mode, white};
    hipLaunchKernelGGL(ptd::resolve_kernel, dim3((n + 255) / 256), dim3(256), 0, st, accum, n, P, out, out8);
    return hipGetLastError();
}
