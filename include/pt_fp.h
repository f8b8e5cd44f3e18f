/*
 * pt_fp.h — the floating-point convention of the MI355X path tracer.
 *
 * The reference integrator runs GLSL compiled by glslc for whatever Vulkan
 * driver is present, so its transcendental functions, FMA contraction and
 * rounding are driver-defined ("parity unpinned").  Both the
 * HIP kernels and the CPU oracle therefore follow ONE written convention,
 * defined here, so that a path traced on gfx950 and the same path traced on
 * the host take bit-identical decisions:
 *
 *   - only IEEE-754 binary32 +, -, *, / and sqrt (correctly rounded on both
 *     gfx950 — hipcc's default div/sqrt lowering — and x86 SSE), compiled with
 *     -ffp-contract=off on both compilers (no FMA, no reassociation);
 *   - exp/log/sin/cos/atan2/asin are the polynomial kernels below, written
 *     with an explicit evaluation order (errors vs. libm are pinned by
 *     tests/test_fp_conventions.py);
 *   - min/max follow IEEE minNum/maxNum (a NaN operand loses), which is what
 *     gfx950's v_min_f32/v_max_f32 and C fminf/fmaxf do;
 *   - normalize(v) = v * (1/sqrt(dot(v,v))), dot is evaluated left to right;
 *   - mix(x,y,a) = x*(1-a) + y*a (the GLSL / glm formula);
 *   - packSnorm2x16 rounds half away from zero (glm's round()).
 *
 * This header is shared by product code (path-tracer_amd/csrc) and by the
 * oracle; it contains no integrator logic.  Reference formulas are cited at
 * each function (paths relative to the reference root).
 */
#ifndef PT_FP_H
#define PT_FP_H

#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#define PT_HD __host__ __device__ __forceinline__
#else
#define PT_HD static inline
#endif

/* --- constants (src/core/common.glsl.inc:4-15) ------------------------------ */

#define PT_INFINITY       1e30f
#define PT_EPSILON        1e-9f
#define PT_PI             3.141592653f
#define PT_TAU            6.283185306f
#define PT_HIT_TIME_LIMIT 1048576.0f
#define PT_CIE_LAMBDA_MIN 360.0f
#define PT_CIE_LAMBDA_MAX 830.0f

#define PT_RENDER_FLAG_ACCUMULATE    1u
#define PT_RENDER_FLAG_SAMPLE_JITTER 2u

/* --- bit casts --------------------------------------------------------------- */

PT_HD uint32_t pt_f2u(float x) { union { float f; uint32_t u; } c; c.f = x; return c.u; }
PT_HD float pt_u2f(uint32_t x) { union { float f; uint32_t u; } c; c.u = x; return c.f; }

/* --- scalar helpers ---------------------------------------------------------- */

PT_HD float pt_min(float a, float b) { return fminf(a, b); }
PT_HD float pt_max(float a, float b) { return fmaxf(a, b); }
PT_HD float pt_abs(float a) { return fabsf(a); }
PT_HD float pt_sqrt(float a) { return sqrtf(a); }
PT_HD float pt_floor(float a) { return floorf(a); }
PT_HD float pt_clamp(float x, float lo, float hi) { return pt_min(pt_max(x, lo), hi); }
/* GLSL fract(x) = x - floor(x). */
PT_HD float pt_fract(float x) { return x - floorf(x); }
/* GLSL sign(). */
PT_HD float pt_sign(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }
/* GLSL / glm mix(). */
PT_HD float pt_mix(float x, float y, float a) { return x * (1.0f - a) + y * a; }
PT_HD uint32_t pt_umin(uint32_t a, uint32_t b) { return a < b ? a : b; }

/* Fused multiply-add, correctly rounded on both sides (v_fma_f32 on the
 * device, C99 fmaf on the host): the polynomial kernels below evaluate
 * their Horner steps with it (one rounding per step, half the operations).
 * Written out explicitly, so -ffp-contract=off still governs everything else. */
#ifdef __HIP_DEVICE_COMPILE__
PT_HD float pt_fma(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
#else
PT_HD float pt_fma(float a, float b, float c) { return fmaf(a, b, c); }
#endif

/* 2^k for integer k in [-126, 127] by exponent construction (exact). */
PT_HD float pt_pow2i(int k) { return pt_u2f((uint32_t)(k + 127) << 23); }

/* Round to nearest integer, ties to even, for |x| < 2^22 (exact). */
PT_HD float pt_rint(float x)
{
    const float magic = 12582912.0f; /* 1.5 * 2^23 */
    float r = (x + magic) - magic;
    return r;
}

/* --- exp / log --------------------------------------------------------------- */

/* e^x.  Cody–Waite reduction x = k ln2 + r, |r| <= ln2/2, degree-7 Taylor
 * polynomial in Horner form, then exact scaling by 2^k in two steps
 * 2^k1 * 2^(k - k1) with k1 = clamp(k, -126, 127) (k - k1 = 0 in the normal
 * range, where the second factor is exactly 1; the subnormal and overflow
 * ranges need both).  Branch-free: the out-of-range and NaN inputs are
 * resolved by selects after the common path, on a clamped argument. */
PT_HD float pt_exp(float x)
{
    float xc = pt_min(pt_max(x, -103.97208404541015625f), 88.72283935546875f);
    float k = pt_rint(xc * 1.44269502162933349609375f);
    float r = (xc - k * 0.693145751953125f) - k * 1.428606765330187045e-06f;
    float p = 1.98412698412698413e-04f;            /* 1/5040 */
    p = pt_fma(p, r, 1.38888888888888889e-03f);          /* 1/720 */
    p = pt_fma(p, r, 8.33333333333333333e-03f);          /* 1/120 */
    p = pt_fma(p, r, 4.16666666666666667e-02f);          /* 1/24 */
    p = pt_fma(p, r, 1.66666666666666667e-01f);          /* 1/6 */
    p = pt_fma(p, r, 0.5f);
    p = pt_fma(p, r, 1.0f);
    p = pt_fma(p, r, 1.0f);
    int ki = (int)k;
    int k1 = ki < -126 ? -126 : (ki > 127 ? 127 : ki);
    float y = p * pt_pow2i(k1) * pt_pow2i(ki - k1);
    y = x > 88.72283935546875f ? pt_u2f(0x7f800000u) : y;
    y = x < -103.97208404541015625f ? 0.0f : y;
    return x == x ? y : x;                         /* NaN */
}

/* Natural logarithm (fdlibm e_logf.c structure: x = 2^e (1+f),
 * log(1+f) = f - hfsq + s (hfsq + R), s = f/(2+f)). */
PT_HD float pt_log(float x)
{
    if (!(x == x)) return x;
    if (x < 0.0f) return pt_u2f(0x7fc00000u);
    if (x == 0.0f) return pt_u2f(0xff800000u);
    if (x == pt_u2f(0x7f800000u)) return x;
    uint32_t ix = pt_f2u(x);
    int e = 0;
    if (ix < 0x00800000u) { x = x * 33554432.0f; ix = pt_f2u(x); e = -25; }
    e += (int)(ix >> 23) - 127;
    ix &= 0x007fffffu;
    /* normalise mantissa into [sqrt(1/2), sqrt(2)) */
    uint32_t i = (ix + (0x95f64u << 3)) & 0x800000u;
    float m = pt_u2f(ix | (i ^ 0x3f800000u));
    e += (int)(i >> 23);
    float f = m - 1.0f;
    float s = f / (2.0f + f);
    float z = s * s;
    float w = z * z;
    float t1 = w * pt_fma(w, 2.2222198546e-01f, 4.0000000596e-01f);
    float t2 = z * pt_fma(w, 2.8571429849e-01f, 6.6666668653e-01f);
    float R = t2 + t1;
    float hfsq = 0.5f * f * f;
    float dk = (float)e;
    return dk * 6.9313812256e-01f - ((hfsq - (s * (hfsq + R) + dk * 9.0580006145e-06f)) - f);
}

/* x^y as e^(y log x): GLSL defines pow(x, y) as exp2(y * log2(x)) (undefined
 * for x < 0, and for x = 0 with y <= 0); the same identity in base e on the
 * two kernels above.  x = 0, y > 0 gives e^-inf = 0. */
PT_HD float pt_pow(float x, float y) { return pt_exp(y * pt_log(x)); }

/* --- sin / cos --------------------------------------------------------------- */

/* Reduce x by pi/2: returns r in [-pi/4, pi/4] and quadrant q (valid for
 * |x| < 2^13, which covers every angle the integrator forms). */
PT_HD float pt_reduce_pio2(float x, int* q)
{
    float k = pt_rint(x * 0.636619772367581343f);
    float r = x - k * 1.5703125f;                  /* 1.5703125 = 201/128, exact products */
    r = r - k * 4.837512969970703125e-04f;
    r = r - k * 7.549789948768648e-08f;
    *q = (int)k;
    return r;
}

/* Cephes sinf/cosf kernels on |r| <= pi/4 (single-precision minimax). */
PT_HD float pt_sin_kernel(float r)
{
    float z = r * r;
    float p = -1.9515295891e-4f;
    p = pt_fma(p, z, 8.3321608736e-3f);
    p = pt_fma(p, z, -1.6666654611e-1f);
    return pt_fma(p * z, r, r);
}

PT_HD float pt_cos_kernel(float r)
{
    float z = r * r;
    float p = 2.443315711809948e-5f;
    p = pt_fma(p, z, -1.388731625493765e-3f);
    p = pt_fma(p, z, 4.166664568298827e-2f);
    float y = p * z * z;
    y = pt_fma(-0.5f, z, y);
    return y + 1.0f;
}

/* Quadrant selection by selects (both kernels are evaluated). */
PT_HD float pt_sin(float x)
{
    int q;
    float r = pt_reduce_pio2(x, &q);
    float s = pt_sin_kernel(r), c = pt_cos_kernel(r);
    float v = (q & 1) ? c : s;
    return (q & 2) ? -v : v;
}

PT_HD float pt_cos(float x)
{
    int q;
    float r = pt_reduce_pio2(x, &q);
    float s = pt_sin_kernel(r), c = pt_cos_kernel(r);
    float v = (q & 1) ? s : c;
    return ((q + 1) & 2) ? -v : v;
}

/* --- atan2 / asin ------------------------------------------------------------ */

/* atan(t) for t >= 0 (Cephes atanf reduction to |t| <= tan(pi/8)). */
PT_HD float pt_atan_pos(float t)
{
    float y0 = 0.0f;
    if (t > 2.414213562373095f) { y0 = 1.5707963267948966f; t = -1.0f / t; }
    else if (t > 0.4142135623730950f) { y0 = 0.7853981633974483f; t = (t - 1.0f) / (t + 1.0f); }
    float z = t * t;
    float p = 8.05374449538e-2f;
    p = pt_fma(p, z, -1.38776856032e-1f);
    p = pt_fma(p, z, 1.99777106478e-1f);
    p = pt_fma(p, z, -3.33329491539e-1f);
    return y0 + pt_fma(p * z, t, t);
}

/* GLSL atan(y, x); returns 0 for (0, 0). */
PT_HD float pt_atan2(float y, float x)
{
    if (x == 0.0f && y == 0.0f) return 0.0f;
    float ax = pt_abs(x), ay = pt_abs(y);
    float a;
    if (ax >= ay) a = pt_atan_pos(ay / ax);
    else a = 1.5707963267948966f - pt_atan_pos(ax / ay);
    if (x < 0.0f) a = 3.14159265358979f - a;
    return y < 0.0f ? -a : a;
}

/* GLSL asin(x) for |x| <= 1 (Cephes asinf). */
PT_HD float pt_asin(float x)
{
    float a = pt_abs(x);
    if (a > 1.0f) return pt_u2f(0x7fc00000u);
    float z, s, flag = 0.0f;
    if (a > 0.5f) { z = 0.5f * (1.0f - a); s = pt_sqrt(z); flag = 1.0f; }
    else { z = a * a; s = a; }
    float p = 4.2163199048e-2f;
    p = pt_fma(p, z, 2.4181311049e-2f);
    p = pt_fma(p, z, 4.5470025998e-2f);
    p = pt_fma(p, z, 7.4953002686e-2f);
    p = pt_fma(p, z, 1.6666752422e-1f);
    float r = pt_fma(p * z, s, s);
    if (flag != 0.0f) r = 1.5707963267948966f - (r + r);
    return x < 0.0f ? -r : r;
}

/* --- PCG hash RNG (src/core/common.glsl.inc:189-203) ------------------------- */

PT_HD uint32_t pt_random(uint32_t* state)
{
    *state = *state * 747796405u + 2891336453u;
    uint32_t s = *state;
    uint32_t w = ((s >> ((s >> 28u) + 4u)) ^ s) * 277803737u;
    return (w >> 22u) ^ w;
}

/* Random() / 4294967296.0f: u32 -> f32 (round to nearest even) then exact /2^32.
 * Can return exactly 1.0f for inputs >= 2^32 - 128, as the GLSL does. */
PT_HD float pt_random01(uint32_t* state)
{
    return (float)pt_random(state) * 2.3283064365386963e-10f;
}

/* Per-dispatch seed (src/integrator/basic_scatter.glsl:315-318). */
PT_HD uint32_t pt_seed(uint32_t gx, uint32_t gy, uint32_t random_seed)
{
    return gy * 65537u + gx + random_seed * 277803737u;
}

/* --- snorm16 / half packing -------------------------------------------------- */

/* glm::round semantics (half away from zero) for |x| <= 32767. */
PT_HD float pt_round_half_away(float x)
{
    float t = truncf(x);
    if (pt_abs(x - t) >= 0.5f) t = t + (x < 0.0f ? -1.0f : 1.0f);
    return t;
}

PT_HD uint32_t pt_pack_snorm16(float v)
{
    float c = pt_clamp(v, -1.0f, 1.0f) * 32767.0f;
    int32_t i = (int32_t)pt_round_half_away(c);
    return (uint32_t)(uint16_t)(int16_t)i;
}

/* glm::unpackSnorm2x16 component: clamp(x / 32767, -1, 1) for the int16 x.
   The quotient is evaluated as q = RN(x * RN(1/32767)) and one FMA residual
   correction (Markstein), which equals the IEEE quotient for every one of
   the 65 536 inputs (checked exhaustively with exact rational arithmetic and
   against the division, tests/test_numerics.py): 3 operations instead of a
   division on the device. */
PT_HD float pt_unpack_snorm16(uint32_t bits)
{
    const float r = 1.0f / 32767.0f;
    float x = (float)(int16_t)(uint16_t)bits;
    float q = x * r;
    float e = pt_fma(-q, 32767.0f, x);
    float f = pt_fma(e, r, q);
    return pt_clamp(f, -1.0f, 1.0f);
}

/* IEEE half -> float, exact. */
PT_HD float pt_half_to_float(uint32_t h)
{
    uint32_t sign = (h & 0x8000u) << 16;
    uint32_t exp = (h >> 10) & 0x1fu;
    uint32_t man = h & 0x3ffu;
    if (exp == 0) {
        float f = (float)man * 5.9604644775390625e-08f; /* 2^-24 */
        return (h & 0x8000u) ? -f : f;
    }
    if (exp == 31) return pt_u2f(sign | 0x7f800000u | (man << 13));
    return pt_u2f(sign | ((exp + 112u) << 23) | (man << 13));
}

#endif /* PT_FP_H */
