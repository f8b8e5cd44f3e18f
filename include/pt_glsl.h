/*
 * pt_glsl.h — GLSL 450 vector/matrix built-ins under the pt_fp.h convention.
 *
 * Language semantics only (no integrator logic): component-wise operators,
 * dot/cross/normalize/length, min/max/abs/sign, mix, and the column-major
 * mat4 * vec4 and vec4 * mat4 products.  Every reduction is evaluated left to
 * right (x, then y, then z, then w), which is the order both the HIP kernels
 * and the CPU oracle are required to follow.  C++ only (host or HIP device).
 */
#ifndef PT_GLSL_H
#define PT_GLSL_H

#include "pt_fp.h"

struct pt2 { float x, y; };
struct pt3 { float x, y, z; };
struct pt4 { float x, y, z, w; };

PT_HD pt2 v2(float x, float y) { pt2 r; r.x = x; r.y = y; return r; }
PT_HD pt3 v3(float x, float y, float z) { pt3 r; r.x = x; r.y = y; r.z = z; return r; }
PT_HD pt3 v3s(float s) { return v3(s, s, s); }
PT_HD pt4 v4(float x, float y, float z, float w) { pt4 r; r.x = x; r.y = y; r.z = z; r.w = w; return r; }
PT_HD pt4 v4s(float s) { return v4(s, s, s, s); }

/* vec2 */
PT_HD pt2 operator+(pt2 a, pt2 b) { return v2(a.x + b.x, a.y + b.y); }
PT_HD pt2 operator-(pt2 a, pt2 b) { return v2(a.x - b.x, a.y - b.y); }
PT_HD pt2 operator*(pt2 a, pt2 b) { return v2(a.x * b.x, a.y * b.y); }
PT_HD pt2 operator*(pt2 a, float s) { return v2(a.x * s, a.y * s); }
PT_HD pt2 operator*(float s, pt2 a) { return v2(s * a.x, s * a.y); }
PT_HD pt2 operator/(pt2 a, pt2 b) { return v2(a.x / b.x, a.y / b.y); }
PT_HD float dot(pt2 a, pt2 b) { return a.x * b.x + a.y * b.y; }
PT_HD float length(pt2 v) { return pt_sqrt(dot(v, v)); }

/* vec3 */
PT_HD pt3 operator+(pt3 a, pt3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
PT_HD pt3 operator-(pt3 a, pt3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
PT_HD pt3 operator-(pt3 a) { return v3(-a.x, -a.y, -a.z); }
PT_HD pt3 operator*(pt3 a, pt3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
PT_HD pt3 operator*(pt3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
PT_HD pt3 operator*(float s, pt3 a) { return v3(s * a.x, s * a.y, s * a.z); }
PT_HD pt3 operator/(pt3 a, pt3 b) { return v3(a.x / b.x, a.y / b.y, a.z / b.z); }
PT_HD pt3 operator/(pt3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
PT_HD float dot(pt3 a, pt3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
PT_HD pt3 cross(pt3 a, pt3 b)
{
    return v3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
PT_HD float length(pt3 v) { return pt_sqrt(dot(v, v)); }
PT_HD pt3 normalize(pt3 v) { float s = 1.0f / pt_sqrt(dot(v, v)); return v * s; }
PT_HD pt3 vabs(pt3 a) { return v3(pt_abs(a.x), pt_abs(a.y), pt_abs(a.z)); }
PT_HD pt3 vmin(pt3 a, pt3 b) { return v3(pt_min(a.x, b.x), pt_min(a.y, b.y), pt_min(a.z, b.z)); }
PT_HD pt3 vmax(pt3 a, pt3 b) { return v3(pt_max(a.x, b.x), pt_max(a.y, b.y), pt_max(a.z, b.z)); }

/* vec4 */
PT_HD pt4 operator+(pt4 a, pt4 b) { return v4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
PT_HD pt4 operator-(pt4 a, pt4 b) { return v4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }
PT_HD pt4 operator-(pt4 a) { return v4(-a.x, -a.y, -a.z, -a.w); }
PT_HD pt4 operator*(pt4 a, pt4 b) { return v4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w); }
PT_HD pt4 operator*(pt4 a, float s) { return v4(a.x * s, a.y * s, a.z * s, a.w * s); }
PT_HD pt4 operator*(float s, pt4 a) { return v4(s * a.x, s * a.y, s * a.z, s * a.w); }
PT_HD pt4 operator/(pt4 a, pt4 b) { return v4(a.x / b.x, a.y / b.y, a.z / b.z, a.w / b.w); }
PT_HD pt4 operator/(pt4 a, float s) { return v4(a.x / s, a.y / s, a.z / s, a.w / s); }
PT_HD pt4 operator+(float s, pt4 a) { return v4(s + a.x, s + a.y, s + a.z, s + a.w); }
PT_HD pt4 operator-(float s, pt4 a) { return v4(s - a.x, s - a.y, s - a.z, s - a.w); }
PT_HD pt4 operator/(float s, pt4 a) { return v4(s / a.x, s / a.y, s / a.z, s / a.w); }
PT_HD pt4 vabs(pt4 a) { return v4(pt_abs(a.x), pt_abs(a.y), pt_abs(a.z), pt_abs(a.w)); }
PT_HD pt4 vmax(pt4 a, float s) { return v4(pt_max(a.x, s), pt_max(a.y, s), pt_max(a.z, s), pt_max(a.w, s)); }
PT_HD pt4 vsqrt(pt4 a) { return v4(pt_sqrt(a.x), pt_sqrt(a.y), pt_sqrt(a.z), pt_sqrt(a.w)); }
PT_HD pt4 vexp(pt4 a) { return v4(pt_exp(a.x), pt_exp(a.y), pt_exp(a.z), pt_exp(a.w)); }
PT_HD pt4 vlog(pt4 a) { return v4(pt_log(a.x), pt_log(a.y), pt_log(a.z), pt_log(a.w)); }
PT_HD pt4 vsign(pt4 a) { return v4(pt_sign(a.x), pt_sign(a.y), pt_sign(a.z), pt_sign(a.w)); }
PT_HD pt4 vpow(pt4 a, float e) { return v4(pt_pow(a.x, e), pt_pow(a.y, e), pt_pow(a.z, e), pt_pow(a.w, e)); }
/* max4 (src/core/common.glsl.inc:107-110) */
PT_HD float max4(pt4 v) { return pt_max(pt_max(v.x, v.y), pt_max(v.z, v.w)); }

/* Column-major 4x4 matrix as stored in pt_packed_transform (float[16]). */
PT_HD pt3 mat4_mul_point(const float* m, pt3 p)
{
    /* (M * vec4(p, 1)).xyz */
    return v3(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12] * 1.0f,
              m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13] * 1.0f,
              m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14] * 1.0f);
}
PT_HD pt3 mat4_mul_vector(const float* m, pt3 v)
{
    /* (M * vec4(v, 0)).xyz */
    return v3(m[0] * v.x + m[4] * v.y + m[8] * v.z + m[12] * 0.0f,
              m[1] * v.x + m[5] * v.y + m[9] * v.z + m[13] * 0.0f,
              m[2] * v.x + m[6] * v.y + m[10] * v.z + m[14] * 0.0f);
}
PT_HD pt3 vec_mul_mat4(pt3 v, const float* m)
{
    /* (vec4(v, 0) * M).xyz : component i = dot(vec4(v,0), column i) */
    return v3(v.x * m[0] + v.y * m[1] + v.z * m[2] + 0.0f * m[3],
              v.x * m[4] + v.y * m[5] + v.z * m[6] + 0.0f * m[7],
              v.x * m[8] + v.y * m[9] + v.z * m[10] + 0.0f * m[11]);
}

#endif /* PT_GLSL_H */
