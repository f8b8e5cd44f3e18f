// hmath.hpp — host-side vector/matrix arithmetic for the scene layer.
//
// The reference's host code (src/core/common.hpp, src/scene/scene.cpp) uses
// glm 1.0.1, which is not vendored in /root/reference.
// These are restatements of the glm operations it calls, with glm's
// published evaluation order, so the packed scene buffers are reproducible:
//   glm::inverse(mat4)   glm/detail/func_matrix.inl compute_inverse<4>
//   glm::eulerAngleZYX   glm/gtx/euler_angles.inl
//   glm::translate/scale glm/ext/matrix_transform.inl
//   glm::packSnorm2x16   glm/gtc/packing.inl (round half away from zero)
//   glm::packHalf2x16    IEEE binary16, round to nearest even
// Compiled with -ffp-contract=off.
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>
#include <algorithm>
#include <limits>

namespace pth {

struct vec2 {
    float x = 0, y = 0;
    vec2() = default;
    vec2(float a, float b) : x(a), y(b) {}
    float& operator[](int i) { return (&x)[i]; }
    float operator[](int i) const { return (&x)[i]; }
};

struct vec3 {
    float x = 0, y = 0, z = 0;
    vec3() = default;
    vec3(float a) : x(a), y(a), z(a) {}
    vec3(float a, float b, float c) : x(a), y(b), z(c) {}
    float& operator[](int i) { return (&x)[i]; }
    float operator[](int i) const { return (&x)[i]; }
};

struct vec4 {
    float x = 0, y = 0, z = 0, w = 0;
    vec4() = default;
    vec4(float a, float b, float c, float d) : x(a), y(b), z(c), w(d) {}
    vec4(vec3 v, float d) : x(v.x), y(v.y), z(v.z), w(d) {}
    float& operator[](int i) { return (&x)[i]; }
    float operator[](int i) const { return (&x)[i]; }
    vec3 xyz() const { return {x, y, z}; }
};

inline vec3 operator+(vec3 a, vec3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline vec3 operator-(vec3 a, vec3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline vec3 operator*(vec3 a, vec3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline vec3 operator*(vec3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline vec3 operator*(float s, vec3 a) { return {s * a.x, s * a.y, s * a.z}; }
inline vec3 operator/(vec3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
inline vec3 operator-(vec3 a) { return {-a.x, -a.y, -a.z}; }
inline vec3& operator+=(vec3& a, vec3 b) { a = a + b; return a; }
inline vec4 operator+(vec4 a, vec4 b) { return {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }
inline vec4 operator-(vec4 a, vec4 b) { return {a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w}; }
inline vec4 operator*(vec4 a, vec4 b) { return {a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w}; }
inline vec4 operator*(vec4 a, float s) { return {a.x * s, a.y * s, a.z * s, a.w * s}; }

inline float dot(vec3 a, vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline vec3 cross(vec3 a, vec3 b)
{
    return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y};
}
inline float length(vec3 v) { return std::sqrt(dot(v, v)); }
// glm::normalize: x * inversesqrt(dot(x, x))
inline vec3 normalize(vec3 v) { return v * (1.0f / std::sqrt(dot(v, v))); }
// glm::min / glm::max on floats use (a < b ? a : b) / (a > b ? a : b) semantics.
inline float gmin(float a, float b) { return b < a ? b : a; }
inline float gmax(float a, float b) { return a < b ? b : a; }
inline vec3 vmin(vec3 a, vec3 b) { return {gmin(a.x, b.x), gmin(a.y, b.y), gmin(a.z, b.z)}; }
inline vec3 vmax(vec3 a, vec3 b) { return {gmax(a.x, b.x), gmax(a.y, b.y), gmax(a.z, b.z)}; }

// Column-major 4x4 (glm memory order): c[col][row].
struct mat4 {
    vec4 c[4];
    mat4() = default;
    explicit mat4(float d) { for (int i = 0; i < 4; i++) { c[i] = vec4(0, 0, 0, 0); c[i][i] = d; } }
    vec4& operator[](int i) { return c[i]; }
    const vec4& operator[](int i) const { return c[i]; }
};

inline vec4 operator*(const mat4& m, vec4 v)
{
    // glm (type_mat4x4.inl, operator*(mat4, vec4)): Add0 = m[0]*v[0] + m[1]*v[1],
    // Add1 = m[2]*v[2] + m[3]*v[3], result = Add0 + Add1 (pairwise).
    vec4 r;
    for (int i = 0; i < 4; i++)
        r[i] = (m[0][i] * v[0] + m[1][i] * v[1]) + (m[2][i] * v[2] + m[3][i] * v[3]);
    return r;
}

inline mat4 operator*(const mat4& a, const mat4& b)
{
    mat4 r;
    for (int j = 0; j < 4; j++)
        for (int i = 0; i < 4; i++)
            r[j][i] = a[0][i] * b[j][0] + a[1][i] * b[j][1] + a[2][i] * b[j][2] + a[3][i] * b[j][3];
    return r;
}

inline mat4 translate(vec3 p)
{
    mat4 r(1.0f);
    // glm::translate(mat4(1), v): Result[3] = m[0]*v[0] + m[1]*v[1] + m[2]*v[2] + m[3]
    for (int i = 0; i < 4; i++)
        r[3][i] = r[0][i] * p.x + r[1][i] * p.y + r[2][i] * p.z + r[3][i];
    return r;
}

inline mat4 scale(vec3 s)
{
    mat4 r(1.0f);
    for (int i = 0; i < 4; i++) { r[0][i] = r[0][i] * s.x; r[1][i] = r[1][i] * s.y; r[2][i] = r[2][i] * s.z; }
    return r;
}

// glm::eulerAngleZYX(t1 = z, t2 = y, t3 = x)
inline mat4 eulerAngleZYX(float t1, float t2, float t3)
{
    float c1 = std::cos(t1), s1 = std::sin(t1);
    float c2 = std::cos(t2), s2 = std::sin(t2);
    float c3 = std::cos(t3), s3 = std::sin(t3);
    mat4 r(1.0f);
    r[0][0] = c1 * c2;
    r[0][1] = c2 * s1;
    r[0][2] = -s2;
    r[0][3] = 0;
    r[1][0] = c1 * s2 * s3 - c3 * s1;
    r[1][1] = c1 * c3 + s1 * s2 * s3;
    r[1][2] = c2 * s3;
    r[1][3] = 0;
    r[2][0] = s1 * s3 + c1 * c3 * s2;
    r[2][1] = c3 * s1 * s2 - c1 * s3;
    r[2][2] = c2 * c3;
    r[2][3] = 0;
    r[3][0] = 0; r[3][1] = 0; r[3][2] = 0; r[3][3] = 1;
    return r;
}

// glm compute_inverse<4>
inline mat4 inverse(const mat4& m)
{
    float Coef00 = m[2][2] * m[3][3] - m[3][2] * m[2][3];
    float Coef02 = m[1][2] * m[3][3] - m[3][2] * m[1][3];
    float Coef03 = m[1][2] * m[2][3] - m[2][2] * m[1][3];
    float Coef04 = m[2][1] * m[3][3] - m[3][1] * m[2][3];
    float Coef06 = m[1][1] * m[3][3] - m[3][1] * m[1][3];
    float Coef07 = m[1][1] * m[2][3] - m[2][1] * m[1][3];
    float Coef08 = m[2][1] * m[3][2] - m[3][1] * m[2][2];
    float Coef10 = m[1][1] * m[3][2] - m[3][1] * m[1][2];
    float Coef11 = m[1][1] * m[2][2] - m[2][1] * m[1][2];
    float Coef12 = m[2][0] * m[3][3] - m[3][0] * m[2][3];
    float Coef14 = m[1][0] * m[3][3] - m[3][0] * m[1][3];
    float Coef15 = m[1][0] * m[2][3] - m[2][0] * m[1][3];
    float Coef16 = m[2][0] * m[3][2] - m[3][0] * m[2][2];
    float Coef18 = m[1][0] * m[3][2] - m[3][0] * m[1][2];
    float Coef19 = m[1][0] * m[2][2] - m[2][0] * m[1][2];
    float Coef20 = m[2][0] * m[3][1] - m[3][0] * m[2][1];
    float Coef22 = m[1][0] * m[3][1] - m[3][0] * m[1][1];
    float Coef23 = m[1][0] * m[2][1] - m[2][0] * m[1][1];

    vec4 Fac0(Coef00, Coef00, Coef02, Coef03);
    vec4 Fac1(Coef04, Coef04, Coef06, Coef07);
    vec4 Fac2(Coef08, Coef08, Coef10, Coef11);
    vec4 Fac3(Coef12, Coef12, Coef14, Coef15);
    vec4 Fac4(Coef16, Coef16, Coef18, Coef19);
    vec4 Fac5(Coef20, Coef20, Coef22, Coef23);

    vec4 Vec0(m[1][0], m[0][0], m[0][0], m[0][0]);
    vec4 Vec1(m[1][1], m[0][1], m[0][1], m[0][1]);
    vec4 Vec2(m[1][2], m[0][2], m[0][2], m[0][2]);
    vec4 Vec3(m[1][3], m[0][3], m[0][3], m[0][3]);

    vec4 Inv0 = Vec1 * Fac0 - Vec2 * Fac1 + Vec3 * Fac2;
    vec4 Inv1 = Vec0 * Fac0 - Vec2 * Fac3 + Vec3 * Fac4;
    vec4 Inv2 = Vec0 * Fac1 - Vec1 * Fac3 + Vec3 * Fac5;
    vec4 Inv3 = Vec0 * Fac2 - Vec1 * Fac4 + Vec2 * Fac5;

    vec4 SignA(+1, -1, +1, -1);
    vec4 SignB(-1, +1, -1, +1);
    mat4 Inverse;
    Inverse[0] = Inv0 * SignA;
    Inverse[1] = Inv1 * SignB;
    Inverse[2] = Inv2 * SignA;
    Inverse[3] = Inv3 * SignB;

    vec4 Row0(Inverse[0][0], Inverse[1][0], Inverse[2][0], Inverse[3][0]);
    vec4 Dot0 = m[0] * Row0;
    float Dot1 = (Dot0.x + Dot0.y) + (Dot0.z + Dot0.w);
    float OneOverDeterminant = 1.0f / Dot1;
    mat4 r;
    for (int i = 0; i < 4; i++) r[i] = Inverse[i] * OneOverDeterminant;
    return r;
}

// src/core/common.hpp:62-82
inline mat4 MakeTransformMatrix(vec3 Position, vec3 Rotation, vec3 Scale)
{
    return translate(Position) * eulerAngleZYX(Rotation.z, Rotation.y, Rotation.x) * scale(Scale);
}

inline float fractf(float x) { return x - std::floor(x); }

// glm::packSnorm2x16
inline uint32_t packSnorm2x16(vec2 v)
{
    auto one = [](float f) -> uint32_t {
        float c = std::min(std::max(f, -1.0f), 1.0f) * 32767.0f;
        int16_t i = static_cast<int16_t>(std::round(c));
        return static_cast<uint16_t>(i);
    };
    return one(v.x) | (one(v.y) << 16);
}

inline uint32_t floatToHalf(float f)
{
    uint32_t x;
    std::memcpy(&x, &f, 4);
    uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t absx = x & 0x7fffffffu;
    if (absx >= 0x7f800000u) return sign | 0x7c00u | (absx > 0x7f800000u ? 0x200u : 0u);
    if (absx >= 0x477ff000u) return sign | 0x7c00u;  // overflow after rounding
    if (absx < 0x38800000u) {                        // subnormal half
        if (absx < 0x33000000u) return sign;
        uint32_t m = (absx & 0x7fffffu) | 0x800000u;
        int shift = 113 - (int)(absx >> 23) + 13;
        uint32_t h = m >> shift;
        uint32_t rem = m & ((1u << shift) - 1);
        uint32_t half = 1u << (shift - 1);
        if (rem > half || (rem == half && (h & 1))) h++;
        return sign | h;
    }
    uint32_t h = ((absx >> 13) - (112u << 10));
    uint32_t rem = absx & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1))) h++;
    return sign | h;
}

inline uint32_t packHalf2x16(vec2 v) { return floatToHalf(v.x) | (floatToHalf(v.y) << 16); }

inline vec2 SignNotZero(vec2 V) { return {V.x >= 0.0f ? 1.0f : -1.0f, V.y >= 0.0f ? 1.0f : -1.0f}; }

// src/core/common.hpp:100-106 (host PackUnitVector)
inline uint32_t PackUnitVector(vec3 V)
{
    float inv = 1.0f / (std::fabs(V.x) + std::fabs(V.y) + std::fabs(V.z));
    vec2 P(V.x * inv, V.y * inv);
    if (V.z <= 0.0f) {
        vec2 S = SignNotZero(P);
        P = vec2((1.0f - std::fabs(P.y)) * S.x, (1.0f - std::fabs(P.x)) * S.y);
    }
    return packSnorm2x16(P);
}

constexpr float PI = 3.141592653f;
constexpr float TAU = 6.283185306f;
constexpr float EPSILON = 1e-9f;
constexpr float INF = std::numeric_limits<float>::infinity();

}  // namespace pth
