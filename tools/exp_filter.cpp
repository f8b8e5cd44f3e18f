// Experiment (CPU): how often would a filtered slab test -- one FMA per plane
// from the per-ray reciprocal and a precomputed O*Y, with a rounding-error
// margin -- be unable to decide a BLAS box pair the way the exact IEEE
// division decides it?  Traverses the BLAS exactly like the reference
// (scene.glsl.inc:336-399) and, at every internal node, classifies the
// filtered decision as robust-and-equal, robust-but-different (a bound
// violation: must never happen) or ambiguous (the kernel would fall back).
// Build: g++ -O2 -ffp-contract=off -shared -fPIC -o /tmp/exp_filter.so tools/exp_filter.cpp
#include <cmath>
#include <cstdint>
#include <cstring>

namespace {
struct node { float mn[3]; uint32_t a; float mx[3]; uint32_t b; };
struct face { float p0[3]; uint32_t v0; float p1[3]; uint32_t v1; float p2[3]; uint32_t v2; };

const float INF = INFINITY;

float exact_box(const float* O, const float* V, float reach, const node& n)
{
    float e = -INF, x = INF;
    float en[3], ex[3];
    for (int i = 0; i < 3; i++) {
        float a = (n.mn[i] - O[i]) / V[i];
        float b = (n.mx[i] - O[i]) / V[i];
        en[i] = fminf(a, b);
        ex[i] = fmaxf(a, b);
    }
    e = fmaxf(fmaxf(en[0], en[1]), en[2]);
    x = fminf(fminf(ex[0], ex[1]), ex[2]);
    if (x < e) return INF;
    if (x <= 0) return INF;
    if (e >= reach) return INF;
    return e;
}

// filtered: returns approx T (INF on miss) and sets amb when a comparison is
// within the error margin.  K: margin multiplier on u = 2^-24.
float filt_box(const float* Y, const float* OY, float oyM, float reach, const node& n, float K, bool& amb,
               int* why, float& margin)
{
    float en[3], ex[3];
    for (int i = 0; i < 3; i++) {
        float a = fmaf(n.mn[i], Y[i], -OY[i]);
        float b = fmaf(n.mx[i], Y[i], -OY[i]);
        en[i] = fminf(a, b);
        ex[i] = fmaxf(a, b);
    }
    float e = fmaxf(fmaxf(en[0], en[1]), en[2]);
    float x = fminf(fminf(ex[0], ex[1]), ex[2]);
    float m = K * 0x1p-24f * fmaxf(fmaxf(fabsf(e), fabsf(x)), oyM);
    margin = m;
    float m2 = 2 * m;
    bool a1 = fabsf(x - e) <= m2, a2 = fabsf(x) <= m2, a3 = fabsf(reach - e) <= m2;
    if (a1) why[0]++;
    if (a2) why[1]++;
    if (a3) why[2]++;
    amb = a1 | a2 | a3;
    bool miss = (x < e) | (x <= 0) | (e >= reach);
    return miss ? INF : e;
}

bool face_test(const float* O, const float* V, const face& f, float& T, float& U, float& W, float tmax)
{
    float e1[3], e2[3], s[3];
    for (int i = 0; i < 3; i++) { e1[i] = f.p1[i] - f.p0[i]; e2[i] = f.p2[i] - f.p0[i]; s[i] = O[i] - f.p0[i]; }
    float r[3] = {V[1] * e2[2] - V[2] * e2[1], V[2] * e2[0] - V[0] * e2[2], V[0] * e2[1] - V[1] * e2[0]};
    float det = e1[0] * r[0] + e1[1] * r[1] + e1[2] * r[2];
    if (fabsf(det) < 1e-9f) return false;
    float inv = 1.0f / det;
    U = inv * (s[0] * r[0] + s[1] * r[1] + s[2] * r[2]);
    if (U < 0 || U > 1) return false;
    float c[3] = {s[1] * e1[2] - s[2] * e1[1], s[2] * e1[0] - s[0] * e1[2], s[0] * e1[1] - s[1] * e1[0]};
    W = inv * (V[0] * c[0] + V[1] * c[1] + V[2] * c[2]);
    if (W < 0 || U + W > 1) return false;
    T = inv * (e2[0] * c[0] + e2[1] * c[1] + e2[2] * c[2]);
    if (T < 0 || T > tmax) return false;
    return true;
}
}  // namespace

extern "C" {
// stats[0] internal steps, [1] ambiguous steps, [2] robust-but-wrong, [3] pair-order ambiguous,
// [4..6] why (x-e, x, reach-e), [7] rays, [8] exact-tie TA==TB both hit
void exp_filter(const node* nodes, const face* faces, uint32_t root, uint32_t n, const float* O3, const float* V3,
                float duration, float K, uint64_t* stats)
{
    for (uint32_t r = 0; r < n; r++) {
        const float* O = O3 + 3 * r;
        const float* V = V3 + 3 * r;
        float Y[3], OY[3];
        for (int i = 0; i < 3; i++) { Y[i] = 1.0f / V[i]; OY[i] = O[i] * Y[i]; }
        float oyM = fmaxf(fmaxf(fabsf(OY[0]), fabsf(OY[1])), fabsf(OY[2]));
        float time = duration;
        uint32_t stack[32], depth = 0;
        node N = nodes[root];
        stats[7]++;
        int why[3] = {0, 0, 0};
        while (true) {
            if (N.b > 0) {
                for (uint32_t F = N.a; F < N.b; F++) {
                    float T, U, W;
                    if (face_test(O, V, faces[F], T, U, W, time)) time = T;
                }
            } else {
                uint32_t I = N.a;
                node A = nodes[I], B = nodes[I + 1];
                float TA = exact_box(O, V, time, A), TB = exact_box(O, V, time, B);
                bool ambA, ambB;
                float mA, mB;
                float PA = filt_box(Y, OY, oyM, time, A, K, ambA, why, mA);
                float PB = filt_box(Y, OY, oyM, time, B, K, ambB, why, mB);
                bool amb = ambA | ambB;
                bool bothhit = PA < INF && PB < INF;
                bool ord = bothhit && fabsf(PA - PB) <= 2 * (mA + mB);
                stats[0]++;
                if (ord) stats[3]++;
                amb |= ord;
                if (TA < INF && TB < INF && TA == TB) stats[8]++;
                bool exA = TA < INF, exB = TB < INF, exGo = TA > TB;
                bool fA = PA < INF, fB = PB < INF, fGo = PA > PB;
                if (amb) stats[1]++;
                else if (exA != fA || exB != fB || exGo != fGo) stats[2]++;
                if (TA > TB) {
                    if (TA < INF && depth < 32) stack[depth++] = I;
                    N = B;
                    continue;
                }
                if (TB < INF) { if (depth < 32) stack[depth++] = I + 1; N = A; continue; }
                if (TA < INF) { N = A; continue; }
            }
            if (depth == 0) break;
            N = nodes[stack[--depth]];
        }
        stats[4] += why[0];
        stats[5] += why[1];
        stats[6] += why[2];
    }
}
}
