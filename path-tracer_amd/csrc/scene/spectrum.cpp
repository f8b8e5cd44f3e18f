// spectrum.cpp — restatement of the reference's RGB -> parametric spectrum
// table builder and lookup (src/core/spectrum.cpp:1-506).  Double-precision
// Gauss–Newton in CIELAB exactly as the reference; the only change is that
// the Beta-independent factor Observer(λ)·D65(λ) of each of the 471 samples
// is computed once (same operands, same order, so the same bits).
#include "spectrum.hpp"

#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

namespace pth {

namespace {

// spectrum.cpp:8-20
const float CIE_XYZ_TO_SRGB[9] = {
    +3.2406f, -0.9689f, +0.0557f,
    -1.5372f, +1.8758f, -0.2040f,
    -0.4986f, +0.0415f, +1.0570f,
};
const float CIE_SRGB_TO_XYZ[9] = {
    +0.4124f, +0.2126f, +0.0193f,
    +0.3576f, +0.7152f, +0.1192f,
    +0.1805f, +0.0722f, +0.9505f,
};

// glm mat3 (column-major) * vec3
vec3 MulMat3(const float* m, vec3 v)
{
    vec3 r;
    for (int i = 0; i < 3; i++) r[i] = m[0 * 3 + i] * v.x + m[1 * 3 + i] * v.y + m[2 * 3 + i] * v.z;
    return r;
}

// spectrum.cpp:33-129 (CIE D65, 360..830 nm, 1 nm steps)
const float D65[471] = {
     46.638f,  47.183f,  47.728f,  48.273f,  48.819f,  49.364f,  49.909f,  50.454f,  50.999f,  51.544f,
     52.089f,  51.878f,  51.666f,  51.455f,  51.244f,  51.032f,  50.821f,  50.610f,  50.398f,  50.187f,
     49.975f,  50.443f,  50.910f,  51.377f,  51.845f,  52.312f,  52.779f,  53.246f,  53.714f,  54.181f,
     54.648f,  57.459f,  60.270f,  63.080f,  65.891f,  68.701f,  71.512f,  74.323f,  77.134f,  79.944f,
     82.755f,  83.628f,  84.501f,  85.374f,  86.247f,  87.120f,  87.994f,  88.867f,  89.740f,  90.613f,
     91.486f,  91.681f,  91.875f,  92.070f,  92.264f,  92.459f,  92.653f,  92.848f,  93.043f,  93.237f,
     93.432f,  92.757f,  92.082f,  91.407f,  90.732f,  90.057f,  89.382f,  88.707f,  88.032f,  87.357f,
     86.682f,  88.501f,  90.319f,  92.137f,  93.955f,  95.774f,  97.592f,  99.410f, 101.228f, 103.047f,
    104.865f, 106.079f, 107.294f, 108.508f, 109.722f, 110.936f, 112.151f, 113.365f, 114.579f, 115.794f,
    117.008f, 117.088f, 117.169f, 117.249f, 117.330f, 117.410f, 117.490f, 117.571f, 117.651f, 117.732f,
    117.812f, 117.517f, 117.222f, 116.927f, 116.632f, 116.336f, 116.041f, 115.746f, 115.451f, 115.156f,
    114.861f, 114.967f, 115.073f, 115.180f, 115.286f, 115.392f, 115.498f, 115.604f, 115.711f, 115.817f,
    115.923f, 115.212f, 114.501f, 113.789f, 113.078f, 112.367f, 111.656f, 110.945f, 110.233f, 109.522f,
    108.811f, 108.865f, 108.920f, 108.974f, 109.028f, 109.082f, 109.137f, 109.191f, 109.245f, 109.300f,
    109.354f, 109.199f, 109.044f, 108.888f, 108.733f, 108.578f, 108.423f, 108.268f, 108.112f, 107.957f,
    107.802f, 107.501f, 107.200f, 106.898f, 106.597f, 106.296f, 105.995f, 105.694f, 105.392f, 105.091f,
    104.790f, 105.080f, 105.370f, 105.660f, 105.950f, 106.239f, 106.529f, 106.819f, 107.109f, 107.399f,
    107.689f, 107.361f, 107.032f, 106.704f, 106.375f, 106.047f, 105.719f, 105.390f, 105.062f, 104.733f,
    104.405f, 104.369f, 104.333f, 104.297f, 104.261f, 104.225f, 104.190f, 104.154f, 104.118f, 104.082f,
    104.046f, 103.641f, 103.237f, 102.832f, 102.428f, 102.023f, 101.618f, 101.214f, 100.809f, 100.405f,
    100.000f,  99.633f,  99.267f,  98.900f,  98.534f,  98.167f,  97.800f,  97.434f,  97.067f,  96.701f,
     96.334f,  96.280f,  96.225f,  96.170f,  96.116f,  96.061f,  96.007f,  95.952f,  95.897f,  95.843f,
     95.788f,  95.078f,  94.368f,  93.657f,  92.947f,  92.237f,  91.527f,  90.816f,  90.106f,  89.396f,
     88.686f,  88.818f,  88.950f,  89.082f,  89.214f,  89.346f,  89.478f,  89.610f,  89.742f,  89.874f,
     90.006f,  89.966f,  89.925f,  89.884f,  89.843f,  89.803f,  89.762f,  89.721f,  89.680f,  89.640f,
     89.599f,  89.409f,  89.219f,  89.029f,  88.839f,  88.649f,  88.459f,  88.269f,  88.079f,  87.889f,
     87.699f,  87.258f,  86.817f,  86.376f,  85.935f,  85.494f,  85.053f,  84.612f,  84.171f,  83.730f,
     83.289f,  83.330f,  83.371f,  83.412f,  83.453f,  83.494f,  83.535f,  83.576f,  83.617f,  83.658f,
     83.699f,  83.332f,  82.965f,  82.597f,  82.230f,  81.863f,  81.496f,  81.129f,  80.761f,  80.394f,
     80.027f,  80.046f,  80.064f,  80.083f,  80.102f,  80.121f,  80.139f,  80.158f,  80.177f,  80.196f,
     80.215f,  80.421f,  80.627f,  80.834f,  81.040f,  81.246f,  81.453f,  81.659f,  81.865f,  82.072f,
     82.278f,  81.878f,  81.479f,  81.080f,  80.680f,  80.281f,  79.882f,  79.482f,  79.083f,  78.684f,
     78.284f,  77.428f,  76.572f,  75.715f,  74.859f,  74.003f,  73.147f,  72.290f,  71.434f,  70.578f,
     69.721f,  69.910f,  70.099f,  70.288f,  70.476f,  70.665f,  70.854f,  71.043f,  71.231f,  71.420f,
     71.609f,  71.883f,  72.157f,  72.431f,  72.705f,  72.979f,  73.253f,  73.527f,  73.801f,  74.075f,
     74.349f,  73.075f,  71.800f,  70.525f,  69.251f,  67.977f,  66.702f,  65.427f,  64.153f,  62.879f,
     61.604f,  62.432f,  63.260f,  64.088f,  64.917f,  65.745f,  66.573f,  67.401f,  68.229f,  69.057f,
     69.886f,  70.406f,  70.926f,  71.446f,  71.966f,  72.486f,  73.006f,  73.527f,  74.047f,  74.567f,
     75.087f,  73.938f,  72.788f,  71.639f,  70.489f,  69.340f,  68.190f,  67.041f,  65.892f,  64.742f,
     63.593f,  61.875f,  60.158f,  58.440f,  56.723f,  55.005f,  53.288f,  51.571f,  49.853f,  48.136f,
     46.418f,  48.457f,  50.496f,  52.534f,  54.573f,  56.612f,  58.651f,  60.689f,  62.728f,  64.767f,
     66.805f,  66.463f,  66.121f,  65.779f,  65.436f,  65.094f,  64.752f,  64.410f,  64.067f,  63.725f,
     63.383f,  63.475f,  63.567f,  63.659f,  63.751f,  63.843f,  63.935f,  64.028f,  64.120f,  64.212f,
     64.304f,  63.819f,  63.334f,  62.848f,  62.363f,  61.878f,  61.393f,  60.907f,  60.422f,  59.937f,
     59.452f,  58.703f,  57.953f,  57.204f,  56.455f,  55.705f,  54.956f,  54.207f,  53.458f,  52.708f,
     51.959f,  52.507f,  53.055f,  53.603f,  54.152f,  54.700f,  55.248f,  55.796f,  56.344f,  56.892f,
     57.441f,  57.728f,  58.015f,  58.302f,  58.589f,  58.877f,  59.164f,  59.451f,  59.738f,  60.025f,
     60.312f,
};

struct dvec3 {
    double x = 0, y = 0, z = 0;
    double& operator[](int i) { return (&x)[i]; }
    double operator[](int i) const { return (&x)[i]; }
};
inline dvec3 operator-(dvec3 a, dvec3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline dvec3 operator*(dvec3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
inline dvec3 operator/(dvec3 a, double s) { return {a.x / s, a.y / s, a.z / s}; }

// SampleD65 (spectrum.cpp:135-141): glm::mix(float, float, double) computes
// in double and narrows to float.
double SampleD65(double NormalizedLambda)
{
    constexpr int N = 471;
    double Offset = NormalizedLambda * (N - 1);
    int Index = std::min(std::max(int(Offset), 0), N - 2);
    double a = Offset - Index;
    return (double)(float)((double)D65[Index] * (1.0 - a) + (double)D65[Index + 1] * a);
}

// SampleObserver (spectrum.cpp:149-175): float Wyman fit at a double λ.
vec3 SampleObserverF(double NormalizedLambda)
{
    float Lambda = (float)((double)360.0f * (1.0 - NormalizedLambda) + (double)830.0f * NormalizedLambda);
    vec3 Result;
    {
        float T1 = (Lambda - 442.0f) * (Lambda < 442.0f ? 0.0624f : 0.0374f);
        float T2 = (Lambda - 599.8f) * (Lambda < 599.8f ? 0.0264f : 0.0323f);
        float T3 = (Lambda - 501.1f) * (Lambda < 501.1f ? 0.0490f : 0.0382f);
        Result.x = 0.362f * std::exp(-0.5f * T1 * T1) + 1.056f * std::exp(-0.5f * T2 * T2) - 0.065f * std::exp(-0.5f * T3 * T3);
    }
    {
        float T1 = (Lambda - 568.8f) * (Lambda < 568.8f ? 0.0213f : 0.0247f);
        float T2 = (Lambda - 530.9f) * (Lambda < 530.9f ? 0.0613f : 0.0322f);
        Result.y = 0.821f * std::exp(-0.5f * T1 * T1) + 0.286f * std::exp(-0.5f * T2 * T2);
    }
    {
        float T1 = (Lambda - 437.0f) * (Lambda < 437.0f ? 0.0845f : 0.0278f);
        float T2 = (Lambda - 459.0f) * (Lambda < 459.0f ? 0.0385f : 0.0725f);
        Result.z = 1.217f * std::exp(-0.5f * T1 * T1) + 0.681f * std::exp(-0.5f * T2 * T2);
    }
    return Result;
}

// Observer(λ_i) * W(λ_i) for the 471 samples of ObserveSpectrumUnderD65.
struct observer_weights {
    dvec3 OW[471];
    double NormalizedLambda[471];
    observer_weights()
    {
        for (int I = 0; I < 471; I++) {
            double NL = I / double(471 - 1);
            double W = SampleD65(NL) / 10566.864005;
            vec3 O = SampleObserverF(NL);
            OW[I] = dvec3{(double)O.x * W, (double)O.y * W, (double)O.z * W};
            NormalizedLambda[I] = NL;
        }
    }
};
const observer_weights& Weights()
{
    static observer_weights w;
    return w;
}

// SampleSpectrum (spectrum.cpp:182-186)
inline double SampleSpectrum(dvec3 B, double NL)
{
    double X = (B.x * NL + B.y) * NL + B.z;
    return 0.5 + X / (2.0 * std::sqrt(1.0 + X * X));
}

// ObserveSpectrumUnderD65 (spectrum.cpp:191-208):
//   XYZ += Observer * W * S * DeltaLambda, DeltaLambda = (830-360+1)/471 = 1.
dvec3 ObserveSpectrumUnderD65(dvec3 B)
{
    const observer_weights& w = Weights();
    const double DeltaLambda = (double)((830.0f - 360.0f + 1) / 471);
    dvec3 XYZ{};
    for (int I = 0; I < 471; I++) {
        double S = SampleSpectrum(B, w.NormalizedLambda[I]);
        XYZ.x += w.OW[I].x * S * DeltaLambda;
        XYZ.y += w.OW[I].y * S * DeltaLambda;
        XYZ.z += w.OW[I].z * S * DeltaLambda;
    }
    return XYZ;
}

// XYZToLab (spectrum.cpp:213-234)
dvec3 XYZToLab(dvec3 XYZ)
{
    auto F = [](double T) -> double {
        double const Delta = 6 / 29.0;
        if (T > Delta * Delta * Delta) return std::pow(T, 1 / 3.0);
        return T / (3 * Delta * Delta) + 4 / 29.0;
    };
    double FX = F(XYZ.x / 0.950489);
    double FY = F(XYZ.y);
    double FZ = F(XYZ.z / 1.088840);
    return {116.0 * FX - 16.0, 500.0 * (FX - FY), 200.0 * (FY - FZ)};
}

// glm dmat3 helpers (column-major m[col][row]).
struct dmat3 { dvec3 c[3]; };

double Determinant(const dmat3& M)
{
    auto m = [&](int a, int b) { return M.c[a][b]; };
    return +m(0, 0) * (m(1, 1) * m(2, 2) - m(2, 1) * m(1, 2))
           - m(1, 0) * (m(0, 1) * m(2, 2) - m(2, 1) * m(0, 2))
           + m(2, 0) * (m(0, 1) * m(1, 2) - m(1, 1) * m(0, 2));
}

dmat3 Inverse(const dmat3& M)
{
    auto m = [&](int a, int b) { return M.c[a][b]; };
    double OneOverDeterminant = 1.0 / (+m(0, 0) * (m(1, 1) * m(2, 2) - m(2, 1) * m(1, 2))
                                       - m(1, 0) * (m(0, 1) * m(2, 2) - m(2, 1) * m(0, 2))
                                       + m(2, 0) * (m(0, 1) * m(1, 2) - m(1, 1) * m(0, 2)));
    dmat3 R;
    R.c[0][0] = +(m(1, 1) * m(2, 2) - m(2, 1) * m(1, 2)) * OneOverDeterminant;
    R.c[1][0] = -(m(1, 0) * m(2, 2) - m(2, 0) * m(1, 2)) * OneOverDeterminant;
    R.c[2][0] = +(m(1, 0) * m(2, 1) - m(2, 0) * m(1, 1)) * OneOverDeterminant;
    R.c[0][1] = -(m(0, 1) * m(2, 2) - m(2, 1) * m(0, 2)) * OneOverDeterminant;
    R.c[1][1] = +(m(0, 0) * m(2, 2) - m(2, 0) * m(0, 2)) * OneOverDeterminant;
    R.c[2][1] = -(m(0, 0) * m(2, 1) - m(2, 0) * m(0, 1)) * OneOverDeterminant;
    R.c[0][2] = +(m(0, 1) * m(1, 2) - m(1, 1) * m(0, 2)) * OneOverDeterminant;
    R.c[1][2] = -(m(0, 0) * m(1, 2) - m(1, 0) * m(0, 2)) * OneOverDeterminant;
    R.c[2][2] = +(m(0, 0) * m(1, 1) - m(1, 0) * m(0, 1)) * OneOverDeterminant;
    return R;
}

dvec3 MulMat(const dmat3& M, dvec3 v)
{
    dvec3 r;
    for (int i = 0; i < 3; i++) r[i] = M.c[0][i] * v.x + M.c[1][i] * v.y + M.c[2][i] * v.z;
    return r;
}

// OptimizeSpectrum (spectrum.cpp:240-304); returns float coefficients like
// the reference (its return type is vec3).
vec3 OptimizeSpectrum(dvec3 NormalizedBeta, dvec3 const& TargetXYZ, int IterationCount = 15)
{
    double const Epsilon = 1e-5;
    dvec3 TargetLab = XYZToLab(TargetXYZ);
    for (int I = 0; I < IterationCount; I++) {
        dvec3 ObservedXYZ = ObserveSpectrumUnderD65(NormalizedBeta);
        dvec3 Residual = XYZToLab(ObservedXYZ) - TargetLab;
        double Error = std::sqrt(Residual.x * Residual.x + Residual.y * Residual.y + Residual.z * Residual.z);
        if (Error < 1e-3) break;

        dmat3 Jacobian{};
        for (int K = 0; K < 3; K++) {
            dvec3 Beta0 = NormalizedBeta; Beta0[K] -= Epsilon;
            dvec3 Lab0 = XYZToLab(ObserveSpectrumUnderD65(Beta0));
            dvec3 Beta1 = NormalizedBeta; Beta1[K] += Epsilon;
            dvec3 Lab1 = XYZToLab(ObserveSpectrumUnderD65(Beta1));
            Jacobian.c[K] = (Lab1 - Lab0) / (2 * Epsilon);
        }
        if (std::fabs(Determinant(Jacobian)) < 1e-15) break;

        dvec3 Step = MulMat(Inverse(Jacobian), Residual);
        NormalizedBeta = NormalizedBeta - Step;

        double Max = std::max(std::max(NormalizedBeta.x, NormalizedBeta.y), NormalizedBeta.z);
        if (Max > 200.0) NormalizedBeta = NormalizedBeta * (200.0 / Max);
    }
    return vec3((float)NormalizedBeta.x, (float)NormalizedBeta.y, (float)NormalizedBeta.z);
}

// spectrum.cpp:306-313
float IndexToScale(int K)
{
    constexpr int M = parametric_spectrum_table::SCALE_BINS;
    float R = K / float(M - 1);
    float S = R * R * (3.f - 2.f * R);
    float T = S * S * (3.f - 2.f * S);
    return T;
}

// spectrum.cpp:315-324
int ScaleToIndex(float Scale)
{
    constexpr int M = parametric_spectrum_table::SCALE_BINS;
    int K0 = 0, K1 = M;
    while (K1 - K0 > 1) {
        int K = (K0 + K1) / 2;
        (Scale > IndexToScale(K) ? K0 : K1) = K;
    }
    return K0;
}

// spectrum.cpp:326-334
vec3 IndexToColor(int I, int J, int K, int L)
{
    constexpr int N = parametric_spectrum_table::COLOR_BINS;
    vec3 Color;
    Color[L] = 1.0f;
    Color[(L + 1) % 3] = I / float(N - 1);
    Color[(L + 2) % 3] = J / float(N - 1);
    return Color * IndexToScale(K);
}

// DenormalizeBeta lambda (spectrum.cpp:370-381)
vec3 DenormalizeBeta(dvec3 B)
{
    constexpr float C0 = 360.0f;
    constexpr float C1 = 1.f / (830.0f - 360.0f);
    return vec3((float)(B[0] * C1 * C1),
                (float)(B[1] * C1 - 2 * B[0] * C0 * C1 * C1),
                (float)(B[2] - B[1] * C0 * C1 + B[0] * C0 * C0 * C1 * C1));
}

inline int ChainId(int L, int J, int I)
{
    constexpr int N = parametric_spectrum_table::COLOR_BINS;
    return (L * N + J) * N + I;
}

std::string& TablePath()
{
    static std::string path;
    return path;
}

}  // namespace

parametric_spectrum_table::parametric_spectrum_table()
{
    for (int i = 0; i < CHAIN_COUNT; i++) ChainReady[i].store(0, std::memory_order_relaxed);
}

void BuildParametricSpectrumChain(parametric_spectrum_table* Table, int L, int J, int I)
{
    constexpr int M = parametric_spectrum_table::SCALE_BINS;
    dvec3 NormalizedBeta{};
    // Light colors (spectrum.cpp:392-399).
    for (int K = M / 5; K < M; K++) {
        vec3 T = MulMat3(CIE_SRGB_TO_XYZ, IndexToColor(I, J, K, L));
        vec3 B = OptimizeSpectrum(NormalizedBeta, dvec3{T.x, T.y, T.z}, 15);
        NormalizedBeta = dvec3{B.x, B.y, B.z};
        Table->Coefficients[L][K][J][I] = DenormalizeBeta(NormalizedBeta);
    }
    // Dark colors (spectrum.cpp:401-408).
    NormalizedBeta = dvec3{};
    for (int K = M / 5; K >= 0; K--) {
        vec3 T = MulMat3(CIE_SRGB_TO_XYZ, IndexToColor(I, J, K, L));
        vec3 B = OptimizeSpectrum(NormalizedBeta, dvec3{T.x, T.y, T.z}, 15);
        NormalizedBeta = dvec3{B.x, B.y, B.z};
        Table->Coefficients[L][K][J][I] = DenormalizeBeta(NormalizedBeta);
    }
}

static void EnsureChain(parametric_spectrum_table* Table, int L, int J, int I)
{
    int id = ChainId(L, J, I);
    if (Table->ChainReady[id].load(std::memory_order_acquire)) return;
    std::lock_guard<std::mutex> lock(Table->Mutex);
    if (Table->ChainReady[id].load(std::memory_order_relaxed)) return;
    BuildParametricSpectrumChain(Table, L, J, I);
    Table->ChainReady[id].store(1, std::memory_order_release);
}

void BuildParametricSpectrumTableForSRGB(parametric_spectrum_table* Table, int threads)
{
    if (threads <= 0) {
        threads = (int)std::thread::hardware_concurrency();
        if (const char* e = std::getenv("OMP_NUM_THREADS")) threads = std::max(1, atoi(e));
        if (threads <= 0) threads = 1;
    }
    std::atomic<int> next{0};
    auto worker = [&]() {
        for (;;) {
            int id = next.fetch_add(1);
            if (id >= parametric_spectrum_table::CHAIN_COUNT) break;
            if (Table->ChainReady[id].load(std::memory_order_acquire)) continue;
            constexpr int N = parametric_spectrum_table::COLOR_BINS;
            BuildParametricSpectrumChain(Table, id / (N * N), (id / N) % N, id % N);
            Table->ChainReady[id].store(1, std::memory_order_release);
        }
    };
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; t++) pool.emplace_back(worker);
    for (auto& t : pool) t.join();
}

bool SaveParametricSpectrumTable(parametric_spectrum_table const* Table, char const* Path)
{
    FILE* File = std::fopen(Path, "wb");
    if (!File) return false;
    size_t n = std::fwrite(Table->Coefficients, sizeof(Table->Coefficients), 1, File);
    std::fclose(File);
    return n == 1;
}

bool LoadParametricSpectrumTable(parametric_spectrum_table* Table, char const* Path)
{
    FILE* File = std::fopen(Path, "rb");
    if (!File) return false;
    size_t n = std::fread(Table->Coefficients, sizeof(Table->Coefficients), 1, File);
    std::fclose(File);
    if (n != 1) return false;
    for (int i = 0; i < parametric_spectrum_table::CHAIN_COUNT; i++) Table->ChainReady[i].store(1);
    return true;
}

// ColorToIndex (spectrum.cpp:336-363) + trilinear lookup (spectrum.cpp:439-479)
vec3 GetParametricSpectrumCoefficients(parametric_spectrum_table* Table, vec3 const& InColor)
{
    constexpr int N = parametric_spectrum_table::COLOR_BINS;
    constexpr int M = parametric_spectrum_table::SCALE_BINS;

    vec3 Color(std::min(std::max(InColor.x, 0.0f), 1.0f),
               std::min(std::max(InColor.y, 0.0f), 1.0f),
               std::min(std::max(InColor.z, 0.0f), 1.0f));

    int L = 0;
    for (int K = 1; K < 3; K++)
        if (Color[K] >= Color[L]) L = K;

    float Scale = std::max(Color[L], 1e-6f);
    float X = (N - 1) * Color[(L + 1) % 3] / Scale;
    float Y = (N - 1) * Color[(L + 2) % 3] / Scale;
    int I = std::min(int(X), N - 2);
    int J = std::min(int(Y), N - 2);
    int K = std::min(ScaleToIndex(Scale), M - 2);
    float S0 = IndexToScale(K);
    float S1 = IndexToScale(K + 1);
    vec3 Alpha(X - I, Y - J, (Scale - S0) / (S1 - S0));

    EnsureChain(Table, L, J, I);
    EnsureChain(Table, L, J, I + 1);
    EnsureChain(Table, L, J + 1, I);
    EnsureChain(Table, L, J + 1, I + 1);

    auto mix3 = [](vec3 a, vec3 b, float t) {
        return vec3(a.x * (1 - t) + b.x * t, a.y * (1 - t) + b.y * t, a.z * (1 - t) + b.z * t);
    };
    auto& C = Table->Coefficients[L];
    vec3 Beta00 = mix3(C[K + 0][J + 0][I + 0], C[K + 0][J + 0][I + 1], Alpha.x);
    vec3 Beta01 = mix3(C[K + 0][J + 1][I + 0], C[K + 0][J + 1][I + 1], Alpha.x);
    vec3 Beta10 = mix3(C[K + 1][J + 0][I + 0], C[K + 1][J + 0][I + 1], Alpha.x);
    vec3 Beta11 = mix3(C[K + 1][J + 1][I + 0], C[K + 1][J + 1][I + 1], Alpha.x);
    vec3 Beta0 = mix3(Beta00, Beta01, Alpha.y);
    vec3 Beta1 = mix3(Beta10, Beta11, Alpha.y);
    return mix3(Beta0, Beta1, Alpha.z);
}

void SetSpectrumTablePath(const std::string& path) { TablePath() = path; }

parametric_spectrum_table* GetSharedSpectrumTable()
{
    static parametric_spectrum_table* table = []() {
        auto* t = new parametric_spectrum_table;
        std::string path = TablePath();
        if (path.empty()) {
            const char* e = std::getenv("PT_SPECTRUM_TABLE");
            path = e ? e : "sRGBSpectrumTable.dat";
        }
        LoadParametricSpectrumTable(t, path.c_str());
        return t;
    }();
    return table;
}

float SampleParametricSpectrum(vec3 const& Beta, float Lambda)
{
    float X = (Beta.x * Lambda + Beta.y) * Lambda + Beta.z;
    return 0.5f + X / (2.0f * std::sqrt(1.0f + X * X));
}

}  // namespace pth
