// spectrum.cpp — restatement of the reference's RGB -> parametric spectrum
// table builder and lookup (src/core/spectrum.cpp:1-506).  Double-precision
// Gauss–Newton in CIELAB exactly as the reference; the only change is that
// the Beta-independent factor Observer(λ)·D65(λ) of each of the 471 samples
// is computed once (same operands, same order, so the same bits).
#include "spectrum.hpp"
#include "../../../include/pt_cie.h"

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
const float D65[471] = {PT_CIE_D65_VALUES};

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
