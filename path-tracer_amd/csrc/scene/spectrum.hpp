// spectrum.hpp — RGB -> Jakob–Hanika parametric spectrum coefficients.
// Restates src/core/spectrum.hpp / spectrum.cpp of the reference.
#pragma once

#include "hmath.hpp"

#include <atomic>
#include <mutex>
#include <string>

namespace pth {

// Same memory layout as the reference's parametric_spectrum_table
// (src/core/spectrum.hpp:5-11): vec3 Coefficients[3][64][64][64], so
// sRGBSpectrumTable.dat files are interchangeable (spectrum.cpp:413-437).
struct parametric_spectrum_table {
    static constexpr int SCALE_BINS = 64;
    static constexpr int COLOR_BINS = 64;
    static constexpr int CHAIN_COUNT = 3 * COLOR_BINS * COLOR_BINS;

    vec3 Coefficients[3][SCALE_BINS][COLOR_BINS][COLOR_BINS];

    // Lazy evaluation: one "chain" = all 64 scale bins of one (L, J, I),
    // which the reference computes with a warm-started sweep over K
    // (spectrum.cpp:390-408).  Chains are independent, so they are computed
    // on demand (or all at once, in parallel) with identical results.
    std::atomic<uint8_t> ChainReady[CHAIN_COUNT];
    std::mutex Mutex;

    parametric_spectrum_table();
};

// Fills in chain (L, J, I) — spectrum.cpp:380-410 for one (L, J, I).
void BuildParametricSpectrumChain(parametric_spectrum_table* Table, int L, int J, int I);

// BuildParametricSpectrumTableForSRGB (spectrum.cpp:365-411), all chains,
// spread over `threads` host threads (0 = hardware concurrency).
void BuildParametricSpectrumTableForSRGB(parametric_spectrum_table* Table, int threads = 0);

bool SaveParametricSpectrumTable(parametric_spectrum_table const* Table, char const* Path);
bool LoadParametricSpectrumTable(parametric_spectrum_table* Table, char const* Path);

// GetParametricSpectrumCoefficients (spectrum.cpp:439-479); computes any
// chain it needs that is not ready yet.
vec3 GetParametricSpectrumCoefficients(parametric_spectrum_table* Table, vec3 const& Color);

// Shared process-wide table: loaded from $PT_SPECTRUM_TABLE (or
// "sRGBSpectrumTable.dat") if present, else evaluated lazily.
parametric_spectrum_table* GetSharedSpectrumTable();
void SetSpectrumTablePath(const std::string& path);

float SampleParametricSpectrum(vec3 const& Beta, float Lambda);

}  // namespace pth
