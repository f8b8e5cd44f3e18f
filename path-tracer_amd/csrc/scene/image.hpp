// image.hpp — texture file decoding (JPEG, PNG, BMP, TGA, Radiance HDR) for LoadTexture.
#pragma once

#include <climits>
#include <cstdint>
#include <initializer_list>
#include <string>
#include <vector>

#include "hmath.hpp"

namespace pth {

// stb_image's allocation guards (stbi__mad3sizes_valid / stbi__mad4sizes_valid):
// the product of the factors must not overflow and must stay <= INT_MAX, or
// the image is rejected as too large before anything is allocated.
inline bool StbSizesValid(std::initializer_list<uint64_t> factors)
{
    uint64_t p = 1;
    for (uint64_t f : factors) {
        if (f != 0 && p > (uint64_t)INT_MAX / f) return false;
        p *= f;
    }
    return p <= (uint64_t)INT_MAX;
}

// stbi_loadf(path, ..., 4) semantics: RGBA floats, LDR colour channels
// linearised by pow(v / 255, 2.2), alpha v / 255; HDR decoded linearly.
bool LoadImageFloat(const char* Path, int& Width, int& Height, std::vector<vec4>& Pixels, std::string& Error);

// The 8-bit RGBA samples of a JPEG / PNG / BMP / TGA (before linearisation), for tests.
bool LoadImageRGBA8(const char* Path, int& Width, int& Height, std::vector<uint8_t>& RGBA, std::string& Error);

// Baseline / progressive JPEG to RGBA8 with stb_image's output semantics (jpeg.cpp).
bool DecodeJPEG(const std::vector<uint8_t>& File, int& Width, int& Height, std::vector<uint8_t>& RGBA, std::string& Error);

}  // namespace pth
