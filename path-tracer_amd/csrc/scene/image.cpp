// image.cpp — texture file decoding for LoadTexture (scene.cpp:294-313).
//
// The reference reads images with stbi_loadf(path, &w, &h, &n, 4): 8-bit (and
// 16->8-bit reduced) images come back as floats with the colour channels
// linearised by pow(v / 255, 2.2) and alpha as v / 255; Radiance .hdr files
// decode RGBE to linear floats with alpha 1.  This decoder follows the PNG
// (ISO/IEC 15948) and Radiance RGBE specifications and applies those
// conversions; it reads PNG of every colour type / bit depth (incl. palette,
// tRNS and Adam7 interlacing) and RLE or flat RGBE .hdr.
#include "image.hpp"

#include <zlib.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>

namespace pth {

namespace {

uint32_t BE32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

int Paeth(int a, int b, int c)
{
    int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    if (pa <= pb && pa <= pc) return a;
    return pb <= pc ? b : c;
}

// Unfilters one (sub-)image of w x h pixels from `src`, appending rows to `out`.
bool Unfilter(const uint8_t*& src, const uint8_t* end, uint32_t w, uint32_t h, int bits_pp, std::vector<uint8_t>& out)
{
    size_t stride = ((size_t)w * bits_pp + 7) / 8;
    int bpp = std::max(1, bits_pp / 8);
    std::vector<uint8_t> prev(stride, 0), cur(stride);
    out.resize(stride * h);
    for (uint32_t y = 0; y < h; y++) {
        if (src + 1 + stride > end) return false;
        int ft = *src++;
        for (size_t i = 0; i < stride; i++) {
            int a = i >= (size_t)bpp ? cur[i - bpp] : 0, b = prev[i], c = i >= (size_t)bpp ? prev[i - bpp] : 0;
            int x = src[i];
            switch (ft) {
            case 0: break;
            case 1: x += a; break;
            case 2: x += b; break;
            case 3: x += (a + b) >> 1; break;
            case 4: x += Paeth(a, b, c); break;
            default: return false;
            }
            cur[i] = (uint8_t)x;
        }
        src += stride;
        std::memcpy(&out[y * stride], cur.data(), stride);
        std::swap(prev, cur);
    }
    return true;
}

// Sample k of a row at bit depth d (1, 2, 4, 8, 16 -> value in [0, 2^d-1]).
uint32_t Sample(const uint8_t* row, size_t k, int d)
{
    if (d == 8) return row[k];
    if (d == 16) return (uint32_t)row[2 * k] << 8 | row[2 * k + 1];
    size_t bit = k * d;
    return (row[bit / 8] >> (8 - d - bit % 8)) & ((1u << d) - 1);
}

bool DecodePNG(const std::vector<uint8_t>& f, int& W, int& H, std::vector<uint8_t>& rgba8, std::string& err)
{
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (f.size() < 8 || std::memcmp(f.data(), sig, 8) != 0) { err = "not a PNG"; return false; }
    uint32_t w = 0, h = 0;
    int depth = 0, ctype = 0, interlace = 0;
    std::vector<uint8_t> idat, plte, trns;
    size_t pos = 8;
    bool ihdr = false;
    while (pos + 12 <= f.size()) {
        uint32_t n = BE32(&f[pos]);
        if (pos + 12 + (size_t)n > f.size()) { err = "truncated PNG chunk"; return false; }
        const uint8_t* type = &f[pos + 4];
        const uint8_t* d = &f[pos + 8];
        if (!std::memcmp(type, "IHDR", 4) && n >= 13) {
            w = BE32(d); h = BE32(d + 4); depth = d[8]; ctype = d[9]; interlace = d[12];
            ihdr = true;
        } else if (!std::memcmp(type, "PLTE", 4)) {
            plte.assign(d, d + n);
        } else if (!std::memcmp(type, "tRNS", 4)) {
            trns.assign(d, d + n);
        } else if (!std::memcmp(type, "IDAT", 4)) {
            idat.insert(idat.end(), d, d + n);
        } else if (!std::memcmp(type, "IEND", 4)) {
            break;
        }
        pos += 12 + n;
    }
    if (!ihdr || w == 0 || h == 0 || w > (1u << 24) || h > (1u << 24)) { err = "bad PNG header"; return false; }
    int channels = ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 3 ? 1 : ctype == 4 ? 2 : ctype == 6 ? 4 : 0;
    bool depth_ok = ctype == 0 ? (depth == 1 || depth == 2 || depth == 4 || depth == 8 || depth == 16)
                  : ctype == 3 ? (depth == 1 || depth == 2 || depth == 4 || depth == 8)
                               : (depth == 8 || depth == 16);
    if (!channels || !depth_ok || interlace > 1) { err = "unsupported PNG format"; return false; }
    if (ctype == 3 && plte.empty()) { err = "PNG palette missing"; return false; }
    int bits_pp = channels * depth;

    // inflate
    size_t raw_size = 0;
    static const int a7x[7] = {0, 4, 0, 2, 0, 1, 0}, a7y[7] = {0, 0, 4, 0, 2, 0, 1};
    static const int a7dx[7] = {8, 8, 4, 4, 2, 2, 1}, a7dy[7] = {8, 8, 8, 4, 4, 2, 2};
    auto pass_dim = [&](int p, uint32_t& pw, uint32_t& ph) {
        pw = (w - a7x[p] + a7dx[p] - 1) / a7dx[p];
        ph = (h - a7y[p] + a7dy[p] - 1) / a7dy[p];
        if (w <= (uint32_t)a7x[p]) pw = 0;
        if (h <= (uint32_t)a7y[p]) ph = 0;
    };
    if (interlace) {
        for (int p = 0; p < 7; p++) {
            uint32_t pw, ph;
            pass_dim(p, pw, ph);
            if (pw && ph) raw_size += (1 + ((size_t)pw * bits_pp + 7) / 8) * ph;
        }
    } else {
        raw_size = (1 + ((size_t)w * bits_pp + 7) / 8) * h;
    }
    std::vector<uint8_t> raw(raw_size);
    uLongf out_len = (uLongf)raw_size;
    int zr = uncompress(raw.data(), &out_len, idat.data(), (uLong)idat.size());
    if (zr != Z_OK || out_len != raw_size) { err = "PNG inflate failed"; return false; }

    W = (int)w;
    H = (int)h;
    rgba8.assign((size_t)w * h * 4, 0);
    auto store = [&](uint32_t x, uint32_t y, const uint8_t* row, size_t k) {
        uint8_t* o = &rgba8[((size_t)y * w + x) * 4];
        auto to8 = [&](uint32_t s) -> uint8_t {      // stb: 16-bit -> top byte; low depths scaled to 0..255
            if (depth == 16) return (uint8_t)(s >> 8);
            if (depth == 8) return (uint8_t)s;
            static const uint8_t scale[5] = {0, 0xff, 0x55, 0, 0x11};
            return (uint8_t)(s * scale[depth]);
        };
        if (ctype == 3) {
            uint32_t i = Sample(row, k, depth);
            if (3 * i + 2 >= plte.size()) { o[0] = o[1] = o[2] = 0; o[3] = 255; return; }
            o[0] = plte[3 * i]; o[1] = plte[3 * i + 1]; o[2] = plte[3 * i + 2];
            o[3] = i < trns.size() ? trns[i] : 255;
            return;
        }
        uint32_t s[4] = {0, 0, 0, 0};
        for (int c = 0; c < channels; c++) s[c] = Sample(row, k * channels + c, depth);
        if (ctype == 0) { o[0] = o[1] = o[2] = to8(s[0]); o[3] = 255; }
        else if (ctype == 2) { o[0] = to8(s[0]); o[1] = to8(s[1]); o[2] = to8(s[2]); o[3] = 255; }
        else if (ctype == 4) { o[0] = o[1] = o[2] = to8(s[0]); o[3] = to8(s[1]); }
        else { o[0] = to8(s[0]); o[1] = to8(s[1]); o[2] = to8(s[2]); o[3] = to8(s[3]); }
        // colour-key transparency for grey / RGB (tRNS holds 16-bit samples)
        if (!trns.empty() && (ctype == 0 || ctype == 2)) {
            bool match = ctype == 0 ? (trns.size() >= 2 && s[0] == ((uint32_t)trns[0] << 8 | trns[1]))
                                    : (trns.size() >= 6 && s[0] == ((uint32_t)trns[0] << 8 | trns[1]) &&
                                       s[1] == ((uint32_t)trns[2] << 8 | trns[3]) &&
                                       s[2] == ((uint32_t)trns[4] << 8 | trns[5]));
            if (match) o[3] = 0;
        }
    };
    const uint8_t* src = raw.data();
    const uint8_t* end = raw.data() + raw.size();
    std::vector<uint8_t> img;
    if (!interlace) {
        if (!Unfilter(src, end, w, h, bits_pp, img)) { err = "bad PNG filter"; return false; }
        size_t stride = ((size_t)w * bits_pp + 7) / 8;
        for (uint32_t y = 0; y < h; y++)
            for (uint32_t x = 0; x < w; x++) store(x, y, &img[y * stride], x);
    } else {
        for (int p = 0; p < 7; p++) {
            uint32_t pw, ph;
            pass_dim(p, pw, ph);
            if (!pw || !ph) continue;
            if (!Unfilter(src, end, pw, ph, bits_pp, img)) { err = "bad PNG filter"; return false; }
            size_t stride = ((size_t)pw * bits_pp + 7) / 8;
            for (uint32_t j = 0; j < ph; j++)
                for (uint32_t i = 0; i < pw; i++)
                    store(a7x[p] + i * a7dx[p], a7y[p] + j * a7dy[p], &img[j * stride], i);
        }
    }
    return true;
}

// Radiance RGBE (.hdr): header, "-Y H +X W", then flat or new-style RLE scanlines.
bool DecodeHDR(const std::vector<uint8_t>& f, int& W, int& H, std::vector<vec4>& px, std::string& err)
{
    size_t pos = 0;
    auto line = [&]() {
        std::string s;
        while (pos < f.size() && f[pos] != '\n') s += (char)f[pos++];
        if (pos < f.size()) pos++;
        return s;
    };
    std::string l = line();
    if (l != "#?RADIANCE" && l != "#?RGBE") { err = "not a Radiance HDR"; return false; }
    bool fmt = false;
    for (;;) {
        if (pos >= f.size()) { err = "truncated HDR header"; return false; }
        l = line();
        if (l.empty()) break;
        if (l == "FORMAT=32-bit_rle_rgbe") fmt = true;
    }
    if (!fmt) { err = "unsupported HDR format"; return false; }
    l = line();
    int h = 0, w = 0;
    if (std::sscanf(l.c_str(), "-Y %d +X %d", &h, &w) != 2 || w <= 0 || h <= 0) { err = "unsupported HDR layout"; return false; }
    W = w;
    H = h;
    px.assign((size_t)w * h, vec4(0, 0, 0, 1));
    std::vector<uint8_t> scan((size_t)w * 4);
    auto convert = [&](const uint8_t* rgbe, vec4& o) {   // RGBE -> float (stbi__hdr_convert, 4 channels)
        if (rgbe[3] != 0) {
            float f1 = (float)std::ldexp(1.0f, rgbe[3] - (int)(128 + 8));
            o = vec4(rgbe[0] * f1, rgbe[1] * f1, rgbe[2] * f1, 1.0f);
        } else {
            o = vec4(0, 0, 0, 1);
        }
    };
    for (int y = 0; y < h; y++) {
        bool rle = w >= 8 && w < 32768 && pos + 4 <= f.size() && f[pos] == 2 && f[pos + 1] == 2 &&
                   !(f[pos + 2] & 0x80) && ((int)f[pos + 2] << 8 | f[pos + 3]) == w;
        if (!rle) {                                      // flat RGBE pixels
            if (pos + (size_t)w * 4 > f.size()) { err = "truncated HDR data"; return false; }
            for (int x = 0; x < w; x++) convert(&f[pos + 4 * (size_t)x], px[(size_t)y * w + x]);
            pos += (size_t)w * 4;
            continue;
        }
        pos += 4;
        for (int c = 0; c < 4; c++) {
            int x = 0;
            while (x < w) {
                if (pos >= f.size()) { err = "truncated HDR RLE"; return false; }
                int count = f[pos++];
                if (count > 128) {
                    count -= 128;
                    if (count > w - x || pos >= f.size()) { err = "bad HDR RLE run"; return false; }
                    uint8_t v = f[pos++];
                    for (int k = 0; k < count; k++) scan[4 * (size_t)(x++) + c] = v;
                } else {
                    if (count == 0 || count > w - x || pos + count > f.size()) { err = "bad HDR RLE dump"; return false; }
                    for (int k = 0; k < count; k++) scan[4 * (size_t)(x++) + c] = f[pos++];
                }
            }
        }
        for (int x = 0; x < w; x++) convert(&scan[4 * (size_t)x], px[(size_t)y * w + x]);
    }
    return true;
}

}  // namespace

bool LoadImageFloat(const char* Path, int& Width, int& Height, std::vector<vec4>& Pixels, std::string& Error)
{
    std::ifstream in(Path, std::ios::binary);
    if (!in) { Error = std::string("cannot open ") + Path; return false; }
    std::vector<uint8_t> f((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    if (f.size() >= 2 && f[0] == '#' && f[1] == '?') return DecodeHDR(f, Width, Height, Pixels, Error);
    std::vector<uint8_t> rgba8;
    if (!DecodePNG(f, Width, Height, rgba8, Error)) return false;
    Pixels.resize((size_t)Width * Height);
    for (size_t i = 0; i < Pixels.size(); i++) {     // stbi__ldr_to_hdr: gamma 2.2 on colour, alpha linear
        const uint8_t* p = &rgba8[4 * i];
        Pixels[i] = vec4(std::pow(p[0] / 255.0f, 2.2f), std::pow(p[1] / 255.0f, 2.2f), std::pow(p[2] / 255.0f, 2.2f),
                         p[3] / 255.0f);
    }
    return true;
}

bool LoadImageRGBA8(const char* Path, int& Width, int& Height, std::vector<uint8_t>& RGBA, std::string& Error)
{
    std::ifstream in(Path, std::ios::binary);
    if (!in) { Error = std::string("cannot open ") + Path; return false; }
    std::vector<uint8_t> f((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    return DecodePNG(f, Width, Height, RGBA, Error);
}

}  // namespace pth
