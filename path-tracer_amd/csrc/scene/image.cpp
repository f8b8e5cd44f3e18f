// image.cpp — texture file decoding for LoadTexture (scene.cpp:294-313).
//
// The reference reads images with stbi_loadf(path, &w, &h, &n, 4): 8-bit (and
// 16->8-bit reduced) images come back as floats with the colour channels
// linearised by pow(v / 255, 2.2) and alpha as v / 255; Radiance .hdr files
// decode RGBE to linear floats with alpha 1.  This decoder follows the PNG
// (ISO/IEC 15948) and Radiance RGBE specifications and applies those
// conversions; it reads JPEG (jpeg.cpp), PNG of every colour type / bit depth (incl. palette,
// tRNS and Adam7 interlacing), BMP, GIF (first frame), PSD (composite), binary
// PNM, TGA and RLE or flat RGBE .hdr.
#include "image.hpp"

#include <zlib.h>

#include <algorithm>
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
    if (!StbSizesValid({w, h, 4})) { err = "too large"; return false; }
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
    if (w > (1 << 24) || h > (1 << 24) || !StbSizesValid({(uint64_t)w, (uint64_t)h, 4, sizeof(float)})) {
        err = "too large";
        return false;
    }
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

uint32_t LE16(const uint8_t* p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8; }
uint32_t LE32(const uint8_t* p) { return LE16(p) | LE16(p + 2) << 16; }

// A 5-bit channel widened to 8 bits the way stb_image's TGA reader does:
// (v * 255) / 31, integer division.
uint8_t Widen5(uint32_t v) { return (uint8_t)((v * 255u) / 31u); }

// Truevision TGA (stbi__tga_load semantics): image types 1 / 2 / 3
// (colour-mapped, true-colour, grey) and their RLE forms 9 / 10 / 11;
// 8-bit grey or index, 16-bit grey+alpha, 15/16-bit RGB555 (the attribute
// bit ignored, alpha 255), 24-bit BGR, 32-bit BGRA; palettes of 15/16/24/32-bit
// entries.  Rows are stored bottom-up unless descriptor bit 5 is set.
bool DecodeTGA(const std::vector<uint8_t>& f, int& W, int& H, std::vector<uint8_t>& rgba8, std::string& err)
{
    if (f.size() < 18) { err = "not a TGA"; return false; }
    uint32_t idlen = f[0], cmtype = f[1], itype = f[2];
    uint32_t cmfirst = LE16(&f[3]), cmlen = LE16(&f[5]), cmbits = f[7];
    uint32_t w = LE16(&f[12]), h = LE16(&f[14]), bits = f[16], desc = f[17];
    bool rle = itype >= 8;
    uint32_t base = rle ? itype - 8 : itype;
    bool mapped = base == 1;
    if (cmtype > 1 || (base != 1 && base != 2 && base != 3) || (mapped != (cmtype == 1)) || w == 0 || h == 0) {
        err = "unsupported TGA";
        return false;
    }
    if (mapped ? !(bits == 8 && (cmbits == 15 || cmbits == 16 || cmbits == 24 || cmbits == 32))
               : base == 3 ? !(bits == 8 || bits == 16)
                           : !(bits == 15 || bits == 16 || bits == 24 || bits == 32)) {
        err = "unsupported TGA pixel format";
        return false;
    }
    {
        // stbi__tga_get_comp: the source components (palette entries for a
        // colour-mapped image) -> stb's size guard.
        const uint32_t eb = mapped ? cmbits : bits;
        const uint64_t comp = base == 3 ? (bits == 16 ? 2 : 1) : (eb == 32 ? 4 : 3);
        if (!StbSizesValid({w, h, comp})) { err = "too large"; return false; }
        if (!StbSizesValid({4, w, h})) { err = "outofmem"; return false; }   // the RGBA8 output
    }
    size_t pos = 18 + idlen;
    // A pixel (or palette entry) of `b` bits -> RGBA8; grey when `grey`.
    auto pixel = [](const uint8_t* p, uint32_t b, bool grey, uint8_t* o) {
        if (grey) {
            o[0] = o[1] = o[2] = p[0];
            o[3] = b == 16 ? p[1] : 255;
        } else if (b == 15 || b == 16) {
            uint32_t v = LE16(p);
            o[0] = Widen5((v >> 10) & 31u);
            o[1] = Widen5((v >> 5) & 31u);
            o[2] = Widen5(v & 31u);
            o[3] = 255;
        } else {
            o[0] = p[2]; o[1] = p[1]; o[2] = p[0];
            o[3] = b == 32 ? p[3] : 255;
        }
    };
    std::vector<uint8_t> pal;
    if (mapped) {
        // As stb: the colour-map origin is skipped as a byte count and indices
        // address the stored entries directly (origin 0 in practice), an index
        // past the map reading entry 0.
        pos += cmfirst;
        uint32_t eb = (cmbits + 7) / 8;
        if (cmlen == 0 || pos + (size_t)cmlen * eb > f.size()) { err = "truncated TGA palette"; return false; }
        pal.resize((size_t)cmlen * 4);
        for (uint32_t i = 0; i < cmlen; i++) pixel(&f[pos + (size_t)i * eb], cmbits, false, &pal[4 * (size_t)i]);
        pos += (size_t)cmlen * eb;
    } else if (cmtype == 1) {
        pos += (size_t)cmlen * ((cmbits + 7) / 8);
    }
    uint32_t pb = (bits + 7) / 8;
    size_t n = (size_t)w * h;
    std::vector<uint8_t> img(n * 4);
    auto decode = [&](const uint8_t* p, uint8_t* o) -> bool {
        if (!mapped) { pixel(p, bits, base == 3, o); return true; }
        uint32_t i = p[0] < cmlen ? p[0] : 0u;
        std::memcpy(o, &pal[4 * (size_t)i], 4);
        return true;
    };
    for (size_t k = 0; k < n;) {
        if (!rle) {
            if (pos + pb > f.size()) { err = "truncated TGA"; return false; }
            decode(&f[pos], &img[4 * k]);
            pos += pb;
            k++;
            continue;
        }
        if (pos >= f.size()) { err = "truncated TGA"; return false; }
        uint32_t hdr = f[pos++], count = (hdr & 127u) + 1;
        if (hdr & 128u) {   // run: one pixel repeated
            if (pos + pb > f.size()) { err = "truncated TGA"; return false; }
            uint8_t px[4];
            decode(&f[pos], px);
            pos += pb;
            for (uint32_t c = 0; c < count && k < n; c++, k++) std::memcpy(&img[4 * k], px, 4);
        } else {            // raw packet
            for (uint32_t c = 0; c < count && k < n; c++, k++) {
                if (pos + pb > f.size()) { err = "truncated TGA"; return false; }
                decode(&f[pos], &img[4 * k]);
                pos += pb;
            }
        }
    }
    W = (int)w;
    H = (int)h;
    rgba8.resize(n * 4);
    bool top_down = (desc & 0x20u) != 0;
    for (uint32_t y = 0; y < h; y++) {
        uint32_t sy = top_down ? y : h - 1 - y;
        std::memcpy(&rgba8[(size_t)y * w * 4], &img[(size_t)sy * w * 4], (size_t)w * 4);
    }
    return true;
}

// Widens an n-bit field (n <= 8) to 8 bits by bit replication, as stb_image's
// BMP reader does (stbi__shiftsigned: v * {0xff, 0x55, 0x49, 0x11, 0x21, 0x41,
// 0x81, 0x01}[n-1] >> {0, 0, 1, 0, 2, 4, 6, 0}[n-1]).
uint8_t WidenBits(uint32_t v, uint32_t n)
{
    static const uint32_t mul[9] = {0, 0xff, 0x55, 0x49, 0x11, 0x21, 0x41, 0x81, 0x01};
    static const uint32_t sh[9] = {0, 0, 0, 1, 0, 2, 4, 6, 0};
    return (uint8_t)((v * mul[n]) >> sh[n]);
}

// Windows BMP (stbi__bmp_load semantics): BITMAPCOREHEADER (12) and
// BITMAPINFOHEADER and its v2-v5 extensions (40, 52, 56, 108, 124);
// 1/4/8-bit palettes, 16/32-bit with bit-field masks (defaults 5-5-5 and
// 8-8-8 when uncompressed), 24-bit BGR; negative height = top-down rows;
// rows padded to 4 bytes.  A 32-bit image whose alpha is 0 everywhere gets
// alpha 255 (stb's all-zero-alpha rule).  RLE compression is not supported
// (stb rejects it too).
bool DecodeBMP(const std::vector<uint8_t>& f, int& W, int& H, std::vector<uint8_t>& rgba8, std::string& err)
{
    if (f.size() < 26 || f[0] != 'B' || f[1] != 'M') { err = "not a BMP"; return false; }
    uint32_t off = LE32(&f[10]), hsz = LE32(&f[14]);
    if (hsz != 12 && hsz != 40 && hsz != 52 && hsz != 56 && hsz != 108 && hsz != 124) { err = "unsupported BMP header"; return false; }
    if (f.size() < 14 + (size_t)hsz) { err = "truncated BMP"; return false; }
    int32_t w, h;
    uint32_t bpp, comp = 0;
    if (hsz == 12) {
        w = (int16_t)LE16(&f[18]);
        h = (int16_t)LE16(&f[20]);
        bpp = LE16(&f[24]);
    } else {
        w = (int32_t)LE32(&f[18]);
        h = (int32_t)LE32(&f[22]);
        bpp = LE16(&f[28]);
        comp = LE32(&f[30]);
    }
    bool top_down = h < 0;
    if (top_down) h = -h;
    if (w <= 0 || h <= 0 || w > (1 << 24) || h > (1 << 24)) { err = "bad BMP size"; return false; }
    if (!StbSizesValid({4, (uint64_t)w, (uint64_t)h})) { err = "too large"; return false; }
    if (comp != 0 && comp != 3) { err = "unsupported BMP compression"; return false; }
    if (bpp != 1 && bpp != 4 && bpp != 8 && bpp != 16 && bpp != 24 && bpp != 32) { err = "unsupported BMP depth"; return false; }
    uint32_t mr = 0, mg = 0, mb = 0, ma = 0;
    size_t pal_pos = 14 + (size_t)hsz;
    if (bpp == 16 || bpp == 32) {
        if (comp == 0) {
            if (bpp == 32) { mr = 0xffu << 16; mg = 0xffu << 8; mb = 0xffu; ma = 0xffu << 24; }
            else { mr = 31u << 10; mg = 31u << 5; mb = 31u; }
        } else if (hsz == 40) {   // BI_BITFIELDS: three masks after the header
            if (f.size() < 14 + 40 + 12) { err = "truncated BMP masks"; return false; }
            mr = LE32(&f[54]); mg = LE32(&f[58]); mb = LE32(&f[62]);
            pal_pos += 12;
        } else if (hsz >= 52) {
            mr = LE32(&f[54]); mg = LE32(&f[58]); mb = LE32(&f[62]);
            ma = hsz >= 56 ? LE32(&f[66]) : 0;
        } else {
            err = "BMP bit fields without masks";
            return false;
        }
        if (mr == 0 || mg == 0 || mb == 0) { err = "bad BMP masks"; return false; }
    }
    std::vector<uint8_t> pal;
    if (bpp <= 8) {
        uint32_t es = hsz == 12 ? 3 : 4;
        size_t entries = off > pal_pos ? (off - pal_pos) / es : 0;
        entries = std::min<size_t>(entries, 256);
        if (entries == 0 || pal_pos + entries * es > f.size()) { err = "bad BMP palette"; return false; }
        pal.resize(entries * 4);
        for (size_t i = 0; i < entries; i++) {
            const uint8_t* p = &f[pal_pos + i * es];
            pal[4 * i] = p[2]; pal[4 * i + 1] = p[1]; pal[4 * i + 2] = p[0]; pal[4 * i + 3] = 255;
        }
    }
    size_t stride = (((size_t)w * bpp + 31) / 32) * 4;
    if ((size_t)off + stride * (size_t)h > f.size()) { err = "truncated BMP pixels"; return false; }
    auto field = [](uint32_t v, uint32_t m) -> uint8_t {   // masked field -> 8 bits
        if (m == 0) return 255;
        uint32_t s = 0;
        while (!((m >> s) & 1u)) s++;
        uint32_t n = 0;
        while (s + n < 32 && ((m >> (s + n)) & 1u)) n++;
        uint32_t x = (v & m) >> s;
        if (n > 8) { x >>= n - 8; n = 8; }
        return WidenBits(x, n);
    };
    W = w;
    H = h;
    rgba8.assign((size_t)w * h * 4, 0);
    bool any_alpha = false;
    for (int32_t r = 0; r < h; r++) {
        const uint8_t* row = &f[off + stride * (size_t)r];
        int32_t y = top_down ? r : h - 1 - r;
        uint8_t* o = &rgba8[(size_t)y * w * 4];
        for (int32_t x = 0; x < w; x++, o += 4) {
            if (bpp <= 8) {
                uint32_t bit = (uint32_t)x * bpp;
                uint32_t i = (row[bit / 8] >> (8 - bpp - bit % 8)) & ((1u << bpp) - 1u);
                if (i < pal.size() / 4) std::memcpy(o, &pal[4 * (size_t)i], 4);
                else { o[0] = o[1] = o[2] = 0; o[3] = 255; }
            } else if (bpp == 24) {
                const uint8_t* p = &row[3 * (size_t)x];
                o[0] = p[2]; o[1] = p[1]; o[2] = p[0]; o[3] = 255;
            } else {
                uint32_t v = bpp == 16 ? LE16(&row[2 * (size_t)x]) : LE32(&row[4 * (size_t)x]);
                o[0] = field(v, mr); o[1] = field(v, mg); o[2] = field(v, mb);
                o[3] = field(v, ma);
                any_alpha |= ma != 0 && o[3] != 0;
            }
        }
    }
    if (bpp == 32 && ma != 0 && !any_alpha)
        for (size_t i = 3; i < rgba8.size(); i += 4) rgba8[i] = 255;
    return true;
}

// A byte stream with stbi__get8's end-of-data behaviour (0 past the end).
struct byte_reader {
    const std::vector<uint8_t>& f;
    size_t pos = 0;
    bool eof() const { return pos >= f.size(); }
    uint8_t get8() { return pos < f.size() ? f[pos++] : 0; }
    uint32_t get16le() { uint32_t a = get8(); return a | (uint32_t)get8() << 8; }
    void skip(size_t n) { pos = std::min(f.size(), pos + n); }
};

// Binary PNM (P5 grey / P6 RGB), as stbi__pnm_info / stbi__pnm_load
// (stb_image 2.29, the reference's copy): header integers separated by
// whitespace and '#' comments, the single byte after maxval ends the header;
// maxval only selects 8- or 16-bit samples (it does not scale them).  16-bit
// samples are read in host byte order and reduced by >> 8
// (stbi__convert_16_to_8), so the second byte of each big-endian sample is
// the result.  `matched` is false when the signature is not P5 / P6.
bool DecodePNM(const std::vector<uint8_t>& f, int& W, int& H, std::vector<uint8_t>& rgba8, std::string& err,
               bool& matched)
{
    byte_reader r{f};
    char p = (char)r.get8(), t = (char)r.get8();
    matched = p == 'P' && (t == '5' || t == '6');
    if (!matched) return false;
    const int comp = t == '6' ? 3 : 1;
    auto space = [](char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r'; };
    char c = (char)r.get8();
    auto skip_ws = [&]() {
        for (;;) {
            while (!r.eof() && space(c)) c = (char)r.get8();
            if (r.eof() || c != '#') break;
            while (!r.eof() && c != '\n' && c != '\r') c = (char)r.get8();
        }
    };
    bool overflow = false;
    auto integer = [&]() {
        int v = 0;
        while (!r.eof() && c >= '0' && c <= '9') {
            v = v * 10 + (c - '0');
            c = (char)r.get8();
            if (v > 214748364 || (v == 214748364 && c > '7')) { overflow = true; return 0; }
        }
        return v;
    };
    skip_ws();
    int w = integer();
    if (w == 0) { err = overflow ? "PNM header integer overflow" : "PNM: invalid width"; return false; }
    skip_ws();
    int h = integer();
    if (h == 0) { err = overflow ? "PNM header integer overflow" : "PNM: invalid height"; return false; }
    skip_ws();
    int maxv = integer();
    if (overflow) { err = "PNM header integer overflow"; return false; }
    if (maxv > 65535) { err = "PNM: max value > 65535"; return false; }
    const int bytes = maxv > 255 ? 2 : 1;
    if (w > (1 << 24) || h > (1 << 24) || !StbSizesValid({(uint64_t)comp, (uint64_t)w, (uint64_t)h, (uint64_t)bytes}) ||
        !StbSizesValid({4, (uint64_t)w, (uint64_t)h})) {
        err = "PNM: too large";
        return false;
    }
    const size_t n = (size_t)w * h;
    if (f.size() - std::min(f.size(), r.pos) < n * comp * bytes) { err = "PNM file truncated"; return false; }
    const uint8_t* d = f.data() + r.pos;
    W = w;
    H = h;
    rgba8.resize(n * 4);
    for (size_t i = 0; i < n; i++) {
        uint8_t v[3];
        for (int k = 0; k < comp; k++) v[k] = d[(i * comp + k) * bytes + (bytes - 1)];
        uint8_t* o = &rgba8[4 * i];
        o[0] = v[0];
        o[1] = comp == 3 ? v[1] : v[0];
        o[2] = comp == 3 ? v[2] : v[0];
        o[3] = 255;
    }
    return true;
}

// GIF, first frame only, as stbi_load gives it (stbi__gif_load ->
// stbi__gif_load_next once; stb_image 2.29).  Every behaviour below is that
// loader's: palettes with the graphic-control transparent entry at alpha 0
// (pixels of alpha <= 128 are not drawn and stay 0,0,0,0); the LZW stream
// must start with a clear code, table entries keep being added past 4096
// (up to 8192) at 12 bits; codes beyond the frame rectangle are dropped;
// interlaced frames walk rows 0,8,.. 4,.. 2,.. 1,..; and on the first frame,
// when the background index is not 0, the pixels the frame never touched
// take the global palette's background entry copied in its stored B,G,R
// order with alpha 255.
bool DecodeGIF(const std::vector<uint8_t>& f, int& W, int& H, std::vector<uint8_t>& rgba8, std::string& err)
{
    byte_reader r{f};
    if (r.get8() != 'G' || r.get8() != 'I' || r.get8() != 'F' || r.get8() != '8') { err = "not GIF"; return false; }
    uint8_t version = r.get8();
    if ((version != '7' && version != '9') || r.get8() != 'a') { err = "not GIF"; return false; }
    const uint32_t gw = r.get16le(), gh = r.get16le();
    const uint32_t flags = r.get8(), bgindex = r.get8();
    r.get8();   // aspect ratio
    if (gw > (1u << 24) || gh > (1u << 24) || !StbSizesValid({4, gw, gh})) { err = "GIF: too large"; return false; }
    uint8_t pal[256][4] = {}, lpal[256][4] = {};   // B, G, R, A as stb stores them
    auto colortable = [&](uint8_t (*t)[4], int entries, int transp) {
        for (int i = 0; i < entries; i++) {
            t[i][2] = r.get8();
            t[i][1] = r.get8();
            t[i][0] = r.get8();
            t[i][3] = transp == i ? 0 : 255;
        }
    };
    if (flags & 0x80) colortable(pal, 2 << (flags & 7), -1);
    const size_t pcount = (size_t)gw * gh;
    if (pcount == 0) { err = "GIF: empty image"; return false; }
    std::vector<uint8_t> out(4 * pcount, 0), history(pcount, 0);
    int transparent = -1;
    uint32_t eflags = 0;
    for (;;) {
        int tag = r.get8();
        if (tag == 0x2C) {   // image descriptor
            uint32_t x = r.get16le(), y = r.get16le(), w = r.get16le(), h = r.get16le();
            if (x + w > gw || y + h > gh) { err = "GIF: bad image descriptor"; return false; }
            const int64_t line = (int64_t)gw * 4;
            const int64_t start_x = (int64_t)x * 4, start_y = (int64_t)y * line;
            const int64_t max_x = start_x + (int64_t)w * 4, max_y = start_y + (int64_t)h * line;
            int64_t cur_x = start_x, cur_y = start_y;
            if (w == 0) cur_y = max_y;
            uint32_t lflags = r.get8();
            int64_t step;
            int parse;
            if (lflags & 0x40) { step = 8 * line; parse = 3; } else { step = line; parse = 0; }
            uint8_t (*table)[4];
            if (lflags & 0x80) {
                colortable(lpal, 2 << (lflags & 7), (eflags & 0x01) ? transparent : -1);
                table = lpal;
            } else if (flags & 0x80) {
                table = pal;
            } else {
                err = "GIF: missing color table";
                return false;
            }
            // stbi__process_gif_raster
            const uint32_t lzw_cs = r.get8();
            if (lzw_cs > 12) { err = "GIF: bad LZW code size"; return false; }
            struct code { int16_t prefix; uint8_t first, suffix; };
            std::vector<code> codes(8192);
            const int32_t clear = 1 << lzw_cs;
            for (int32_t i = 0; i < clear; i++) codes[(size_t)i] = {-1, (uint8_t)i, (uint8_t)i};
            bool first = true;
            int32_t codesize = (int32_t)lzw_cs + 1, codemask = (1 << codesize) - 1;
            int32_t avail = clear + 2, oldcode = -1, bits = 0, valid_bits = 0, len = 0;
            std::vector<uint8_t> chain;
            // stbi__out_gif_code: the code's string, prefix first.
            auto emit = [&](int32_t c) {
                chain.clear();
                for (int32_t k = c; k >= 0; k = codes[(size_t)k].prefix) chain.push_back(codes[(size_t)k].suffix);
                for (size_t j = chain.size(); j-- > 0;) {
                    if (cur_y >= max_y) return;
                    const int64_t idx = cur_x + cur_y;
                    history[(size_t)(idx / 4)] = 1;
                    const uint8_t* cc = table[chain[j]];
                    if (cc[3] > 128) {
                        uint8_t* o = &out[(size_t)idx];
                        o[0] = cc[2]; o[1] = cc[1]; o[2] = cc[0]; o[3] = cc[3];
                    }
                    cur_x += 4;
                    if (cur_x >= max_x) {
                        cur_x = start_x;
                        cur_y += step;
                        while (cur_y >= max_y && parse > 0) {
                            step = ((int64_t)1 << parse) * line;
                            cur_y = start_y + (step >> 1);
                            --parse;
                        }
                    }
                }
            };
            for (;;) {
                if (valid_bits < codesize) {
                    if (len == 0) {
                        len = r.get8();
                        if (len == 0) goto frame_done;
                    }
                    --len;
                    bits |= (int32_t)r.get8() << valid_bits;
                    valid_bits += 8;
                    continue;
                }
                int32_t c = bits & codemask;
                bits >>= codesize;
                valid_bits -= codesize;
                if (c == clear) {
                    codesize = (int32_t)lzw_cs + 1;
                    codemask = (1 << codesize) - 1;
                    avail = clear + 2;
                    oldcode = -1;
                    first = false;
                } else if (c == clear + 1) {   // end of information: skip the rest of the data
                    r.skip((size_t)len);
                    while ((len = r.get8()) > 0) r.skip((size_t)len);
                    goto frame_done;
                } else if (c <= avail) {
                    if (first) { err = "GIF: no clear code"; return false; }
                    if (oldcode >= 0) {
                        code& nc = codes[(size_t)avail++];
                        if (avail > 8192) { err = "GIF: too many codes"; return false; }
                        nc.prefix = (int16_t)oldcode;
                        nc.first = codes[(size_t)oldcode].first;
                        nc.suffix = (c == avail) ? nc.first : codes[(size_t)c].first;
                    } else if (c == avail) {
                        err = "GIF: illegal code in raster";
                        return false;
                    }
                    emit(c);
                    if ((avail & codemask) == 0 && avail <= 0x0FFF) {
                        codesize++;
                        codemask = (1 << codesize) - 1;
                    }
                    oldcode = c;
                } else {
                    err = "GIF: illegal code in raster";
                    return false;
                }
            }
        frame_done:
            if (bgindex > 0)
                for (size_t i = 0; i < pcount; i++)
                    if (!history[i]) {
                        pal[bgindex][3] = 255;
                        std::memcpy(&out[4 * i], pal[bgindex], 4);
                    }
            W = (int)gw;
            H = (int)gh;
            rgba8.swap(out);
            return true;
        } else if (tag == 0x21) {   // extension
            int ext = r.get8();
            if (ext == 0xF9) {   // graphic control
                int len = r.get8();
                if (len == 4) {
                    eflags = r.get8();
                    r.get16le();   // delay
                    if (transparent >= 0) pal[transparent][3] = 255;
                    if (eflags & 0x01) {
                        transparent = r.get8();
                        pal[transparent][3] = 0;
                    } else {
                        r.skip(1);
                        transparent = -1;
                    }
                } else {
                    r.skip((size_t)len);
                    continue;   // (stb leaves the sub-block terminator to the tag loop)
                }
            }
            int len;
            while ((len = r.get8()) != 0) r.skip((size_t)len);
        } else if (tag == 0x3B) {   // trailer before any frame
            err = "GIF: no image";
            return false;
        } else {
            err = "GIF: unknown block";
            return false;
        }
    }
}

// Photoshop PSD, the composited image, as stbi__psd_load at 8 bits per
// channel (stbi_loadf's path): RGB colour mode only, 8- or 16-bit samples
// (16-bit reduced to the high byte), raw or PackBits RLE planes (RLE is
// decoded as one byte per sample whatever the depth, as stb does), channels
// past the fourth ignored, missing ones filled with 0 (alpha 255); with four
// or more channels the "white matte" is removed from partly transparent
// pixels by stb's float expression v * (1/a) + 255 * (1 - 1/a), truncated to
// an integer and stored modulo 256.
bool DecodePSD(const std::vector<uint8_t>& f, int& W, int& H, std::vector<uint8_t>& rgba8, std::string& err)
{
    byte_reader r{f};
    auto get16be = [&]() { uint32_t a = r.get8(); return (a << 8) | r.get8(); };
    auto get32be = [&]() { uint32_t a = get16be(); return (a << 16) | get16be(); };
    if (get32be() != 0x38425053u) { err = "not PSD"; return false; }
    if (get16be() != 1) { err = "PSD: unsupported version"; return false; }
    r.skip(6);
    const int channels = (int)get16be();
    if (channels > 16) { err = "PSD: unsupported channel count"; return false; }
    const int32_t h = (int32_t)get32be(), w = (int32_t)get32be();
    if (h > (1 << 24) || w > (1 << 24) || h <= 0 || w <= 0) { err = "PSD: bad size"; return false; }
    if (!StbSizesValid({4, (uint64_t)w, (uint64_t)h})) { err = "PSD: too large"; return false; }
    const uint32_t depth = get16be();
    if (depth != 8 && depth != 16) { err = "PSD: bit depth is not 8 or 16"; return false; }
    if (get16be() != 3) { err = "PSD: not in RGB color mode"; return false; }
    r.skip(get32be());   // mode data
    r.skip(get32be());   // image resources
    r.skip(get32be());   // layer and mask information
    const uint32_t compression = get16be();
    if (compression > 1) { err = "PSD: unknown compression"; return false; }
    const size_t n = (size_t)w * h;
    if (!compression) {
        const size_t need = n * (size_t)std::min(channels, 4) * (depth == 16 ? 2 : 1);
        if (f.size() - std::min(f.size(), r.pos) < need) { err = "PSD: truncated image data"; return false; }
    } else if (f.size() - std::min(f.size(), r.pos) < (size_t)h * channels * 2) {
        err = "PSD: truncated RLE row counts";
        return false;
    }
    std::vector<uint8_t> out(4 * n);
    if (compression) {
        r.skip((size_t)h * channels * 2);   // per-row byte counts
        for (int ch = 0; ch < 4; ch++) {
            uint8_t* p = out.data() + ch;
            if (ch >= channels) {
                for (size_t i = 0; i < n; i++, p += 4) *p = ch == 3 ? 255 : 0;
                continue;
            }
            size_t count = 0;
            while (count < n) {
                const size_t nleft = n - count;
                uint32_t len = r.get8();
                if (len == 128) continue;
                if (len < 128) {
                    len++;
                    if (len > nleft) { err = "PSD: bad RLE data"; return false; }
                    count += len;
                    for (; len; len--, p += 4) *p = r.get8();
                } else {
                    len = 257 - len;
                    if (len > nleft) { err = "PSD: bad RLE data"; return false; }
                    const uint8_t v = r.get8();
                    count += len;
                    for (; len; len--, p += 4) *p = v;
                }
            }
        }
    } else {
        for (int ch = 0; ch < 4; ch++) {
            uint8_t* p = out.data() + ch;
            if (ch >= channels) {
                for (size_t i = 0; i < n; i++, p += 4) *p = ch == 3 ? 255 : 0;
            } else if (depth == 16) {
                for (size_t i = 0; i < n; i++, p += 4) *p = (uint8_t)(get16be() >> 8);
            } else {
                for (size_t i = 0; i < n; i++, p += 4) *p = r.get8();
            }
        }
    }
    if (channels >= 4)
        for (size_t i = 0; i < n; i++) {
            uint8_t* px = &out[4 * i];
            if (px[3] != 0 && px[3] != 255) {
                const float a = px[3] / 255.0f;
                const float ra = 1.0f / a;
                const float inv_a = 255.0f * (1 - ra);
                for (int k = 0; k < 3; k++) px[k] = (uint8_t)(int32_t)(px[k] * ra + inv_a);
            }
        }
    W = w;
    H = h;
    rgba8.swap(out);
    return true;
}

// The stb_image formats LoadTexture's stbi_loadf reads, in stbi__load_main's
// order for the signatures that could collide (PNG, BMP, GIF, PSD, JPEG, PNM;
// TGA, which has none, last).  JPEG: an SOI marker after any 0xFF fill.  Not
// read: Softimage PIC.
bool DecodeLDR(const std::vector<uint8_t>& f, int& W, int& H, std::vector<uint8_t>& rgba8, std::string& err)
{
    static const uint8_t png_sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (f.size() >= 8 && std::memcmp(f.data(), png_sig, 8) == 0) return DecodePNG(f, W, H, rgba8, err);
    if (f.size() >= 2 && f[0] == 'B' && f[1] == 'M') return DecodeBMP(f, W, H, rgba8, err);
    if (f.size() >= 6 && std::memcmp(f.data(), "GIF8", 4) == 0 && (f[4] == '7' || f[4] == '9') && f[5] == 'a')
        return DecodeGIF(f, W, H, rgba8, err);
    if (f.size() >= 4 && std::memcmp(f.data(), "8BPS", 4) == 0) return DecodePSD(f, W, H, rgba8, err);
    size_t k = 0;
    while (k < f.size() && f[k] == 0xFF) k++;
    if (k >= 1 && k < f.size() && f[k] == 0xD8) return DecodeJPEG(f, W, H, rgba8, err);
    bool pnm = false;
    if (DecodePNM(f, W, H, rgba8, err, pnm)) return true;
    if (pnm) return false;
    if (DecodeTGA(f, W, H, rgba8, err)) return true;
    if (err == "too large" || err == "outofmem") return false;   // a TGA header stb would also reject by size
    err = "unsupported image format (JPEG, PNG, BMP, GIF, PSD, PNM, TGA, Radiance HDR)";
    return false;
}

}  // namespace

bool LoadImageFloat(const char* Path, int& Width, int& Height, std::vector<vec4>& Pixels, std::string& Error)
{
    std::ifstream in(Path, std::ios::binary);
    if (!in) { Error = std::string("cannot open ") + Path; return false; }
    std::vector<uint8_t> f((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    if (f.size() >= 2 && f[0] == '#' && f[1] == '?') return DecodeHDR(f, Width, Height, Pixels, Error);
    std::vector<uint8_t> rgba8;
    if (!DecodeLDR(f, Width, Height, rgba8, Error)) return false;
    // stbi__ldr_to_hdr's float buffer (stbi__malloc_mad4(x, y, 4, sizeof(float))).
    if (!StbSizesValid({(uint64_t)Width, (uint64_t)Height, 4, sizeof(float)})) { Error = "outofmem"; return false; }
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
    return DecodeLDR(f, Width, Height, RGBA, Error);
}

}  // namespace pth
