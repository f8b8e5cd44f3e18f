// jpeg.cpp — JPEG decoding for LoadTexture (scene.cpp:294-313: stbi_loadf
// with 4 components).
//
// Baseline and progressive DCT JPEG (SOF0/1/2), 1, 3 or 4 components, any
// integer sampling factors, restart intervals, 8- and 16-bit quantisation
// tables, following ISO/IEC 10918-1 for the bitstream and stb_image's
// decoder (src/core/stb_image.h, vendored by the reference) for everything
// that decides the output bytes:
//   * the integer inverse DCT (stbi__idct_block, :2425-2523: IJG "islow"
//     with 12-bit constants, 2 extra bits between passes, +128 level shift
//     folded into the rounding bias);
//   * upsampling (load_jpeg_image :3898-3940 and the row resamplers
//     :3455-3526, 3645-3653): 1x1 copy, vertical 2x and horizontal 2x
//     triangle filters, the 2x2 triangle filter with "near" / "far" rows,
//     nearest neighbour for every other ratio;
//   * colour conversion: the reduced-precision fixed-point YCbCr->RGB of
//     stbi__YCbCr_to_RGB_row (:3656-3683), Adobe RGB / CMYK / YCCK
//     (:3941-3982, stbi__blinn_8x8 :3858-3862), grey replicated;
//   * tolerance of damaged streams: bits past a marker read as zeros, a
//     restart interval ending without an RST marker ends the scan, junk
//     after a scan is skipped, an unknown marker after the frame ends the
//     image with what has been decoded.
// The SSE2 kernels the reference's x64 build selects (stbi__idct_simd,
// stbi__YCbCr_to_RGB_simd, stbi__resample_row_hv_2_simd) are documented by
// stb as bit-identical to these scalar forms.  Parity with stb_image itself
// is unpinned: compiling the vendored sources was not authorised (DESIGN.md
// §2); tests/test_jpeg.py checks decoding against independent encodes.
#include "image.hpp"

#include <climits>
#include <cstring>

namespace pth {

namespace {

// Position in the 8x8 row-major block of the k-th coefficient in zigzag
// order (ISO/IEC 10918-1 Figure A.6), padded so that a corrupt run that
// walks past 63 stays inside the block.
const uint8_t kDezigzag[64 + 16] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

// Canonical Huffman table (Annex C): codes of each length are consecutive;
// `first[l]` is the first code of length l, `index[l]` the position of its
// symbol in `symbols`.
struct huffman {
    bool defined = false;
    int count[17] = {};
    int32_t first[17] = {}, last[17] = {};   // last = first + count - 1 (or -1)
    int index[17] = {};
    uint8_t symbols[256] = {};
    int n = 0;
};

bool BuildHuffman(huffman& h, const int* counts, const uint8_t* syms)
{
    int n = 0;
    for (int l = 1; l <= 16; l++) n += counts[l - 1];
    if (n > 256) return false;
    int32_t code = 0;
    int k = 0;
    for (int l = 1; l <= 16; l++) {
        h.count[l] = counts[l - 1];
        h.first[l] = code;
        h.index[l] = k;
        code += counts[l - 1];
        k += counts[l - 1];
        h.last[l] = code - 1;
        if (counts[l - 1] && code - 1 >= (1 << l)) return false;   // over-subscribed length
        code <<= 1;
    }
    std::memcpy(h.symbols, syms, (size_t)n);
    h.n = n;
    h.defined = true;
    return true;
}

struct component {
    int id = 0, h = 1, v = 1, tq = 0, td = 0, ta = 0;
    int dc_pred = 0;
    int x = 0, y = 0;        // effective size in samples
    int w2 = 0, h2 = 0;      // allocated size (whole MCUs)
    std::vector<uint8_t> data;
    std::vector<int16_t> coeff;   // progressive: (w2/8) x (h2/8) blocks of 64
    int coeff_w = 0;
};

int F2F(float x) { return (int)((x * 4096) + 0.5); }   // stbi__f2f: float product, double rounding bias
int F2Fixed(float x) { return ((int)(x * 4096.0f + 0.5f)) << 8; }   // stbi__float2fixed (all-float)

uint8_t Clamp255(int x) { return x < 0 ? 0 : x > 255 ? 255 : (uint8_t)x; }

// One 1-D pass of the IJG islow IDCT with stb's 12-bit constants.  Even part
// from s0, s2, s4, s6; odd part from s1, s3, s5, s7; outputs before the
// final butterfly: x0..x3 (even) and t0..t3 (odd).
struct idct1d {
    int x0, x1, x2, x3, t0, t1, t2, t3;
    idct1d(int s0, int s1, int s2, int s3, int s4, int s5, int s6, int s7)
    {
        static const int c0541 = F2F(0.5411961f), cm1847 = F2F(-1.847759065f), c0765 = F2F(0.765366865f);
        static const int c1175 = F2F(1.175875602f), c0298 = F2F(0.298631336f), c2053 = F2F(2.053119869f);
        static const int c3072 = F2F(3.072711026f), c1501 = F2F(1.501321110f), cm0899 = F2F(-0.899976223f);
        static const int cm2562 = F2F(-2.562915447f), cm1961 = F2F(-1.961570560f), cm0390 = F2F(-0.390180644f);
        int p1 = (s2 + s6) * c0541;
        int e2 = p1 + s6 * cm1847;
        int e3 = p1 + s2 * c0765;
        int e0 = (s0 + s4) * 4096;
        int e1 = (s0 - s4) * 4096;
        x0 = e0 + e3;
        x3 = e0 - e3;
        x1 = e1 + e2;
        x2 = e1 - e2;
        // odd part: inputs s7, s5, s3, s1 as t0..t3
        int a = s7 + s3, b = s5 + s1, c = s7 + s1, d = s5 + s3;
        int p5 = (a + b) * c1175;
        int o0 = s7 * c0298, o1 = s5 * c2053, o2 = s3 * c3072, o3 = s1 * c1501;
        int q1 = p5 + c * cm0899;
        int q2 = p5 + d * cm2562;
        int q3 = a * cm1961;
        int q4 = b * cm0390;
        t3 = o3 + (q1 + q4);
        t2 = o2 + (q2 + q3);
        t1 = o1 + (q2 + q4);
        t0 = o0 + (q1 + q3);
    }
};

void Idct8x8(uint8_t* out, int stride, const int16_t* blk)
{
    int tmp[64];
    for (int c = 0; c < 8; c++) {
        const int16_t* d = blk + c;
        int* v = tmp + c;
        if (!(d[8] | d[16] | d[24] | d[32] | d[40] | d[48] | d[56])) {
            int dc = d[0] * 4;
            for (int r = 0; r < 8; r++) v[8 * r] = dc;
            continue;
        }
        idct1d p(d[0], d[8], d[16], d[24], d[32], d[40], d[48], d[56]);
        int x0 = p.x0 + 512, x1 = p.x1 + 512, x2 = p.x2 + 512, x3 = p.x3 + 512;
        v[0] = (x0 + p.t3) >> 10;
        v[56] = (x0 - p.t3) >> 10;
        v[8] = (x1 + p.t2) >> 10;
        v[48] = (x1 - p.t2) >> 10;
        v[16] = (x2 + p.t1) >> 10;
        v[40] = (x2 - p.t1) >> 10;
        v[24] = (x3 + p.t0) >> 10;
        v[32] = (x3 - p.t0) >> 10;
    }
    for (int r = 0; r < 8; r++, out += stride) {
        const int* v = tmp + 8 * r;
        idct1d p(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
        const int bias = 65536 + (128 << 17);   // rounding + level shift
        int x0 = p.x0 + bias, x1 = p.x1 + bias, x2 = p.x2 + bias, x3 = p.x3 + bias;
        out[0] = Clamp255((x0 + p.t3) >> 17);
        out[7] = Clamp255((x0 - p.t3) >> 17);
        out[1] = Clamp255((x1 + p.t2) >> 17);
        out[6] = Clamp255((x1 - p.t2) >> 17);
        out[2] = Clamp255((x2 + p.t1) >> 17);
        out[5] = Clamp255((x2 - p.t1) >> 17);
        out[3] = Clamp255((x3 + p.t0) >> 17);
        out[4] = Clamp255((x3 - p.t0) >> 17);
    }
}

class decoder {
public:
    decoder(const std::vector<uint8_t>& f) : f_(f) {}
    bool Decode(int& W, int& H, std::vector<uint8_t>& rgba8, std::string& err);

private:
    const std::vector<uint8_t>& f_;
    size_t pos_ = 0;
    std::string err_;
    // frame
    int width_ = 0, height_ = 0, ncomp_ = 0;
    bool progressive_ = false;
    component comp_[4];
    int hmax_ = 1, vmax_ = 1, mcux_ = 0, mcuy_ = 0;
    uint16_t quant_[4][64] = {};   // row-major (de-zigzagged)
    huffman dc_[4], ac_[4];
    int restart_interval_ = 0;
    bool jfif_ = false;
    int adobe_transform_ = -1;
    int rgb_ids_ = 0;
    // scan
    int scan_n_ = 0, order_[4] = {};
    int ss_ = 0, se_ = 0, ah_ = 0, al_ = 0;
    int eob_run_ = 0, todo_ = 0;
    // entropy-coded bit reader
    uint32_t bits_ = 0;
    int nbits_ = 0;
    int marker_ = -1;   // marker met inside entropy-coded data (-1: none)
    bool nomore_ = false;

    bool Fail(const char* m) { err_ = m; return false; }
    bool Eof() const { return pos_ >= f_.size(); }
    int Byte() { return pos_ < f_.size() ? f_[pos_++] : 0; }
    int Word() { int a = Byte(); return (a << 8) | Byte(); }
    int NextMarker();
    bool Segment(int m);
    bool Frame(int m);
    bool ScanHeader();
    bool Scan();
    void Reset();
    void Fill();
    int Huff(const huffman& h);
    int Receive(int n);
    int Bits(int n);
    int Bit();
    bool BlockBaseline(int16_t* blk, int c);
    bool BlockDC(int16_t* blk, int c);
    bool BlockAC(int16_t* blk, const huffman& h);
    bool Restart();
    void Finish();
    void Output(std::vector<uint8_t>& rgba8);
};

// stbi__get_marker: a pending marker from the entropy-coded data, else the
// next 0xFF xx pair (fill bytes skipped); -1 when the next byte is not 0xFF.
int decoder::NextMarker()
{
    if (marker_ >= 0) { int m = marker_; marker_ = -1; return m; }
    int b = Byte();
    if (b != 0xFF) return -1;
    while (b == 0xFF) b = Byte();
    return b;
}

// Fills the bit buffer to more than 24 bits; 0xFF 0x00 is a stuffed 0xFF,
// 0xFF followed by anything else is a marker, after which zeros are read.
void decoder::Fill()
{
    do {
        uint32_t b = 0;
        if (!nomore_) {
            b = (uint32_t)Byte();
            if (b == 0xFF) {
                int c = Byte();
                while (c == 0xFF) c = Byte();
                if (c != 0) { marker_ = c; nomore_ = true; return; }
            }
        }
        bits_ |= b << (24 - nbits_);
        nbits_ += 8;
    } while (nbits_ <= 24);
}

// One Huffman symbol (Annex F.2.2.3), or -1 for an invalid code.
int decoder::Huff(const huffman& h)
{
    if (nbits_ < 16) Fill();
    for (int l = 1; l <= 16; l++) {
        int32_t code = (int32_t)(bits_ >> (32 - l));
        if (h.count[l] && code <= h.last[l]) {
            if (l > nbits_) return -1;
            bits_ <<= l;
            nbits_ -= l;
            return h.symbols[h.index[l] + (code - h.first[l])];
        }
    }
    nbits_ -= 16;   // no code of 16 bits or fewer matches
    return -1;
}

// RECEIVE + EXTEND (F.2.2.1): n magnitude bits as a signed value; 0 past the data.
int decoder::Receive(int n)
{
    if (nbits_ < n) Fill();
    if (nbits_ < n) return 0;
    uint32_t v = bits_ >> (32 - n);
    bits_ <<= n;
    nbits_ -= n;
    return (v >> (n - 1)) ? (int)v : (int)v - (1 << n) + 1;
}

int decoder::Bits(int n)
{
    if (nbits_ < n) Fill();
    if (nbits_ < n) return 0;
    uint32_t v = bits_ >> (32 - n);
    bits_ <<= n;
    nbits_ -= n;
    return (int)v;
}

int decoder::Bit() { return Bits(1); }

void decoder::Reset()
{
    bits_ = 0;
    nbits_ = 0;
    nomore_ = false;
    marker_ = -1;
    for (component& c : comp_) c.dc_pred = 0;
    eob_run_ = 0;
    todo_ = restart_interval_ ? restart_interval_ : 0x7fffffff;
}

// End of a restart interval: true to go on (an RSTn marker was found and the
// decoder state reset), false to end the scan (stb keeps the partial image).
bool decoder::Restart()
{
    if (--todo_ > 0) return true;
    if (nbits_ < 24) Fill();
    if (!(marker_ >= 0xD0 && marker_ <= 0xD7)) return false;
    Reset();
    return true;
}

// stb_image 2.29's corrupt-stream checks on the DC path (stbi__addints_valid,
// stbi__mul2shorts_valid): the predictor sum must fit an int and the
// dequantised (or point-transformed) DC value a short.
static bool AddIntsValid(int a, int b)
{
    if ((a >= 0) != (b >= 0)) return true;
    if (a < 0 && b < 0) return a >= INT_MIN - b;
    return a <= INT_MAX - b;
}

static bool Mul2ShortsValid(int a, int b)
{
    if (b == 0 || b == -1) return true;
    if ((a >= 0) == (b >= 0)) return a <= SHRT_MAX / b;
    if (b < 0) return a <= SHRT_MIN / b;
    return a >= SHRT_MIN / b;
}

bool decoder::BlockBaseline(int16_t* blk, int ci)
{
    component& c = comp_[ci];
    const uint16_t* q = quant_[c.tq];
    int t = Huff(dc_[c.td]);
    if (t < 0 || t > 15) return Fail("bad Huffman code (DC)");
    std::memset(blk, 0, 64 * sizeof(int16_t));
    int diff = t ? Receive(t) : 0;
    if (!AddIntsValid(c.dc_pred, diff)) return Fail("bad delta");
    c.dc_pred += diff;
    if (!Mul2ShortsValid(c.dc_pred, q[0])) return Fail("can't merge dc and ac");
    blk[0] = (int16_t)(c.dc_pred * q[0]);
    for (int k = 1; k < 64;) {
        int rs = Huff(ac_[c.ta]);
        if (rs < 0) return Fail("bad Huffman code (AC)");
        int r = rs >> 4, s = rs & 15;
        if (s == 0) {
            if (rs != 0xF0) break;   // EOB
            k += 16;
            continue;
        }
        k += r;
        int z = kDezigzag[k++];
        blk[z] = (int16_t)(Receive(s) * q[z]);
    }
    return true;
}

// Progressive DC scans (G.1.2.1): first scan with point transform Al, then
// one bit per refinement scan.
bool decoder::BlockDC(int16_t* blk, int ci)
{
    component& c = comp_[ci];
    if (se_ != 0) return Fail("DC and AC in one progressive scan");
    if (ah_ == 0) {
        std::memset(blk, 0, 64 * sizeof(int16_t));
        int t = Huff(dc_[c.td]);
        if (t < 0 || t > 15) return Fail("bad Huffman code (DC)");
        int diff = t ? Receive(t) : 0;
        if (!AddIntsValid(c.dc_pred, diff)) return Fail("bad delta");
        c.dc_pred += diff;
        if (!Mul2ShortsValid(c.dc_pred, 1 << al_)) return Fail("can't merge dc and ac");
        blk[0] = (int16_t)(c.dc_pred * (1 << al_));
    } else if (Bit()) {
        blk[0] = (int16_t)(blk[0] + (1 << al_));
    }
    return true;
}

// Progressive AC scans (G.1.2.2, G.1.2.3): spectral band [ss, se], first
// pass with end-of-band runs, refinement passes with correction bits.
bool decoder::BlockAC(int16_t* blk, const huffman& h)
{
    if (ss_ == 0) return Fail("DC and AC in one progressive scan");
    if (ah_ == 0) {
        if (eob_run_) { --eob_run_; return true; }
        for (int k = ss_; k <= se_;) {
            int rs = Huff(h);
            if (rs < 0) return Fail("bad Huffman code (AC)");
            int r = rs >> 4, s = rs & 15;
            if (s == 0) {
                if (r < 15) {
                    eob_run_ = (1 << r) - 1 + (r ? Bits(r) : 0);
                    break;
                }
                k += 16;
                continue;
            }
            k += r;
            blk[kDezigzag[k++]] = (int16_t)(Receive(s) * (1 << al_));
        }
        return true;
    }
    const int16_t bit = (int16_t)(1 << al_);
    auto refine = [&](int16_t& p) {
        if (Bit() && (p & bit) == 0) p = (int16_t)(p > 0 ? p + bit : p - bit);
    };
    if (eob_run_) {
        --eob_run_;
        for (int k = ss_; k <= se_; k++) {
            int16_t& p = blk[kDezigzag[k]];
            if (p != 0) refine(p);
        }
        return true;
    }
    int k = ss_;
    do {
        int rs = Huff(h);
        if (rs < 0) return Fail("bad Huffman code (AC)");
        int r = rs >> 4, s = rs & 15, val = 0;
        if (s == 0) {
            if (r < 15) {
                eob_run_ = (1 << r) - 1 + (r ? Bits(r) : 0);
                r = 64;   // the rest of the band only takes correction bits
            }
        } else {
            if (s != 1) return Fail("bad Huffman code (AC refinement)");
            val = Bit() ? bit : -bit;
        }
        while (k <= se_) {
            int16_t& p = blk[kDezigzag[k++]];
            if (p != 0) {
                refine(p);
            } else {
                if (r == 0) { p = (int16_t)val; break; }
                --r;
            }
        }
    } while (k <= se_);
    return true;
}

bool decoder::Scan()
{
    Reset();
    int16_t blk[64];
    if (scan_n_ == 1) {
        // Non-interleaved: the component's own blocks in raster order.
        component& c = comp_[order_[0]];
        int bw = (c.x + 7) >> 3, bh = (c.y + 7) >> 3;
        for (int j = 0; j < bh; j++)
            for (int i = 0; i < bw; i++) {
                if (!progressive_) {
                    if (!BlockBaseline(blk, order_[0])) return false;
                    Idct8x8(c.data.data() + (size_t)c.w2 * j * 8 + i * 8, c.w2, blk);
                } else {
                    int16_t* d = c.coeff.data() + 64 * ((size_t)i + (size_t)j * c.coeff_w);
                    if (!(ss_ == 0 ? BlockDC(d, order_[0]) : BlockAC(d, ac_[c.ta]))) return false;
                }
                if (!Restart()) return true;
            }
        return true;
    }
    // Interleaved MCUs: each component's h x v blocks in turn.
    for (int j = 0; j < mcuy_; j++)
        for (int i = 0; i < mcux_; i++) {
            for (int k = 0; k < scan_n_; k++) {
                component& c = comp_[order_[k]];
                for (int y = 0; y < c.v; y++)
                    for (int x = 0; x < c.h; x++) {
                        int bx = i * c.h + x, by = j * c.v + y;
                        if (!progressive_) {
                            if (!BlockBaseline(blk, order_[k])) return false;
                            Idct8x8(c.data.data() + (size_t)c.w2 * by * 8 + bx * 8, c.w2, blk);
                        } else {
                            int16_t* d = c.coeff.data() + 64 * ((size_t)bx + (size_t)by * c.coeff_w);
                            if (!BlockDC(d, order_[k])) return false;
                        }
                    }
            }
            if (!Restart()) return true;
        }
    return true;
}

// Progressive images: dequantise the accumulated coefficients and transform.
void decoder::Finish()
{
    if (!progressive_) return;
    int16_t blk[64];
    for (int n = 0; n < ncomp_; n++) {
        component& c = comp_[n];
        int bw = (c.x + 7) >> 3, bh = (c.y + 7) >> 3;
        for (int j = 0; j < bh; j++)
            for (int i = 0; i < bw; i++) {
                const int16_t* d = c.coeff.data() + 64 * ((size_t)i + (size_t)j * c.coeff_w);
                for (int k = 0; k < 64; k++) blk[k] = (int16_t)(d[k] * quant_[c.tq][k]);
                Idct8x8(c.data.data() + (size_t)c.w2 * j * 8 + i * 8, c.w2, blk);
            }
    }
}

bool decoder::Segment(int m)
{
    if (m == 0xDD) {   // DRI
        if (Word() != 4) return Fail("bad DRI length");
        restart_interval_ = Word();
        return true;
    }
    if (m == 0xDB) {   // DQT
        int L = Word() - 2;
        while (L > 0) {
            int pq = Byte(), p = pq >> 4, t = pq & 15;
            if (p > 1) return Fail("bad DQT precision");
            if (t > 3) return Fail("bad DQT table");
            for (int i = 0; i < 64; i++) quant_[t][kDezigzag[i]] = (uint16_t)(p ? Word() : Byte());
            L -= p ? 129 : 65;
        }
        return L == 0 ? true : Fail("bad DQT length");
    }
    if (m == 0xC4) {   // DHT
        int L = Word() - 2;
        while (L > 0) {
            int tc_th = Byte(), tc = tc_th >> 4, th = tc_th & 15;
            if (tc > 1 || th > 3) return Fail("bad DHT header");
            int counts[16], n = 0;
            for (int i = 0; i < 16; i++) n += counts[i] = Byte();
            if (n > 256) return Fail("bad DHT header");
            uint8_t syms[256];
            for (int i = 0; i < n; i++) syms[i] = (uint8_t)Byte();
            if (!BuildHuffman(tc ? ac_[th] : dc_[th], counts, syms)) return Fail("bad Huffman code lengths");
            L -= 17 + n;
        }
        return L == 0 ? true : Fail("bad DHT length");
    }
    if ((m >= 0xE0 && m <= 0xEF) || m == 0xFE) {   // APPn, COM
        int L = Word();
        if (L < 2) return Fail("bad APP/COM length");
        L -= 2;
        size_t start = pos_;
        if (m == 0xE0 && L >= 5) {
            jfif_ = jfif_ || (pos_ + 5 <= f_.size() && std::memcmp(&f_[pos_], "JFIF\0", 5) == 0);
        } else if (m == 0xEE && L >= 12 && pos_ + 12 <= f_.size() && std::memcmp(&f_[pos_], "Adobe\0", 6) == 0) {
            adobe_transform_ = f_[pos_ + 11];   // version (1), flags0 (2), flags1 (2), transform (1)
        }
        pos_ = start + (size_t)L;
        return true;
    }
    return Fail("unknown marker");
}

bool decoder::Frame(int m)
{
    progressive_ = m == 0xC2;
    int Lf = Word();
    if (Lf < 11) return Fail("bad SOF length");
    if (Byte() != 8) return Fail("only 8-bit JPEG is supported");
    height_ = Word();
    width_ = Word();
    if (height_ == 0) return Fail("JPEG with a delayed (DNL) height");
    if (width_ == 0) return Fail("zero JPEG width");
    if (width_ > (1 << 24) || height_ > (1 << 24)) return Fail("JPEG too large");
    ncomp_ = Byte();
    if (ncomp_ != 1 && ncomp_ != 3 && ncomp_ != 4) return Fail("bad JPEG component count");
    if (Lf != 8 + 3 * ncomp_) return Fail("bad SOF length");
    if (!StbSizesValid({(uint64_t)width_, (uint64_t)height_, (uint64_t)ncomp_})) return Fail("too large");
    // stbi_load's 4-component output buffer (stbi__malloc_mad3(4, x, y)).
    if (!StbSizesValid({4, (uint64_t)width_, (uint64_t)height_})) return Fail("outofmem");
    rgb_ids_ = 0;
    for (int i = 0; i < ncomp_; i++) {
        component& c = comp_[i];
        c.id = Byte();
        if (ncomp_ == 3 && c.id == "RGB"[i]) rgb_ids_++;
        int hv = Byte();
        c.h = hv >> 4;
        c.v = hv & 15;
        if (c.h < 1 || c.h > 4) return Fail("bad JPEG sampling factor H");
        if (c.v < 1 || c.v > 4) return Fail("bad JPEG sampling factor V");
        c.tq = Byte();
        if (c.tq > 3) return Fail("bad JPEG quantisation table index");
    }
    for (int i = 0; i < ncomp_; i++) {
        hmax_ = std::max(hmax_, comp_[i].h);
        vmax_ = std::max(vmax_, comp_[i].v);
    }
    for (int i = 0; i < ncomp_; i++)
        if (hmax_ % comp_[i].h || vmax_ % comp_[i].v) return Fail("non-integer JPEG sampling ratio");
    mcux_ = (width_ + hmax_ * 8 - 1) / (hmax_ * 8);
    mcuy_ = (height_ + vmax_ * 8 - 1) / (vmax_ * 8);
    for (int i = 0; i < ncomp_; i++) {
        component& c = comp_[i];
        c.x = (width_ * c.h + hmax_ - 1) / hmax_;
        c.y = (height_ * c.v + vmax_ - 1) / vmax_;
        c.w2 = mcux_ * c.h * 8;
        c.h2 = mcuy_ * c.v * 8;
        c.data.assign((size_t)c.w2 * c.h2, 0);
        if (progressive_) {
            c.coeff_w = c.w2 / 8;
            c.coeff.assign((size_t)c.w2 * c.h2, 0);
        }
    }
    return true;
}

bool decoder::ScanHeader()
{
    int Ls = Word();
    scan_n_ = Byte();
    if (scan_n_ < 1 || scan_n_ > 4 || scan_n_ > ncomp_) return Fail("bad SOS component count");
    if (Ls != 6 + 2 * scan_n_) return Fail("bad SOS length");
    for (int i = 0; i < scan_n_; i++) {
        int id = Byte(), t = Byte(), w = 0;
        while (w < ncomp_ && comp_[w].id != id) w++;
        if (w == ncomp_) return Fail("SOS names an unknown component");
        comp_[w].td = t >> 4;
        comp_[w].ta = t & 15;
        if (comp_[w].td > 3 || comp_[w].ta > 3) return Fail("bad SOS Huffman table index");
        order_[i] = w;
    }
    ss_ = Byte();
    se_ = Byte();
    int a = Byte();
    ah_ = a >> 4;
    al_ = a & 15;
    if (progressive_) {
        if (ss_ > 63 || se_ > 63 || ss_ > se_ || ah_ > 13 || al_ > 13) return Fail("bad progressive SOS");
    } else {
        if (ss_ != 0 || ah_ != 0 || al_ != 0) return Fail("bad SOS");
        se_ = 63;
    }
    for (int i = 0; i < scan_n_; i++) {
        const component& c = comp_[order_[i]];
        bool need_dc = !progressive_ || ss_ == 0, need_ac = !progressive_ || ss_ > 0;
        if ((need_dc && ah_ == 0 && !dc_[c.td].defined) || (need_ac && !ac_[c.ta].defined))
            return Fail("scan uses an undefined Huffman table");
    }
    return true;
}

// Upsampling to full resolution and colour conversion into RGBA8
// (load_jpeg_image with req_comp = 4).
void decoder::Output(std::vector<uint8_t>& rgba8)
{
    const int W = width_, H = height_;
    rgba8.assign((size_t)W * H * 4, 255);
    struct plane {
        int hs, vs, ystep, w, ypos;
        const uint8_t *line0, *line1;
        std::vector<uint8_t> buf;
    } pl[4];
    for (int k = 0; k < ncomp_; k++) {
        plane& p = pl[k];
        p.hs = hmax_ / comp_[k].h;
        p.vs = vmax_ / comp_[k].v;
        p.ystep = p.vs >> 1;
        p.w = (W + p.hs - 1) / p.hs;
        p.ypos = 0;
        p.line0 = p.line1 = comp_[k].data.data();
        p.buf.assign((size_t)W + 3, 0);
    }
    const uint8_t* row[4] = {};
    const bool is_rgb = ncomp_ == 3 && (rgb_ids_ == 3 || (adobe_transform_ == 0 && !jfif_));
    for (int j = 0; j < H; j++) {
        for (int k = 0; k < ncomp_; k++) {
            plane& p = pl[k];
            // The nearer source row is line1 in the lower half of an output
            // row pair (vs = 2), line0 in the upper half.
            bool bottom = p.ystep >= (p.vs >> 1);
            const uint8_t* near = bottom ? p.line1 : p.line0;
            const uint8_t* far = bottom ? p.line0 : p.line1;
            uint8_t* o = p.buf.data();
            const int w = p.w;
            if (p.hs == 1 && p.vs == 1) {
                row[k] = near;
            } else if (p.hs == 1 && p.vs == 2) {
                for (int i = 0; i < w; i++) o[i] = (uint8_t)((3 * near[i] + far[i] + 2) >> 2);
                row[k] = o;
            } else if (p.hs == 2 && p.vs == 1) {
                if (w == 1) {
                    o[0] = o[1] = near[0];
                } else {
                    o[0] = near[0];
                    o[1] = (uint8_t)((near[0] * 3 + near[1] + 2) >> 2);
                    int i = 1;
                    for (; i < w - 1; i++) {
                        int n = 3 * near[i] + 2;
                        o[2 * i] = (uint8_t)((n + near[i - 1]) >> 2);
                        o[2 * i + 1] = (uint8_t)((n + near[i + 1]) >> 2);
                    }
                    o[2 * i] = (uint8_t)((near[w - 2] * 3 + near[w - 1] + 2) >> 2);
                    o[2 * i + 1] = near[w - 1];
                }
                row[k] = o;
            } else if (p.hs == 2 && p.vs == 2) {
                if (w == 1) {
                    o[0] = o[1] = (uint8_t)((3 * near[0] + far[0] + 2) >> 2);
                } else {
                    int t1 = 3 * near[0] + far[0];
                    o[0] = (uint8_t)((t1 + 2) >> 2);
                    for (int i = 1; i < w; i++) {
                        int t0 = t1;
                        t1 = 3 * near[i] + far[i];
                        o[2 * i - 1] = (uint8_t)((3 * t0 + t1 + 8) >> 4);
                        o[2 * i] = (uint8_t)((3 * t1 + t0 + 8) >> 4);
                    }
                    o[2 * w - 1] = (uint8_t)((t1 + 2) >> 2);
                }
                row[k] = o;
            } else {
                for (int i = 0; i < w; i++)
                    for (int s = 0; s < p.hs; s++) o[i * p.hs + s] = near[i];
                row[k] = o;
            }
            if (++p.ystep >= p.vs) {
                p.ystep = 0;
                p.line0 = p.line1;
                if (++p.ypos < comp_[k].y) p.line1 += comp_[k].w2;
            }
        }
        uint8_t* out = &rgba8[(size_t)j * W * 4];
        auto ycc = [&](int i, uint8_t* px) {
            // stbi__YCbCr_to_RGB_row: 12-bit constants << 8, Cb's green term
            // truncated to its upper 16 bits, >> 20.
            static const int kr = F2Fixed(1.40200f), kg = -F2Fixed(0.71414f), kgb = -F2Fixed(0.34414f),
                             kb = F2Fixed(1.77200f);
            int y = (row[0][i] << 20) + (1 << 19);
            int cr = row[2][i] - 128, cb = row[1][i] - 128;
            px[0] = Clamp255((y + cr * kr) >> 20);
            px[1] = Clamp255((y + cr * kg + ((cb * kgb) & (int)0xffff0000)) >> 20);
            px[2] = Clamp255((y + cb * kb) >> 20);
        };
        auto blinn = [](int x, int y) { unsigned t = (unsigned)(x * y + 128); return (uint8_t)((t + (t >> 8)) >> 8); };
        for (int i = 0; i < W; i++) {
            uint8_t* px = out + 4 * i;
            if (ncomp_ == 1) {
                px[0] = px[1] = px[2] = row[0][i];
            } else if (ncomp_ == 3) {
                if (is_rgb) { px[0] = row[0][i]; px[1] = row[1][i]; px[2] = row[2][i]; }
                else ycc(i, px);
            } else if (adobe_transform_ == 0) {   // CMYK
                uint8_t m = row[3][i];
                px[0] = blinn(row[0][i], m);
                px[1] = blinn(row[1][i], m);
                px[2] = blinn(row[2][i], m);
            } else if (adobe_transform_ == 2) {   // YCCK
                ycc(i, px);
                uint8_t m = row[3][i];
                px[0] = blinn(255 - px[0], m);
                px[1] = blinn(255 - px[1], m);
                px[2] = blinn(255 - px[2], m);
            } else {                              // YCbCr + a fourth channel, ignored
                ycc(i, px);
            }
            px[3] = 255;
        }
    }
}

bool decoder::Decode(int& W, int& H, std::vector<uint8_t>& rgba8, std::string& err)
{
    auto fail = [&](const std::string& m) { err = "JPEG: " + m; return false; };
    if (NextMarker() != 0xD8) return fail("no SOI marker");
    int m = NextMarker();
    while (!(m == 0xC0 || m == 0xC1 || m == 0xC2)) {
        if (m < 0) return fail("expected a marker");
        if (!Segment(m)) return fail(err_);
        m = NextMarker();
        while (m < 0) {   // padding between segments
            if (Eof()) return fail("no SOF marker");
            m = NextMarker();
        }
    }
    if (!Frame(m)) return fail(err_);
    m = NextMarker();
    while (m != 0xD9) {
        if (m == 0xDA) {   // SOS
            if (!ScanHeader()) return fail(err_);
            if (!Scan()) return fail(err_);
            if (marker_ < 0) {
                // Junk after the entropy-coded data: skip to what looks like
                // a marker (0xFF followed by neither 0x00 nor 0xFF).
                while (!Eof()) {
                    int x = Byte();
                    while (x == 0xFF) {
                        if (Eof()) break;
                        x = Byte();
                        if (x != 0x00 && x != 0xFF) { marker_ = x; break; }
                    }
                    if (marker_ >= 0) break;
                }
            }
            m = NextMarker();
            if (m >= 0xD0 && m <= 0xD7) m = NextMarker();
        } else if (m == 0xDC) {   // DNL
            int Ld = Word(), NL = Word();
            if (Ld != 4) return fail("bad DNL length");
            if (NL != height_) return fail("bad DNL height");
            m = NextMarker();
        } else {
            // Any other marker is a table / APP segment; anything else --
            // an unknown marker, no marker, the end of the file -- ends the
            // image with what has been decoded, as stb does (which then also
            // skips the final dequantisation of a progressive image and
            // returns uninitialised planes; here the coefficients decoded so
            // far are transformed).
            if (m < 0 || !Segment(m)) break;
            m = NextMarker();
        }
    }
    Finish();
    Output(rgba8);
    W = width_;
    H = height_;
    return true;
}

}  // namespace

bool DecodeJPEG(const std::vector<uint8_t>& f, int& W, int& H, std::vector<uint8_t>& rgba8, std::string& err)
{
    decoder d(f);
    return d.Decode(W, H, rgba8, err);
}

}  // namespace pth
