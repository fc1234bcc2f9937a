// pf_jpeg.cpp -- the JPEG codec either side of the fusion path.
//
// Decoder.  The reference decodes its depth-net tiles (LeReS writes JPEG, Main.cpp:576-578) and
// some baselines (`.jpg`, `.unifuse.jpg`, Main.cpp:499-510) with stb_image v2.23 (stbi_load,
// req_comp 0, Depth.cpp:85-100 and :331-351).  This decoder is written against ITU T.81 --
// baseline, extended-sequential and progressive Huffman DCT, 8-bit samples, 1 / 3 / 4
// components, sampling factors 1..4, restart intervals, interleaved and single-component scans --
// and reproduces the sample arithmetic stb's loader uses, so its output is the reference's
// bit for bit (tests/test_codecs_stb.py, tests/golden/stb_codecs.npz):
//   * coefficients are 16-bit: baseline values are dequantised as they are decoded,
//     (int16)(v * q); progressive values are kept as (int16)(v << Al), refined in place and
//     dequantised after the last scan with the same 16-bit product;
//   * the inverse DCT is the 12-bit fixed-point "islow" factorisation with stb's constants
//     (each rounded as (int)(c * 4096 + 0.5), truncating toward zero for the negative ones),
//     2 extra bits after the column pass and a rounded 17-bit shift with the +128 level shift
//     folded in after the row pass;
//   * chroma is upsampled with stb's centred filters: h2v1 and h1v2 3:1 triangles, h2v2 the
//     3:1 x 3:1 separable triangle (rounding +8 >> 4), replication for other factors, walking
//     the component rows with stb's near/far row state;
//   * YCbCr -> RGB in stb's reduced-precision fixed point (constants (int)(c * 4096 + 0.5) << 8,
//     the Cb term of green masked to its high 16 bits, >> 20), Adobe CMYK / YCCK through stb's
//     rounded 8x8-bit products, RGB-tagged (component ids 'R','G','B', or APP14 transform 0
//     without JFIF) passed through;
//   * channels as stbi_load(req_comp 0) reports them: 1 for gray, 3 otherwise.
// Arithmetic coding, lossless and 12-bit files fail to load, as they do in stb.
//
// Encoder.  The reference writes each rendered tile with stbi_write_jpg (stb_image_write v1.15,
// Main.cpp:319-320: vertical flip on write, quality = width*3).  encode_jpeg produces stb's
// bytes: its header layout (JFIF APP0, one DQT with both tables, SOF0 with three components, one
// DHT with the four Annex K tables, SOS), the Annex K quantisers scaled by the IJG quality rule,
// 4:2:0 with 2x2 averaging at quality <= 90 and 4:4:4 above, the float AAN forward DCT with the
// reciprocal AAN-scaled quantisers, rounding (int)(v +- 0.5f), and its bit packing.
#include "pf_image.hpp"

#include <cmath>
#include <cstdio>
#include <cstring>

namespace pfio {

namespace {

// natural (row-major) index of the k-th coefficient in zig-zag order (T.81 Figure A.6)
const uint8_t kZig[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                          12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                          35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                          58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// ============================================================================================
// Decoder
// ============================================================================================

// Canonical Huffman table (T.81 Annex C / F.2.2.3) with a 9-bit lookahead.
struct HuffDec {
    bool present = false;
    int mincode[17] = {}, maxcode[18] = {}, valptr[17] = {};
    uint8_t vals[256] = {};
    uint8_t fast_len[512] = {}, fast_val[512] = {};

    bool build(const uint8_t* counts, const uint8_t* v, int n)
    {
        present = false;
        std::memcpy(vals, v, n);
        std::memset(fast_len, 0, sizeof(fast_len));
        int code = 0, k = 0;
        for (int l = 1; l <= 16; ++l) {
            valptr[l] = k;
            mincode[l] = code;
            if (code + counts[l - 1] > (1 << l)) return false;  // over-full code space
            for (int i = 0; i < counts[l - 1]; ++i, ++k, ++code)
                if (l <= 9)
                    for (int j = 0; j < (1 << (9 - l)); ++j) {
                        fast_len[(code << (9 - l)) + j] = (uint8_t)l;
                        fast_val[(code << (9 - l)) + j] = v[k];
                    }
            maxcode[l] = counts[l - 1] ? code - 1 : -1;
            code <<= 1;
        }
        maxcode[17] = 0x7FFFFFFF;
        return present = true;
    }
};

// Entropy-coded segment reader: removes byte stuffing, stops at a marker (and then supplies
// zero bits, as decoders do at the end of a truncated scan).
struct BitReader {
    const uint8_t* p = nullptr;
    const uint8_t* end = nullptr;
    uint32_t acc = 0;
    int n = 0;
    int marker = -1;  // the marker that ended the segment

    void refill()
    {
        while (n <= 24) {
            uint32_t byte = 0;
            if (marker < 0 && p < end) {
                if (*p == 0xFF) {
                    const uint8_t* q = p + 1;
                    while (q < end && *q == 0xFF) ++q;  // fill bytes
                    if (q >= end || *q == 0x00) {  // stuffed 0xFF (or 0xFF at the very end)
                        byte = 0xFF;
                        p = q < end ? q + 1 : end;
                    } else {
                        marker = *q;
                        p = q + 1;
                    }
                } else {
                    byte = *p++;
                }
            }
            acc |= byte << (24 - n);
            n += 8;
        }
    }
    int bits(int k)
    {
        if (k == 0) return 0;
        refill();
        const int v = (int)(acc >> (32 - k));
        acc <<= k;
        n -= k;
        return v;
    }
    int bit() { return bits(1); }
    int symbol(const HuffDec& h)
    {
        refill();
        const int look = (int)(acc >> 23);
        if (h.fast_len[look]) {
            acc <<= h.fast_len[look];
            n -= h.fast_len[look];
            return h.fast_val[look];
        }
        for (int l = 10; l <= 16; ++l) {
            const int code = (int)(acc >> (32 - l));
            if (h.maxcode[l] >= 0 && code <= h.maxcode[l] && code >= h.mincode[l]) {
                acc <<= l;
                n -= l;
                return h.vals[h.valptr[l] + code - h.mincode[l]];
            }
        }
        return -1;
    }
    // RECEIVE + EXTEND (T.81 F.2.2.1)
    int received(int s)
    {
        const int v = bits(s);
        return (s && v < (1 << (s - 1))) ? v - (1 << s) + 1 : v;
    }
    void restart()
    {
        acc = 0;
        n = 0;
        marker = -1;
    }
};

struct Comp {
    int id = 0, h = 1, v = 1, tq = 0, td = 0, ta = 0;
    int x = 0, y = 0;        // samples carrying image content
    int bw = 0, bh = 0;      // block grid of the MCU-padded plane
    int w2 = 0;              // plane stride (bw * 8)
    int dc_pred = 0;
    std::vector<int16_t> coef;  // bw * bh blocks of 64 (natural order)
    std::vector<uint8_t> plane; // w2 x bh*8 samples
};

// 1-D pass of the fixed-point islow IDCT: constants scaled by 4096 and rounded the way stb's
// loader rounds them (through double, truncated toward zero).
constexpr int fix12(float c) { return (int)((double)(c * 4096.0f) + 0.5); }
struct Pass {
    int x0, x1, x2, x3, t0, t1, t2, t3;
};
inline Pass idct_1d(int s0, int s1, int s2, int s3, int s4, int s5, int s6, int s7)
{
    Pass o;
    // even part
    const int z1 = (s2 + s6) * fix12(0.5411961f);
    const int e2 = z1 + s6 * fix12(-1.847759065f);
    const int e3 = z1 + s2 * fix12(0.765366865f);
    const int e0 = (s0 + s4) * 4096, e1 = (s0 - s4) * 4096;
    o.x0 = e0 + e3;
    o.x3 = e0 - e3;
    o.x1 = e1 + e2;
    o.x2 = e1 - e2;
    // odd part (inputs in reverse order: s7, s5, s3, s1)
    int a = s7, b = s5, c = s3, d = s1;
    int q3 = a + c, q4 = b + d, q1 = a + d, q2 = b + c;
    const int z5 = (q3 + q4) * fix12(1.175875602f);
    a *= fix12(0.298631336f);
    b *= fix12(2.053119869f);
    c *= fix12(3.072711026f);
    d *= fix12(1.501321110f);
    q1 = z5 + q1 * fix12(-0.899976223f);
    q2 = z5 + q2 * fix12(-2.562915447f);
    q3 *= fix12(-1.961570560f);
    q4 *= fix12(-0.390180644f);
    o.t3 = d + (q1 + q4);
    o.t2 = c + (q2 + q3);
    o.t1 = b + (q2 + q4);
    o.t0 = a + (q1 + q3);
    return o;
}

inline uint8_t clamp255(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

void idct_block(const int16_t* in, uint8_t* out, int stride)
{
    int mid[64];
    for (int col = 0; col < 8; ++col) {
        const int16_t* s = in + col;
        int* m = mid + col;
        bool ac_zero = true;
        for (int r = 1; r < 8; ++r) ac_zero = ac_zero && s[8 * r] == 0;
        if (ac_zero) {  // flat column: only the DC term, with the pass's 2 extra bits
            for (int r = 0; r < 8; ++r) m[8 * r] = s[0] * 4;
            continue;
        }
        Pass p = idct_1d(s[0], s[8], s[16], s[24], s[32], s[40], s[48], s[56]);
        p.x0 += 512; p.x1 += 512; p.x2 += 512; p.x3 += 512;
        m[0] = (p.x0 + p.t3) >> 10;  m[56] = (p.x0 - p.t3) >> 10;
        m[8] = (p.x1 + p.t2) >> 10;  m[48] = (p.x1 - p.t2) >> 10;
        m[16] = (p.x2 + p.t1) >> 10; m[40] = (p.x2 - p.t1) >> 10;
        m[24] = (p.x3 + p.t0) >> 10; m[32] = (p.x3 - p.t0) >> 10;
    }
    const int bias = 65536 + (128 << 17);  // rounding of the 17-bit shift + level shift
    for (int row = 0; row < 8; ++row) {
        const int* m = mid + 8 * row;
        Pass p = idct_1d(m[0], m[1], m[2], m[3], m[4], m[5], m[6], m[7]);
        p.x0 += bias; p.x1 += bias; p.x2 += bias; p.x3 += bias;
        uint8_t* o = out + row * stride;
        o[0] = clamp255((p.x0 + p.t3) >> 17); o[7] = clamp255((p.x0 - p.t3) >> 17);
        o[1] = clamp255((p.x1 + p.t2) >> 17); o[6] = clamp255((p.x1 - p.t2) >> 17);
        o[2] = clamp255((p.x2 + p.t1) >> 17); o[5] = clamp255((p.x2 - p.t1) >> 17);
        o[3] = clamp255((p.x3 + p.t0) >> 17); o[4] = clamp255((p.x3 - p.t0) >> 17);
    }
}

// ---- centred upsampling of one component row (w samples -> hs*w) from its nearer and farther
// source rows.  Returns the row to read (the near row itself when nothing is interpolated). ----
const uint8_t* up_none(uint8_t*, const uint8_t* near, const uint8_t*, int, int) { return near; }

const uint8_t* up_v2(uint8_t* out, const uint8_t* near, const uint8_t* far, int w, int)
{
    for (int i = 0; i < w; ++i) out[i] = (uint8_t)((3 * near[i] + far[i] + 2) >> 2);
    return out;
}

const uint8_t* up_h2(uint8_t* out, const uint8_t* near, const uint8_t*, int w, int)
{
    if (w == 1) {
        out[0] = out[1] = near[0];
        return out;
    }
    out[0] = near[0];
    out[1] = (uint8_t)((near[0] * 3 + near[1] + 2) >> 2);
    int i = 1;
    for (; i < w - 1; ++i) {
        const int c3 = 3 * near[i] + 2;
        out[2 * i] = (uint8_t)((c3 + near[i - 1]) >> 2);
        out[2 * i + 1] = (uint8_t)((c3 + near[i + 1]) >> 2);
    }
    out[2 * i] = (uint8_t)((near[w - 2] * 3 + near[w - 1] + 2) >> 2);
    out[2 * i + 1] = near[w - 1];
    return out;
}

const uint8_t* up_hv2(uint8_t* out, const uint8_t* near, const uint8_t* far, int w, int)
{
    if (w == 1) {
        out[0] = out[1] = (uint8_t)((3 * near[0] + far[0] + 2) >> 2);
        return out;
    }
    int cur = 3 * near[0] + far[0];  // vertically filtered column sums (x4)
    out[0] = (uint8_t)((cur + 2) >> 2);
    for (int i = 1; i < w; ++i) {
        const int prev = cur;
        cur = 3 * near[i] + far[i];
        out[2 * i - 1] = (uint8_t)((3 * prev + cur + 8) >> 4);
        out[2 * i] = (uint8_t)((3 * cur + prev + 8) >> 4);
    }
    out[2 * w - 1] = (uint8_t)((cur + 2) >> 2);
    return out;
}

const uint8_t* up_replicate(uint8_t* out, const uint8_t* near, const uint8_t*, int w, int hs)
{
    for (int i = 0; i < w; ++i)
        for (int j = 0; j < hs; ++j) out[i * hs + j] = near[i];
    return out;
}

// YCbCr -> RGB in the loader's reduced-precision fixed point
constexpr int fix20(float c) { return ((int)(c * 4096.0f + 0.5f)) << 8; }
inline void ycc_to_rgb(int Y, int Cb, int Cr, uint8_t* o)
{
    const int yf = (Y << 20) + (1 << 19);
    const int cr = Cr - 128, cb = Cb - 128;
    int r = yf + cr * fix20(1.40200f);
    int g = yf + (cr * -fix20(0.71414f)) + ((int)((unsigned)(cb * -fix20(0.34414f)) & 0xFFFF0000u));
    int b = yf + cb * fix20(1.77200f);
    o[0] = clamp255(r >> 20);
    o[1] = clamp255(g >> 20);
    o[2] = clamp255(b >> 20);
}

// x * y / 255, rounded (the loader's CMYK arithmetic)
inline uint8_t mul255(uint8_t x, uint8_t y)
{
    const unsigned t = (unsigned)x * y + 128;
    return (uint8_t)((t + (t >> 8)) >> 8);
}

class Decoder {
public:
    bool run(const std::vector<uint8_t>& file, Image& out, std::string& err);

private:
    const uint8_t* f_ = nullptr;
    size_t size_ = 0, pos_ = 0;
    uint16_t q_[4][64] = {};
    HuffDec dc_[4], ac_[4];
    std::vector<Comp> comps_;
    int W_ = 0, H_ = 0, hmax_ = 1, vmax_ = 1, mcux_ = 0, mcuy_ = 0;
    int restart_ = 0;
    bool progressive_ = false, jfif_ = false;
    int adobe_transform_ = -1;
    int rgb_ids_ = 0;
    std::string* err_ = nullptr;

    bool fail(const char* m)
    {
        *err_ = std::string("JPEG: ") + m;
        return false;
    }
    int u16(size_t i) const { return f_[i] << 8 | f_[i + 1]; }
    bool frame(size_t seg, size_t lf);  // lf: the segment's length field (T.81 B.2.2)
    bool scan(size_t seg, size_t ls, BitReader& br);
    void finish();
    bool output(Image& out);
};

bool Decoder::frame(size_t seg, size_t len)
{
    if (len < 11) return fail("bad SOF length");
    if (f_[seg] != 8) return fail("only 8-bit samples are supported");
    H_ = u16(seg + 1);
    W_ = u16(seg + 3);
    const int nc = f_[seg + 5];
    if (H_ == 0) return fail("no header height");
    if (W_ == 0) return fail("zero width");
    if (nc != 1 && nc != 3 && nc != 4) return fail("bad component count");
    if (len != 8 + 3 * (size_t)nc) return fail("bad SOF length");
    if ((long long)W_ * H_ * nc > (1ll << 30)) return fail("image too large");
    comps_.assign(nc, Comp());
    rgb_ids_ = 0;
    for (int k = 0; k < nc; ++k) {
        Comp& c = comps_[k];
        c.id = f_[seg + 6 + 3 * k];
        if (nc == 3 && c.id == "RGB"[k]) ++rgb_ids_;
        c.h = f_[seg + 7 + 3 * k] >> 4;
        c.v = f_[seg + 7 + 3 * k] & 15;
        c.tq = f_[seg + 8 + 3 * k];
        if (c.h < 1 || c.h > 4 || c.v < 1 || c.v > 4) return fail("bad sampling factor");
        if (c.tq > 3) return fail("bad quantisation table selector");
        hmax_ = std::max(hmax_, c.h);
        vmax_ = std::max(vmax_, c.v);
    }
    mcux_ = (W_ + 8 * hmax_ - 1) / (8 * hmax_);
    mcuy_ = (H_ + 8 * vmax_ - 1) / (8 * vmax_);
    for (Comp& c : comps_) {
        c.x = (W_ * c.h + hmax_ - 1) / hmax_;
        c.y = (H_ * c.v + vmax_ - 1) / vmax_;
        c.bw = mcux_ * c.h;
        c.bh = mcuy_ * c.v;
        c.w2 = c.bw * 8;
        c.coef.assign((size_t)c.bw * c.bh * 64, 0);
    }
    return true;
}

// One scan (T.81 B.2.3 header + its entropy-coded segment, F.2 / G.1.2).
bool Decoder::scan(size_t seg, size_t len, BitReader& br)
{
    const int ns = f_[seg];
    if (ns < 1 || ns > 4 || ns > (int)comps_.size()) return fail("bad SOS component count");
    if (len != 6 + 2 * (size_t)ns) return fail("bad SOS length");
    std::vector<Comp*> sc;
    for (int k = 0; k < ns; ++k) {
        const int cid = f_[seg + 1 + 2 * k], tbl = f_[seg + 2 + 2 * k];
        Comp* c = nullptr;
        for (Comp& x : comps_)
            if (x.id == cid) c = &x;
        if (!c) return fail("scan names an unknown component");
        c->td = tbl >> 4;
        c->ta = tbl & 15;
        if (c->td > 3 || c->ta > 3) return fail("bad Huffman table selector");
        sc.push_back(c);
    }
    const int ss = f_[seg + 1 + 2 * ns], se = f_[seg + 2 + 2 * ns];
    const int ah = f_[seg + 3 + 2 * ns] >> 4, al = f_[seg + 3 + 2 * ns] & 15;
    if (progressive_) {
        if (ss > 63 || se > 63 || ss > se || ah > 13 || al > 13) return fail("bad progressive SOS");
        if ((ss == 0) != (se == 0)) return fail("a scan mixes DC and AC");
    } else if (ss != 0 || ah != 0 || al != 0) {
        return fail("bad sequential SOS");
    }
    for (Comp* c : sc) {
        const bool dc_needed = !progressive_ || (ss == 0 && ah == 0);
        const bool ac_needed = !progressive_ || ss > 0;
        if (dc_needed && !dc_[c->td].present) return fail("missing DC table");
        if (ac_needed && !ac_[c->ta].present) return fail("missing AC table");
    }

    int eobrun = 0;
    // decode one block of component c at block (bx, by)
    auto block = [&](Comp& c, int bx, int by) -> bool {
        int16_t* d = &c.coef[((size_t)by * c.bw + bx) * 64];
        if (!progressive_) {  // sequential: dequantised as decoded
            const uint16_t* q = q_[c.tq];
            const int t = br.symbol(dc_[c.td]);
            if (t < 0 || t > 16) return fail("corrupt DC code");
            c.dc_pred += br.received(t);
            d[0] = (int16_t)(c.dc_pred * q[0]);
            for (int k = 1; k < 64;) {
                const int rs = br.symbol(ac_[c.ta]);
                if (rs < 0) return fail("corrupt AC code");
                const int r = rs >> 4, s = rs & 15;
                if (s == 0) {
                    if (rs != 0xF0) break;  // EOB
                    k += 16;
                    continue;
                }
                k += r;
                const int z = kZig[k < 63 ? k : 63];  // a run past the block lands on 63
                d[z] = (int16_t)(br.received(s) * q[z]);
                ++k;
            }
            return true;
        }
        if (ss == 0) {  // DC scans
            if (ah == 0) {  // the first DC scan starts the block afresh
                std::memset(d, 0, 64 * sizeof(int16_t));
                const int t = br.symbol(dc_[c.td]);
                if (t < 0 || t > 16) return fail("corrupt DC code");
                c.dc_pred += br.received(t);
                d[0] = (int16_t)(c.dc_pred * (1 << al));
            } else if (br.bit()) {
                d[0] = (int16_t)(d[0] + (1 << al));
            }
            return true;
        }
        if (ah == 0) {  // AC first pass
            if (eobrun) {
                --eobrun;
                return true;
            }
            for (int k = ss; k <= se;) {
                const int rs = br.symbol(ac_[c.ta]);
                if (rs < 0) return fail("corrupt AC code");
                const int r = rs >> 4, s = rs & 15;
                if (s == 0) {
                    if (r < 15) {
                        eobrun = (1 << r) - 1 + (r ? br.bits(r) : 0);
                        break;
                    }
                    k += 16;
                    continue;
                }
                k += r;
                const int z = kZig[k < 63 ? k : 63];
                d[z] = (int16_t)(br.received(s) * (1 << al));
                ++k;
            }
            return true;
        }
        // AC refinement (T.81 G.1.2.3)
        const int16_t bit = (int16_t)(1 << al);
        auto refine = [&](int16_t& v) {
            if (br.bit() && (v & bit) == 0) v = (int16_t)(v > 0 ? v + bit : v - bit);
        };
        int k = ss;
        if (eobrun == 0) {
            for (; k <= se;) {
                const int rs = br.symbol(ac_[c.ta]);
                if (rs < 0) return fail("corrupt AC code");
                int r = rs >> 4;
                const int s = rs & 15;
                int val = 0;
                if (s == 0) {
                    if (r < 15) {
                        eobrun = (1 << r) + (r ? br.bits(r) : 0);
                        break;  // the rest of the band is refined below as an EOB run
                    }
                } else {
                    if (s != 1) return fail("corrupt refinement code");
                    val = br.bit() ? bit : -bit;
                }
                // skip r zero-history coefficients, refining the non-zero ones on the way
                while (k <= se) {
                    int16_t& v = d[kZig[k++]];
                    if (v != 0) {
                        refine(v);
                    } else {
                        if (r == 0) {
                            if (val) v = (int16_t)val;
                            break;
                        }
                        --r;
                    }
                }
            }
        }
        if (eobrun > 0) {  // inside an EOB run: only the correction bits of non-zero history
            for (; k <= se; ++k) {
                int16_t& v = d[kZig[k]];
                if (v != 0) refine(v);
            }
            --eobrun;
        }
        return true;
    };

    int todo = restart_ ? restart_ : 0x7FFFFFFF;
    auto after_unit = [&]() -> bool {  // restart interval bookkeeping after each MCU
        if (--todo > 0) return true;
        br.refill();
        if (br.marker < 0xD0 || br.marker > 0xD7) return false;  // end of the usable data
        br.restart();
        for (Comp& c : comps_) c.dc_pred = 0;
        eobrun = 0;
        todo = restart_ ? restart_ : 0x7FFFFFFF;
        return true;
    };
    for (Comp& c : comps_) c.dc_pred = 0;
    if (ns == 1) {  // non-interleaved: the component's own block raster
        Comp& c = *sc[0];
        const int bx = (c.x + 7) >> 3, by = (c.y + 7) >> 3;
        for (int j = 0; j < by; ++j)
            for (int i = 0; i < bx; ++i) {
                if (!block(c, i, j)) return false;
                if (!after_unit()) return true;
            }
        return true;
    }
    for (int j = 0; j < mcuy_; ++j)
        for (int i = 0; i < mcux_; ++i) {
            for (Comp* c : sc)
                for (int y = 0; y < c->v; ++y)
                    for (int x = 0; x < c->h; ++x)
                        if (!block(*c, i * c->h + x, j * c->v + y)) return false;
            if (!after_unit()) return true;
        }
    return true;
}

void Decoder::finish()
{
    for (Comp& c : comps_) {
        c.plane.assign((size_t)c.w2 * c.bh * 8, 0);
        const int bx = progressive_ ? (c.x + 7) >> 3 : c.bw;
        const int by = progressive_ ? (c.y + 7) >> 3 : c.bh;
        for (int j = 0; j < by; ++j)
            for (int i = 0; i < bx; ++i) {
                int16_t* d = &c.coef[((size_t)j * c.bw + i) * 64];
                if (progressive_)
                    for (int k = 0; k < 64; ++k) d[k] = (int16_t)(d[k] * q_[c.tq][k]);
                idct_block(d, &c.plane[(size_t)j * 8 * c.w2 + (size_t)i * 8], c.w2);
            }
    }
}

bool Decoder::output(Image& out)
{
    typedef const uint8_t* (*Up)(uint8_t*, const uint8_t*, const uint8_t*, int, int);
    const int nc = (int)comps_.size();
    const int n = nc >= 3 ? 3 : 1;  // stbi_load(req_comp 0) channels
    const bool rgb = nc == 3 && (rgb_ids_ == 3 || (adobe_transform_ == 0 && !jfif_));
    struct Walk {
        Up up;
        const uint8_t *line0, *line1;
        int hs, vs, wl, ystep, ypos;
        std::vector<uint8_t> buf;
    };
    std::vector<Walk> wk(nc);
    for (int k = 0; k < nc; ++k) {
        Walk& r = wk[k];
        const Comp& c = comps_[k];
        r.hs = hmax_ / c.h;
        r.vs = vmax_ / c.v;
        r.ystep = r.vs >> 1;
        r.wl = (W_ + r.hs - 1) / r.hs;
        r.ypos = 0;
        r.line0 = r.line1 = c.plane.data();
        r.buf.assign((size_t)W_ + 3 + 4 * (size_t)r.hs, 0);
        r.up = (r.hs == 1 && r.vs == 1) ? up_none
             : (r.hs == 1 && r.vs == 2) ? up_v2
             : (r.hs == 2 && r.vs == 1) ? up_h2
             : (r.hs == 2 && r.vs == 2) ? up_hv2
                                        : up_replicate;
    }
    out = Image();
    out.w = W_;
    out.h = H_;
    out.c = n;
    out.px8.resize((size_t)W_ * H_ * n);
    const uint8_t* row[4] = {nullptr, nullptr, nullptr, nullptr};
    for (int y = 0; y < H_; ++y) {
        for (int k = 0; k < nc; ++k) {
            Walk& r = wk[k];
            const bool bottom = r.ystep >= (r.vs >> 1);
            row[k] = r.up(r.buf.data(), bottom ? r.line1 : r.line0, bottom ? r.line0 : r.line1,
                          r.wl, r.hs);
            if (++r.ystep >= r.vs) {
                r.ystep = 0;
                r.line0 = r.line1;
                if (++r.ypos < comps_[k].y) r.line1 += comps_[k].w2;
            }
        }
        uint8_t* o = &out.px8[(size_t)y * W_ * n];
        if (nc == 1) {
            std::memcpy(o, row[0], (size_t)W_);
        } else if (nc == 3) {
            for (int x = 0; x < W_; ++x, o += 3) {
                if (rgb) {
                    o[0] = row[0][x];
                    o[1] = row[1][x];
                    o[2] = row[2][x];
                } else {
                    ycc_to_rgb(row[0][x], row[1][x], row[2][x], o);
                }
            }
        } else {  // 4 components: Adobe CMYK (transform 0), YCCK (2), else YCbCr + ignored 4th
            for (int x = 0; x < W_; ++x, o += 3) {
                const uint8_t m = row[3][x];
                if (adobe_transform_ == 0) {
                    o[0] = mul255(row[0][x], m);
                    o[1] = mul255(row[1][x], m);
                    o[2] = mul255(row[2][x], m);
                } else {
                    ycc_to_rgb(row[0][x], row[1][x], row[2][x], o);
                    if (adobe_transform_ == 2) {
                        o[0] = mul255((uint8_t)(255 - o[0]), m);
                        o[1] = mul255((uint8_t)(255 - o[1]), m);
                        o[2] = mul255((uint8_t)(255 - o[2]), m);
                    }
                }
            }
        }
    }
    return true;
}

bool Decoder::run(const std::vector<uint8_t>& file, Image& out, std::string& err)
{
    err_ = &err;
    f_ = file.data();
    size_ = file.size();
    if (size_ < 4 || f_[0] != 0xFF || f_[1] != 0xD8) return fail("no SOI marker");
    pos_ = 2;
    bool have_frame = false, any_scan = false, eoi = false;
    BitReader br;
    int pending = -1;  // a marker that ended the previous entropy-coded segment
    for (;;) {
        int m;
        if (pending >= 0) {
            m = pending;
            pending = -1;
        } else {
            while (pos_ < size_ && f_[pos_] != 0xFF) ++pos_;  // padding between segments
            while (pos_ < size_ && f_[pos_] == 0xFF) ++pos_;
            if (pos_ >= size_) break;
            m = f_[pos_++];
        }
        if (m == 0xD9) {                               // EOI
            eoi = true;
            break;
        }
        if (m >= 0xD0 && m <= 0xD7) continue;          // stray RSTn
        if (m == 0x01) continue;                       // TEM
        if (pos_ + 2 > size_) return fail("truncated segment");
        const size_t len = (size_t)u16(pos_);
        if (len < 2 || pos_ + len > size_) return fail("bad segment length");
        const size_t seg = pos_ + 2, segend = pos_ + len;
        if (m == 0xDB) {  // DQT
            for (size_t i = seg; i < segend;) {
                const int pq = f_[i] >> 4, tq = f_[i] & 15;
                if (pq > 1) return fail("bad DQT precision");
                if (tq > 3) return fail("bad DQT table");
                if (i + 1 + (pq ? 128 : 64) > segend) return fail("bad DQT length");
                for (int k = 0; k < 64; ++k)
                    q_[tq][kZig[k]] = (uint16_t)(pq ? u16(i + 1 + 2 * k) : f_[i + 1 + k]);
                i += 1 + (pq ? 128 : 64);
            }
        } else if (m == 0xC4) {  // DHT
            for (size_t i = seg; i < segend;) {
                const int tc = f_[i] >> 4, th = f_[i] & 15;
                if (tc > 1 || th > 3) return fail("bad DHT header");
                if (i + 17 > segend) return fail("bad DHT length");
                int nv = 0;
                for (int l = 0; l < 16; ++l) nv += f_[i + 1 + l];
                if (nv > 256 || i + 17 + nv > segend) return fail("bad DHT length");
                if (!(tc ? ac_[th] : dc_[th]).build(&f_[i + 1], &f_[i + 17], nv))
                    return fail("bad Huffman table");
                i += 17 + nv;
            }
        } else if (m == 0xC0 || m == 0xC1 || m == 0xC2) {  // SOF0/1/2
            if (have_frame) return fail("second frame");
            progressive_ = m == 0xC2;
            if (!frame(seg, len)) return false;
            have_frame = true;
        } else if (m == 0xDD) {  // DRI
            if (len != 4) return fail("bad DRI length");
            restart_ = u16(seg);
        } else if (m == 0xDA) {  // SOS + entropy-coded data
            if (!have_frame) return fail("scan before frame");
            br = BitReader();
            br.p = &f_[segend];
            br.end = f_ + size_;
            if (!scan(seg, len, br)) return false;
            any_scan = true;
            // resume after the entropy-coded segment: at the marker that ended it
            br.refill();
            pos_ = (size_t)(br.p - f_);
            if (br.marker >= 0) pending = br.marker;
            continue;
        } else if (m == 0xDC) {  // DNL
            if (len != 4) return fail("bad DNL length");
            if (u16(seg) != H_) return fail("bad DNL height");
        } else if ((m >= 0xE0 && m <= 0xEF) || m == 0xFE) {  // APPn / COM
            if (m == 0xE0 && len - 2 >= 5 && !std::memcmp(&f_[seg], "JFIF\0", 5)) jfif_ = true;
            if (m == 0xEE && len - 2 >= 12 && !std::memcmp(&f_[seg], "Adobe\0", 6))
                adobe_transform_ = f_[seg + 11];
        } else {
            return fail(m >= 0xC3 && m <= 0xCF ? "lossless / arithmetic-coded / 12-bit frames are "
                                                 "not supported"
                                               : "unknown marker");
        }
        pos_ = segend;
    }
    if (!have_frame || !any_scan) return fail("no image data");
    if (!eoi) return fail("no EOI marker");  // stb rejects a file that just ends
    finish();
    return output(out);
}

}  // namespace

bool decode_jpeg(const std::vector<uint8_t>& f, Image& out, std::string& err)
{
    Decoder d;
    return d.run(f, out, err);
}

// ============================================================================================
// Encoder: stbi_write_jpg's byte stream (see the file comment)
// ============================================================================================
namespace {

// Annex K.1 luminance / chrominance quantisers, natural order
const int kLumQ[64] = {16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
                       14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
                       18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
                       49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
const int kChrQ[64] = {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
                       24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
                       99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
                       99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};
// Annex K.3 tables: code counts per length 1..16, then the symbols
const uint8_t kDcLumBits[16] = {0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
const uint8_t kDcChrBits[16] = {0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
const uint8_t kDcVals[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
const uint8_t kAcLumBits[16] = {0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
const uint8_t kAcLumVal[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61,
    0x07, 0x22, 0x71, 0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52,
    0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72, 0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25,
    0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45,
    0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64,
    0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83,
    0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99,
    0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6,
    0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3,
    0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8,
    0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};
const uint8_t kAcChrBits[16] = {0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
const uint8_t kAcChrVal[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61,
    0x71, 0x13, 0x22, 0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33,
    0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1, 0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18,
    0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44,
    0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63,
    0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a,
    0x82, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97,
    0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4,
    0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca,
    0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7,
    0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};

struct Code {
    uint16_t code[256] = {};
    uint8_t len[256] = {};
};

Code canonical_codes(const uint8_t* bits, const uint8_t* vals)
{  // T.81 Annex C
    Code c;
    int k = 0, code = 0;
    for (int l = 1; l <= 16; l++) {
        for (int i = 0; i < bits[l - 1]; i++, k++) {
            c.code[vals[k]] = (uint16_t)code++;
            c.len[vals[k]] = (uint8_t)l;
        }
        code <<= 1;
    }
    return c;
}

// bit packer with 0xFF stuffing; a 24-bit window, bytes leave from its top
struct BitSink {
    std::vector<uint8_t>& o;
    int window = 0, count = 0;
    explicit BitSink(std::vector<uint8_t>& out) : o(out) {}
    void put(int code, int len)
    {
        count += len;
        window |= code << (24 - count);
        while (count >= 8) {
            const uint8_t b = (uint8_t)((window >> 16) & 255);
            o.push_back(b);
            if (b == 0xFF) o.push_back(0);
            window <<= 8;
            count -= 8;
        }
    }
};

// the AAN forward DCT on 8 floats at p[0], p[s], ..., p[7s] (in place, scaled outputs)
void aan_fdct(float* p, int s)
{
    float v0 = p[0], v1 = p[s], v2 = p[2 * s], v3 = p[3 * s];
    float v4 = p[4 * s], v5 = p[5 * s], v6 = p[6 * s], v7 = p[7 * s];
    const float a07 = v0 + v7, d07 = v0 - v7, a16 = v1 + v6, d16 = v1 - v6;
    const float a25 = v2 + v5, d25 = v2 - v5, a34 = v3 + v4, d34 = v3 - v4;
    // even half
    const float e0 = a07 + a34, e3 = a07 - a34, e1 = a16 + a25, e2 = a16 - a25;
    const float r = (e2 + e3) * 0.707106781f;
    p[0] = e0 + e1;
    p[4 * s] = e0 - e1;
    p[2 * s] = e3 + r;
    p[6 * s] = e3 - r;
    // odd half, with the rotator arranged to avoid negations
    const float o0 = d34 + d25, o1 = d25 + d16, o2 = d16 + d07;
    const float rot = (o0 - o2) * 0.382683433f;
    const float c2 = o0 * 0.541196100f + rot;
    const float c4 = o2 * 1.306562965f + rot;
    const float c3 = o1 * 0.707106781f;
    const float s1 = d07 + c3, s3 = d07 - c3;
    p[5 * s] = s3 + c2;
    p[3 * s] = s3 - c2;
    p[s] = s1 + c4;
    p[7 * s] = s1 - c4;
}

// magnitude category and the appended bits of a coefficient value (T.81 F.1.2.1)
inline void magnitude(int v, int& nbits, int& bits)
{
    int a = v < 0 ? -v : v;
    const int w = v < 0 ? v - 1 : v;
    nbits = 1;
    while (a >>= 1) ++nbits;
    bits = w & ((1 << nbits) - 1);
}

// Transform, quantise and code one 8x8 data unit at du (row stride `stride` floats, destroyed).
int code_unit(BitSink& bs, float* du, int stride, const float* recip, int pred, const Code& dc,
              const Code& ac)
{
    for (int r = 0; r < 8; ++r) aan_fdct(du + r * stride, 1);
    for (int c = 0; c < 8; ++c) aan_fdct(du + c, stride);
    int zz[64];  // quantised, zig-zag order
    for (int k = 0; k < 64; ++k) {
        const int j = kZig[k];  // natural index
        const float v = du[(j >> 3) * stride + (j & 7)] * recip[j];
        zz[k] = (int)(v < 0 ? v - 0.5f : v + 0.5f);
    }
    int nb, b;
    const int diff = zz[0] - pred;
    if (diff == 0) {
        bs.put(dc.code[0], dc.len[0]);
    } else {
        magnitude(diff, nb, b);
        bs.put(dc.code[nb], dc.len[nb]);
        bs.put(b, nb);
    }
    int last = 63;
    while (last > 0 && zz[last] == 0) --last;
    if (last == 0) {
        bs.put(ac.code[0x00], ac.len[0x00]);
        return zz[0];
    }
    for (int i = 1; i <= last; ++i) {
        int run = 0;
        while (zz[i] == 0 && i <= last) ++run, ++i;
        for (; run >= 16; run -= 16) bs.put(ac.code[0xF0], ac.len[0xF0]);
        magnitude(zz[i], nb, b);
        bs.put(ac.code[(run << 4) + nb], ac.len[(run << 4) + nb]);
        bs.put(b, nb);
    }
    if (last != 63) bs.put(ac.code[0x00], ac.len[0x00]);
    return zz[0];
}

void put16(std::vector<uint8_t>& o, int v)
{
    o.push_back((uint8_t)(v >> 8));
    o.push_back((uint8_t)v);
}

}  // namespace

bool encode_jpeg(const uint8_t* px, int w, int h, int c, int quality, std::vector<uint8_t>& o,
                 std::string& err, bool flip)
{
    if (!px || w < 1 || h < 1 || w > 65535 || h > 65535 || c < 1 || c > 4) {
        err = "encode_jpeg: bad image";
        return false;
    }
    int q = quality ? quality : 90;
    const bool subsample = q <= 90;
    q = q < 1 ? 1 : (q > 100 ? 100 : q);
    q = q < 50 ? 5000 / q : 200 - q * 2;
    uint8_t ytab[64], ctab[64];  // zig-zag order, as written to the DQT
    for (int k = 0; k < 64; ++k) {
        const int a = (kLumQ[kZig[k]] * q + 50) / 100, b = (kChrQ[kZig[k]] * q + 50) / 100;
        ytab[k] = (uint8_t)(a < 1 ? 1 : (a > 255 ? 255 : a));
        ctab[k] = (uint8_t)(b < 1 ? 1 : (b > 255 ? 255 : b));
    }
    // the AAN output scale factors (x sqrt(8)) folded into reciprocal quantisers, natural order
    static const float aan[8] = {1.0f * 2.828427125f,         1.387039845f * 2.828427125f,
                                 1.306562965f * 2.828427125f, 1.175875602f * 2.828427125f,
                                 1.0f * 2.828427125f,         0.785694958f * 2.828427125f,
                                 0.541196100f * 2.828427125f, 0.275899379f * 2.828427125f};
    int zpos[64];
    for (int k = 0; k < 64; ++k) zpos[kZig[k]] = k;
    float ry[64], rc[64];
    for (int r = 0; r < 8; ++r)
        for (int col = 0; col < 8; ++col) {
            const int j = r * 8 + col;
            ry[j] = 1 / (ytab[zpos[j]] * aan[r] * aan[col]);
            rc[j] = 1 / (ctab[zpos[j]] * aan[r] * aan[col]);
        }
    o.clear();
    const uint8_t app0[] = {0xFF, 0xD8, 0xFF, 0xE0, 0, 0x10, 'J', 'F', 'I', 'F', 0, 1, 1, 0, 0,
                            1, 0, 1, 0, 0};
    o.insert(o.end(), app0, app0 + sizeof(app0));
    o.push_back(0xFF); o.push_back(0xDB); put16(o, 2 + 2 * 65);
    o.push_back(0);
    o.insert(o.end(), ytab, ytab + 64);
    o.push_back(1);
    o.insert(o.end(), ctab, ctab + 64);
    o.push_back(0xFF); o.push_back(0xC0); put16(o, 17);
    o.push_back(8); put16(o, h); put16(o, w); o.push_back(3);
    o.push_back(1); o.push_back(subsample ? 0x22 : 0x11); o.push_back(0);
    o.push_back(2); o.push_back(0x11); o.push_back(1);
    o.push_back(3); o.push_back(0x11); o.push_back(1);
    o.push_back(0xFF); o.push_back(0xC4); put16(o, 2 + 4 * 17 + 12 + 162 + 12 + 162);
    auto table = [&](uint8_t id, const uint8_t* bits, const uint8_t* vals, int n) {
        o.push_back(id);
        o.insert(o.end(), bits, bits + 16);
        o.insert(o.end(), vals, vals + n);
    };
    table(0x00, kDcLumBits, kDcVals, 12);
    table(0x10, kAcLumBits, kAcLumVal, 162);
    table(0x01, kDcChrBits, kDcVals, 12);
    table(0x11, kAcChrBits, kAcChrVal, 162);
    const uint8_t sos[] = {0xFF, 0xDA, 0, 12, 3, 1, 0, 2, 0x11, 3, 0x11, 0, 0x3F, 0};
    o.insert(o.end(), sos, sos + sizeof(sos));

    const Code ydc = canonical_codes(kDcLumBits, kDcVals), yac = canonical_codes(kAcLumBits, kAcLumVal);
    const Code cdc = canonical_codes(kDcChrBits, kDcVals), cac = canonical_codes(kAcChrBits, kAcChrVal);
    BitSink bs(o);
    int py = 0, pu = 0, pv = 0;
    const int gofs = c > 2 ? 1 : 0, bofs = c > 2 ? 2 : 0;  // 2 = gray + alpha: alpha ignored
    const int mcu = subsample ? 16 : 8;
    std::vector<float> Y(mcu * mcu), U(mcu * mcu), V(mcu * mcu);
    for (int y0 = 0; y0 < h; y0 += mcu)
        for (int x0 = 0; x0 < w; x0 += mcu) {
            for (int r = 0; r < mcu; ++r) {  // edges repeat the last row / column
                const int sr = y0 + r < h ? y0 + r : h - 1;
                const size_t base = (size_t)(flip ? h - 1 - sr : sr) * w * c;
                for (int col = 0; col < mcu; ++col) {
                    const size_t p = base + (size_t)(x0 + col < w ? x0 + col : w - 1) * c;
                    const float R = px[p], G = px[p + gofs], B = px[p + bofs];
                    const int i = r * mcu + col;
                    Y[i] = +0.29900f * R + 0.58700f * G + 0.11400f * B - 128;
                    U[i] = -0.16874f * R - 0.33126f * G + 0.50000f * B;
                    V[i] = +0.50000f * R - 0.41869f * G - 0.08131f * B;
                }
            }
            if (subsample) {
                for (int k : {0, 8, 128, 136}) py = code_unit(bs, &Y[k], 16, ry, py, ydc, yac);
                float su[64], sv[64];
                for (int r = 0; r < 8; ++r)
                    for (int col = 0; col < 8; ++col) {
                        const int j = r * 32 + col * 2;
                        su[r * 8 + col] = (U[j] + U[j + 1] + U[j + 16] + U[j + 17]) * 0.25f;
                        sv[r * 8 + col] = (V[j] + V[j + 1] + V[j + 16] + V[j + 17]) * 0.25f;
                    }
                pu = code_unit(bs, su, 8, rc, pu, cdc, cac);
                pv = code_unit(bs, sv, 8, rc, pv, cdc, cac);
            } else {
                py = code_unit(bs, Y.data(), 8, ry, py, ydc, yac);
                pu = code_unit(bs, U.data(), 8, rc, pu, cdc, cac);
                pv = code_unit(bs, V.data(), 8, rc, pv, cdc, cac);
            }
        }
    bs.put(0x7F, 7);  // pad the last byte with 1 bits
    o.push_back(0xFF);
    o.push_back(0xD9);
    return true;
}

bool save_jpeg(const std::string& fn, const uint8_t* px, int w, int h, int c, int quality,
               std::string& err, bool flip)
{
    std::vector<uint8_t> o;
    if (!encode_jpeg(px, w, h, c, quality, o, err, flip)) return false;
    FILE* f = std::fopen(fn.c_str(), "wb");
    if (!f) {
        err = "cannot write " + fn;
        return false;
    }
    const bool ok = std::fwrite(o.data(), 1, o.size(), f) == o.size();
    std::fclose(f);
    if (!ok) err = "short write to " + fn;
    return ok;
}

}  // namespace pfio
