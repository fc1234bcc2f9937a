// pf_jpeg.cpp -- baseline JPEG decoder for the map loaders.
//
// The reference decodes its depth-net tiles (LeReS writes JPEG, Main.cpp:576-578) and some
// baselines (`.jpg`, `.unifuse.jpg`, Main.cpp:499-510) with stb_image (stbi_load, req_comp 0).
// This is a decoder of the same format family written from the JPEG standard (ITU T.81):
// baseline and extended-sequential Huffman DCT, 8-bit samples, 1 (gray) or 3 (YCbCr)
// components, any sampling factors up to 2x2 (triangle "fancy" upsampling for 2x1 / 2x2 chroma,
// replication otherwise), restart intervals.  The IDCT is computed in double and rounded, so
// samples agree with integer IDCTs (stb's, libjpeg's islow) to about one level; bit parity with
// stb's fixed-point IDCT and colour conversion is not claimed.  Progressive, arithmetic-coded,
// 12-bit and CMYK files are rejected with a message.
#include "pf_image.hpp"

#include <cmath>
#include <cstdio>
#include <cstring>

namespace pfio {

namespace {

const int kZig[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                      12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                      35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                      58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct Huff {
    bool present = false;
    // canonical decode: per length l, codes in [mincode[l], maxcode[l]] map to vals[valptr[l]+..]
    int mincode[17], maxcode[18], valptr[17];
    uint8_t vals[256];
    // 9-bit lookahead: code length (0 = longer) and value
    uint8_t fast_len[512], fast_val[512];
};

struct Comp {
    int id = 0, h = 1, v = 1, tq = 0, td = 0, ta = 0;
    int bw = 0, bh = 0;          // blocks per line / column (padded to whole MCUs)
    std::vector<uint8_t> pix;    // bw*8 x bh*8 samples
    int pred = 0;
};

struct Bits {
    const uint8_t* p;
    const uint8_t* end;
    uint32_t acc = 0;
    int n = 0;
    bool marker = false;  // hit a marker: feed zeros from here on
    void fill()
    {
        while (n <= 24) {
            uint32_t byte = 0;
            if (!marker && p < end) {
                byte = *p;
                if (byte == 0xFF) {
                    const uint8_t nx = p + 1 < end ? p[1] : 0;
                    if (nx == 0x00) {
                        p += 2;
                    } else {
                        marker = true;  // leave p on the marker
                        byte = 0;
                    }
                } else {
                    ++p;
                }
            }
            acc |= byte << (24 - n);
            n += 8;
        }
    }
    int get(int k)
    {
        if (k == 0) return 0;
        fill();
        const int v = (int)(acc >> (32 - k));
        acc <<= k;
        n -= k;
        return v;
    }
    int peek9()
    {
        fill();
        return (int)(acc >> 23);
    }
    void skip(int k)
    {
        acc <<= k;
        n -= k;
    }
};

bool build_huff(Huff& h, const uint8_t* counts, const uint8_t* vals, int nvals)
{
    h.present = true;
    std::memcpy(h.vals, vals, nvals);
    std::memset(h.fast_len, 0, sizeof(h.fast_len));
    int code = 0, k = 0;
    for (int l = 1; l <= 16; ++l) {
        h.valptr[l] = k;
        h.mincode[l] = code;
        if (code + counts[l - 1] > (1 << l)) return h.present = false;  // over-full code space
        for (int i = 0; i < counts[l - 1]; ++i, ++k, ++code) {
            if (l <= 9) {
                const int base = code << (9 - l);
                for (int j = 0; j < (1 << (9 - l)); ++j) {
                    h.fast_len[base + j] = (uint8_t)l;
                    h.fast_val[base + j] = vals[k];
                }
            }
        }
        h.maxcode[l] = counts[l - 1] ? code - 1 : -1;
        code <<= 1;
    }
    h.maxcode[17] = 0x7FFFFFFF;
    return true;
}

int decode_sym(Bits& b, const Huff& h)
{
    const int look = b.peek9();
    if (h.fast_len[look]) {
        b.skip(h.fast_len[look]);
        return h.fast_val[look];
    }
    int code = 0;
    for (int l = 1; l <= 16; ++l) {
        code = (code << 1) | b.get(1);
        if (h.maxcode[l] >= 0 && code <= h.maxcode[l] && code >= h.mincode[l])
            return h.vals[h.valptr[l] + code - h.mincode[l]];
    }
    return -1;  // corrupt
}

int extend(int v, int t) { return (t && v < (1 << (t - 1))) ? v - (1 << t) + 1 : v; }

// 8x8 inverse DCT in double (T.81 A.3.3), level shift, round, clamp.
void idct_block(const int* coef, const uint16_t* q, uint8_t* out, int stride)
{
    static double cosv[8][8];
    static bool init = false;
    if (!init) {
        for (int x = 0; x < 8; ++x)
            for (int u = 0; u < 8; ++u)
                cosv[x][u] = (u == 0 ? std::sqrt(0.5) : 1.0) *
                             std::cos((2 * x + 1) * u * 3.14159265358979323846 / 16.0);
        init = true;
    }
    double F[64], tmp[64];
    for (int i = 0; i < 64; ++i) F[i] = (double)coef[i] * q[i];
    for (int y = 0; y < 8; ++y)       // rows: over u
        for (int x = 0; x < 8; ++x) {
            double s = 0;
            for (int u = 0; u < 8; ++u) s += cosv[x][u] * F[y * 8 + u];
            tmp[y * 8 + x] = s;
        }
    for (int x = 0; x < 8; ++x)       // columns: over v
        for (int y = 0; y < 8; ++y) {
            double s = 0;
            for (int v = 0; v < 8; ++v) s += cosv[y][v] * tmp[v * 8 + x];
            long r = std::lround(s / 4.0 + 128.0);
            out[y * stride + x] = (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
        }
}

inline uint8_t clamp8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

// Chroma plane (cw x ch, one sample per hs x vs luma pixels) to full resolution w x h.
void upsample(const Comp& c, int hs, int vs, int w, int h, std::vector<uint8_t>& out)
{
    out.resize((size_t)w * h);
    const int cw = c.bw * 8, ch = c.bh * 8;
    const int sw = (w + hs - 1) / hs, sh = (h + vs - 1) / vs;  // meaningful samples
    auto S = [&](int x, int y) {
        x = x < 0 ? 0 : (x >= sw ? sw - 1 : x);
        y = y < 0 ? 0 : (y >= sh ? sh - 1 : y);
        (void)cw;
        (void)ch;
        return (int)c.pix[(size_t)y * cw + x];
    };
    if (hs == 2 && (vs == 1 || vs == 2)) {  // triangle filter (libjpeg "fancy" upsampling)
        for (int y = 0; y < h; ++y) {
            const int sy = y / vs;
            const int ny = vs == 2 ? ((y & 1) ? sy + 1 : sy - 1) : sy;
            for (int x = 0; x < w; ++x) {
                const int sx = x >> 1, nx = (x & 1) ? sx + 1 : sx - 1;
                if (vs == 2) {
                    const int c0 = 3 * S(sx, sy) + S(sx, ny);
                    const int c1 = 3 * S(nx, sy) + S(nx, ny);
                    out[(size_t)y * w + x] = (uint8_t)((3 * c0 + c1 + 8) >> 4);
                } else {
                    out[(size_t)y * w + x] =
                        (uint8_t)((3 * S(sx, sy) + S(nx, sy) + 2) >> 2);
                }
            }
        }
        return;
    }
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) out[(size_t)y * w + x] = (uint8_t)S(x / hs, y / vs);
}

}  // namespace

bool decode_jpeg(const std::vector<uint8_t>& f, Image& out, std::string& err)
{
    if (f.size() < 4 || f[0] != 0xFF || f[1] != 0xD8) return err = "not a JPEG", false;
    uint16_t qt[4][64];
    bool qok[4] = {false, false, false, false};
    Huff hdc[4], hac[4];
    std::vector<Comp> comps;
    int W = 0, H = 0, hmax = 1, vmax = 1, restart = 0;
    bool frame = false, done = false;
    size_t p = 2;
    auto u16 = [&](size_t i) { return (int)(f[i] << 8 | f[i + 1]); };
    while (p + 4 <= f.size() && !done) {
        if (f[p] != 0xFF) return err = "JPEG: marker expected", false;
        const int m = f[p + 1];
        if (m == 0xFF) { ++p; continue; }
        if (m == 0xD9) break;
        if (m == 0x01 || (m >= 0xD0 && m <= 0xD7)) {  // standalone markers
            p += 2;
            continue;
        }
        const int len = u16(p + 2);
        if (len < 2) return err = "JPEG: bad segment length", false;
        const size_t seg = p + 4, segend = p + 2 + len;
        if (segend > f.size()) return err = "JPEG: truncated segment", false;
        if (m == 0xDB) {  // DQT
            size_t i = seg;
            while (i < segend) {
                const int pq = f[i] >> 4, tq = f[i] & 15;
                if (tq > 3 || pq > 1 || i + 1 + (pq ? 128 : 64) > segend)
                    return err = "JPEG: bad DQT", false;
                ++i;
                for (int k = 0; k < 64; ++k) {
                    qt[tq][kZig[k]] = pq ? (uint16_t)u16(i + 2 * k) : f[i + k];
                }
                i += pq ? 128 : 64;
                qok[tq] = true;
            }
        } else if (m == 0xC4) {  // DHT
            size_t i = seg;
            while (i < segend) {
                const int tc = f[i] >> 4, th = f[i] & 15;
                if (th > 3 || tc > 1) return err = "JPEG: bad DHT", false;
                const uint8_t* counts = &f[i + 1];
                int n = 0;
                for (int l = 0; l < 16; ++l) n += counts[l];
                if (n > 256 || i + 17 + n > segend) return err = "JPEG: bad DHT", false;
                if (!build_huff(tc ? hac[th] : hdc[th], counts, &f[i + 17], n))
                    return err = "JPEG: bad Huffman table", false;
                i += 17 + n;
            }
        } else if (m == 0xC0 || m == 0xC1) {  // SOF0 / SOF1
            if (len < 8 || f[seg] != 8)
                return err = "JPEG: only 8-bit samples are supported", false;
            H = u16(seg + 1);
            W = u16(seg + 3);
            const int nc = f[seg + 5];
            if (W <= 0 || H <= 0 || (nc != 1 && nc != 3) || seg + 6 + 3 * nc > segend)
                return err = "JPEG: only 1- or 3-component images are supported", false;
            if ((long long)W * H > (1ll << 28)) return err = "JPEG: image too large", false;
            comps.resize(nc);
            for (int k = 0; k < nc; ++k) {
                Comp& c = comps[k];
                c.id = f[seg + 6 + 3 * k];
                c.h = f[seg + 7 + 3 * k] >> 4;
                c.v = f[seg + 7 + 3 * k] & 15;
                c.tq = f[seg + 8 + 3 * k] & 3;
                if (c.h < 1 || c.h > 2 || c.v < 1 || c.v > 2)
                    return err = "JPEG: sampling factors above 2 are not supported", false;
                hmax = std::max(hmax, c.h);
                vmax = std::max(vmax, c.v);
            }
            frame = true;
        } else if (m == 0xC2 || m == 0xC3 || (m >= 0xC5 && m <= 0xCF && m != 0xC8 && m != 0xCC)) {
            return err = "JPEG: progressive / lossless / arithmetic coding is not supported",
                   false;
        } else if (m == 0xDD) {  // DRI
            if (len < 4) return err = "JPEG: bad DRI", false;
            restart = u16(seg);
        } else if (m == 0xDA) {  // SOS: one interleaved scan with every component
            if (!frame) return err = "JPEG: scan before frame", false;
            const int ns = f[seg];
            if (seg + 1 + 2 * (size_t)ns > segend) return err = "JPEG: bad SOS", false;
            if (ns != (int)comps.size())
                return err = "JPEG: non-interleaved scans are not supported", false;
            if (ns == 1) {  // a single-component scan is non-interleaved: one block per MCU
                comps[0].h = comps[0].v = 1;
                hmax = vmax = 1;
            }
            for (int k = 0; k < ns; ++k) {
                const int cid = f[seg + 1 + 2 * k], tbl = f[seg + 2 + 2 * k];
                if ((tbl >> 4) > 3 || (tbl & 15) > 3) return err = "JPEG: bad table selector", false;
                for (Comp& c : comps)
                    if (c.id == cid) c.td = tbl >> 4, c.ta = tbl & 15;
            }
            const int mcux = (W + 8 * hmax - 1) / (8 * hmax), mcuy = (H + 8 * vmax - 1) / (8 * vmax);
            for (Comp& c : comps) {
                if (!qok[c.tq] || !hdc[c.td].present || !hac[c.ta].present)
                    return err = "JPEG: missing table", false;
                c.bw = mcux * c.h;
                c.bh = mcuy * c.v;
                c.pix.assign((size_t)c.bw * 8 * c.bh * 8, 0);
                c.pred = 0;
            }
            Bits b{&f[segend], f.data() + f.size()};
            int coef[64];
            int todo = restart ? restart : mcux * mcuy;
            for (int my = 0; my < mcuy; ++my)
                for (int mx = 0; mx < mcux; ++mx) {
                    if (restart && todo == 0) {  // RSTn: realign, reset predictors
                        b.acc = 0;
                        b.n = 0;
                        b.marker = false;
                        while (b.p + 1 < b.end && !(b.p[0] == 0xFF && b.p[1] >= 0xD0 && b.p[1] <= 0xD7))
                            ++b.p;
                        b.p += 2;
                        for (Comp& c : comps) c.pred = 0;
                        todo = restart;
                    }
                    for (Comp& c : comps)
                        for (int by = 0; by < c.v; ++by)
                            for (int bx = 0; bx < c.h; ++bx) {
                                std::memset(coef, 0, sizeof(coef));
                                const int t = decode_sym(b, hdc[c.td]);
                                if (t < 0 || t > 16) return err = "JPEG: corrupt DC", false;
                                c.pred += extend(b.get(t), t);
                                coef[0] = c.pred;
                                for (int k = 1; k < 64;) {
                                    const int rs = decode_sym(b, hac[c.ta]);
                                    if (rs < 0) return err = "JPEG: corrupt AC", false;
                                    const int r = rs >> 4, s = rs & 15;
                                    if (s == 0) {
                                        if (r != 15) break;  // EOB
                                        k += 16;
                                        continue;
                                    }
                                    k += r;
                                    if (k > 63) return err = "JPEG: corrupt AC run", false;
                                    coef[kZig[k]] = extend(b.get(s), s);
                                    ++k;
                                }
                                const int X = (mx * c.h + bx) * 8, Y = (my * c.v + by) * 8;
                                idct_block(coef, qt[c.tq], &c.pix[(size_t)Y * c.bw * 8 + X],
                                           c.bw * 8);
                            }
                    --todo;
                }
            done = true;
            break;
        }
        p = segend;
    }
    if (!done) return err = "JPEG: no image data", false;
    out = Image();
    out.w = W;
    out.h = H;
    out.c = (int)comps.size();
    out.px8.resize((size_t)W * H * out.c);
    if (out.c == 1) {
        const Comp& c = comps[0];
        const int hs = hmax / c.h, vs = vmax / c.v;
        std::vector<uint8_t> full;
        upsample(c, hs, vs, W, H, full);
        out.px8 = full;
        return true;
    }
    std::vector<uint8_t> pl[3];
    for (int k = 0; k < 3; ++k) upsample(comps[k], hmax / comps[k].h, vmax / comps[k].v, W, H, pl[k]);
    for (size_t i = 0; i < (size_t)W * H; ++i) {  // JFIF YCbCr -> RGB
        const double Y = pl[0][i], cb = pl[1][i] - 128.0, cr = pl[2][i] - 128.0;
        out.px8[3 * i + 0] = clamp8((int)std::lround(Y + 1.402 * cr));
        out.px8[3 * i + 1] = clamp8((int)std::lround(Y - 0.344136 * cb - 0.714136 * cr));
        out.px8[3 * i + 2] = clamp8((int)std::lround(Y + 1.772 * cb));
    }
    return true;
}


// ---------------------------------------------------------------------------------------------
// Baseline JPEG encoder for the RGB tile export: the reference writes each
// rendered tile with stbi_write_jpg(..., quality = width*3) (Main.cpp:320), which stb clamps to
// 100 with no chroma subsampling (stb_image_write.h:1448-1451).  Written here from T.81: JFIF
// APP0, the Annex K example quantisation tables scaled by the stb/IJG quality rule (all ones at
// 100), 4:4:4 sampling, the Annex K.3 Huffman tables, full-precision DCT (double) with the
// quantised coefficients rounded half away from zero.  The bytes are not stb's (its float AAN
// DCT rounds differently); decoded samples agree with the input to a level or two.
namespace {

const uint8_t kLumQ[64] = {16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
                           14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
                           18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
                           49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
const uint8_t kChrQ[64] = {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
                           24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
                           99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
                           99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};
// Annex K.3: {bits[1..16], values}
const uint8_t kDcLumBits[16] = {0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
const uint8_t kDcLumVal[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
const uint8_t kDcChrBits[16] = {0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
const uint8_t kDcChrVal[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
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
    uint16_t code[256];
    uint8_t len[256];
};

Code make_codes(const uint8_t* bits, const uint8_t* vals)
{  // canonical Huffman codes (T.81 Annex C)
    Code c{};
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

struct BitOut {
    std::vector<uint8_t>& o;
    uint32_t acc = 0;
    int n = 0;
    explicit BitOut(std::vector<uint8_t>& out) : o(out) {}
    void put(uint32_t v, int k)
    {
        acc = (acc << k) | (v & ((1u << k) - 1));
        n += k;
        while (n >= 8) {
            const uint8_t b = (uint8_t)(acc >> (n - 8));
            o.push_back(b);
            if (b == 0xFF) o.push_back(0);  // byte stuffing
            n -= 8;
        }
    }
    void flush()
    {
        if (n > 0) put(0x7F, 8 - n);  // pad with 1 bits
    }
};

void put16(std::vector<uint8_t>& o, int v)
{
    o.push_back((uint8_t)(v >> 8));
    o.push_back((uint8_t)v);
}

void encode_block(BitOut& bo, const double* px, const uint8_t* q, int& pred, const Code& dc,
                  const Code& ac)
{
    static double cosv[8][8];
    static bool init = false;
    if (!init) {
        for (int u = 0; u < 8; u++)
            for (int x = 0; x < 8; x++) cosv[u][x] = std::cos((2 * x + 1) * u * M_PI / 16.0);
        init = true;
    }
    int zz[64];
    for (int v = 0; v < 8; v++)
        for (int u = 0; u < 8; u++) {
            double s = 0;
            for (int y = 0; y < 8; y++)
                for (int x = 0; x < 8; x++) s += px[y * 8 + x] * cosv[u][x] * cosv[v][y];
            const double cu = u ? 1.0 : M_SQRT1_2, cv = v ? 1.0 : M_SQRT1_2;
            const double f = 0.25 * cu * cv * s / q[v * 8 + u];
            zz[v * 8 + u] = (int)(f < 0 ? f - 0.5 : f + 0.5);
        }
    auto mag = [](int v, int& nb) {
        int a = v < 0 ? -v : v;
        nb = 0;
        while (a) { nb++; a >>= 1; }
        return v < 0 ? v + (1 << nb) - 1 : v;
    };
    int nb;
    const int diff = zz[0] - pred;
    pred = zz[0];
    const int dv = mag(diff, nb);
    bo.put(dc.code[nb], dc.len[nb]);
    if (nb) bo.put((uint32_t)dv, nb);
    int run = 0;
    for (int k = 1; k < 64; k++) {
        const int v = zz[kZig[k]];
        if (v == 0) { run++; continue; }
        while (run > 15) { bo.put(ac.code[0xF0], ac.len[0xF0]); run -= 16; }
        const int av = mag(v, nb);
        const int sym = (run << 4) | nb;
        bo.put(ac.code[sym], ac.len[sym]);
        bo.put((uint32_t)av, nb);
        run = 0;
    }
    if (run) bo.put(ac.code[0], ac.len[0]);  // EOB
}

}  // namespace

bool encode_jpeg(const uint8_t* px, int w, int h, int c, int quality, std::vector<uint8_t>& o,
                 std::string& err)
{
    if (!px || w < 1 || h < 1 || w > 65535 || h > 65535 || (c != 1 && c != 3)) {
        err = "encode_jpeg: bad image";
        return false;
    }
    // quality scaling of the Annex K tables, as stb / IJG (stb_image_write.h:1448-1458)
    int qs = quality ? quality : 90;
    qs = qs < 1 ? 1 : (qs > 100 ? 100 : qs);
    qs = qs < 50 ? 5000 / qs : 200 - qs * 2;
    uint8_t ql[64], qc[64];  // natural (row-major) order
    for (int i = 0; i < 64; i++) {
        const int a = (kLumQ[i] * qs + 50) / 100, b = (kChrQ[i] * qs + 50) / 100;
        ql[i] = (uint8_t)(a < 1 ? 1 : (a > 255 ? 255 : a));
        qc[i] = (uint8_t)(b < 1 ? 1 : (b > 255 ? 255 : b));
    }
    o.clear();
    const uint8_t soi_app0[] = {0xFF, 0xD8, 0xFF, 0xE0, 0, 16, 'J', 'F', 'I', 'F', 0, 1, 1, 0,
                                0, 1, 0, 1, 0, 0};
    o.insert(o.end(), soi_app0, soi_app0 + sizeof(soi_app0));
    const int ntab = c == 3 ? 2 : 1;  // DQT (zig-zag order)
    o.push_back(0xFF); o.push_back(0xDB); put16(o, 2 + 65 * ntab);
    for (int t = 0; t < ntab; t++) {
        o.push_back((uint8_t)t);
        for (int k = 0; k < 64; k++) o.push_back(t ? qc[kZig[k]] : ql[kZig[k]]);
    }
    o.push_back(0xFF); o.push_back(0xC0); put16(o, 8 + 3 * c);  // SOF0, 4:4:4
    o.push_back(8); put16(o, h); put16(o, w); o.push_back((uint8_t)c);
    for (int k = 0; k < c; k++) {
        o.push_back((uint8_t)(k + 1)); o.push_back(0x11); o.push_back(k ? 1 : 0);
    }
    auto dht = [&](int cls_id, const uint8_t* bits, const uint8_t* vals) {
        int n = 0;
        for (int i = 0; i < 16; i++) n += bits[i];
        o.push_back(0xFF); o.push_back(0xC4); put16(o, 2 + 17 + n);
        o.push_back((uint8_t)cls_id);
        o.insert(o.end(), bits, bits + 16);
        o.insert(o.end(), vals, vals + n);
    };
    dht(0x00, kDcLumBits, kDcLumVal);
    dht(0x10, kAcLumBits, kAcLumVal);
    if (c == 3) {
        dht(0x01, kDcChrBits, kDcChrVal);
        dht(0x11, kAcChrBits, kAcChrVal);
    }
    o.push_back(0xFF); o.push_back(0xDA); put16(o, 6 + 2 * c); o.push_back((uint8_t)c);
    for (int k = 0; k < c; k++) { o.push_back((uint8_t)(k + 1)); o.push_back(k ? 0x11 : 0x00); }
    o.push_back(0); o.push_back(63); o.push_back(0);
    const Code dcl = make_codes(kDcLumBits, kDcLumVal), acl = make_codes(kAcLumBits, kAcLumVal);
    const Code dcc = make_codes(kDcChrBits, kDcChrVal), acc = make_codes(kAcChrBits, kAcChrVal);
    BitOut bo(o);
    int pred[3] = {0, 0, 0};
    double blk[3][64];
    for (int by = 0; by < h; by += 8)
        for (int bx = 0; bx < w; bx += 8) {
            for (int y = 0; y < 8; y++)
                for (int x = 0; x < 8; x++) {  // edge blocks repeat the last row / column
                    const int sy = by + y < h ? by + y : h - 1, sx = bx + x < w ? bx + x : w - 1;
                    const uint8_t* p = px + ((size_t)sy * w + sx) * c;
                    if (c == 1) {
                        blk[0][y * 8 + x] = p[0] - 128.0;
                    } else {  // JFIF YCbCr, level shifted
                        const double r = p[0], g = p[1], b = p[2];
                        blk[0][y * 8 + x] = 0.299 * r + 0.587 * g + 0.114 * b - 128.0;
                        blk[1][y * 8 + x] = -0.168735892 * r - 0.331264108 * g + 0.5 * b;
                        blk[2][y * 8 + x] = 0.5 * r - 0.418687589 * g - 0.081312411 * b;
                    }
                }
            encode_block(bo, blk[0], ql, pred[0], dcl, acl);
            if (c == 3) {
                encode_block(bo, blk[1], qc, pred[1], dcc, acc);
                encode_block(bo, blk[2], qc, pred[2], dcc, acc);
            }
        }
    bo.flush();
    o.push_back(0xFF); o.push_back(0xD9);
    return true;
}

bool save_jpeg(const std::string& fn, const uint8_t* px, int w, int h, int c, int quality,
               std::string& err)
{
    std::vector<uint8_t> o;
    if (!encode_jpeg(px, w, h, c, quality, o, err)) return false;
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
