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

}  // namespace pfio
