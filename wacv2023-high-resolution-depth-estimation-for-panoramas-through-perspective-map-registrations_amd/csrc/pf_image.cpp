// pf_image.cpp -- PNG / PGM / PFM readers and PNG writers (see pf_image.hpp).
#include "pf_image.hpp"

#include <zlib.h>

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <type_traits>

namespace pfio {

namespace {

bool read_file(const std::string& fn, std::vector<uint8_t>& buf)
{
    std::ifstream f(fn, std::ios::binary);
    if (!f) return false;
    buf.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    return true;
}

uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | p[1] << 16 | p[2] << 8 | p[3]; }

const uint8_t kSig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};

int paeth(int a, int b, int c)
{
    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    if (pa <= pb && pa <= pc) return a;
    return pb <= pc ? b : c;
}

// Inflate a zlib stream into exactly `need` bytes (trailing data past them is ignored, as stb
// ignores it).
bool inflate_exact(const std::vector<uint8_t>& z, std::vector<uint8_t>& out, size_t need)
{
    out.assign(need, 0);
    z_stream zs{};
    if (inflateInit(&zs) != Z_OK) return false;
    zs.next_in = const_cast<Bytef*>(z.data());
    zs.avail_in = (uInt)z.size();
    zs.next_out = out.data();
    zs.avail_out = (uInt)need;
    int rc = Z_OK;
    while (zs.avail_out > 0 && rc == Z_OK) rc = inflate(&zs, Z_NO_FLUSH);
    inflateEnd(&zs);
    return zs.avail_out == 0;
}

// PNG (ISO 15948) as stb_image loads it with req_comp 0: every colour type and bit depth,
// interlaced (Adam7) or not; palette expanded to RGB (RGBA with a tRNS chunk); sub-8-bit gray
// scaled to 0..255 (stbi__depth_scale_table {0, 0xff, 0x55, 0, 0x11}); a gray / RGB colour key
// (tRNS) adds an alpha channel, 0 where the pixel matches the key (compared after the scaling);
// 16-bit samples kept as 16-bit.
bool decode_png(const std::vector<uint8_t>& f, Image& out, std::string& err)
{
    if (f.size() < 8 || std::memcmp(f.data(), kSig, 8) != 0) return err = "not a PNG", false;
    size_t pos = 8;
    int w = 0, h = 0, depth = 0, ctype = -1, interlace = 0;
    bool seen_ihdr = false;
    std::vector<uint8_t> idat, plte, trns;
    while (pos + 8 <= f.size()) {
        const uint32_t len = be32(&f[pos]);
        const char* type = (const char*)&f[pos + 4];
        if (pos + 12 + (size_t)len > f.size()) return err = "truncated PNG chunk", false;
        const uint8_t* d = &f[pos + 8];
        if (!std::memcmp(type, "IHDR", 4)) {
            if (len < 13) return err = "bad IHDR", false;
            w = (int)be32(d);
            h = (int)be32(d + 4);
            depth = d[8];
            ctype = d[9];
            interlace = d[12];
            seen_ihdr = true;
        } else if (!seen_ihdr) {
            return err = "first chunk is not IHDR", false;
        } else if (!std::memcmp(type, "PLTE", 4)) {
            if (len > 768 || len % 3) return err = "bad PLTE", false;
            plte.assign(d, d + len);
        } else if (!std::memcmp(type, "tRNS", 4)) {
            if (!idat.empty()) return err = "tRNS after IDAT", false;
            trns.assign(d, d + len);
        } else if (!std::memcmp(type, "IDAT", 4)) {
            idat.insert(idat.end(), d, d + len);
        } else if (!std::memcmp(type, "IEND", 4)) {
            break;
        } else if (!(type[0] & 0x20)) {  // unknown critical chunk
            return err = std::string("PNG chunk not known: ") + std::string(type, 4), false;
        }
        pos += 12 + len;
    }
    if (w <= 0 || h <= 0 || w > (1 << 24) || h > (1 << 24)) return err = "bad PNG size", false;
    if (interlace > 1) return err = "bad PNG interlace method", false;
    int nc;
    switch (ctype) {
        case 0: nc = 1; break;
        case 2: nc = 3; break;
        case 3: nc = 1; break;
        case 4: nc = 2; break;
        case 6: nc = 4; break;
        default: return err = "bad PNG color type", false;
    }
    if (!(depth == 1 || depth == 2 || depth == 4 || depth == 8 || depth == 16) ||
        (depth < 8 && ctype != 0 && ctype != 3) || (ctype == 3 && depth == 16))
        return err = "bad PNG bit depth", false;
    if (ctype == 3 && plte.empty()) return err = "no PLTE", false;
    const bool key = !trns.empty() && ctype != 3;
    if (key && (ctype == 4 || ctype == 6)) return err = "tRNS with alpha", false;
    if (key && trns.size() != (size_t)nc * 2) return err = "bad tRNS length", false;
    if (ctype == 3 && trns.size() > plte.size() / 3) return err = "bad tRNS length", false;
    if (idat.empty()) return err = "no IDAT", false;

    // the passes: Adam7 (T.2 / ISO 15948 8.2) or the whole image
    struct PassGeom {
        int x0, y0, dx, dy;
    };
    const PassGeom adam7[7] = {{0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4},
                               {0, 2, 2, 4}, {1, 0, 2, 2}, {0, 1, 1, 2}};
    const PassGeom whole[1] = {{0, 0, 1, 1}};
    const PassGeom* passes = interlace ? adam7 : whole;
    const int npass = interlace ? 7 : 1;
    const int bpp = std::max(1, nc * depth / 8);
    size_t need = 0;
    for (int k = 0; k < npass; ++k) {
        const int pw = (w - passes[k].x0 + passes[k].dx - 1) / passes[k].dx;
        const int ph = (h - passes[k].y0 + passes[k].dy - 1) / passes[k].dy;
        if (pw > 0 && ph > 0) need += ((size_t)pw * nc * depth + 7) / 8 * ph + ph;
    }
    std::vector<uint8_t> raw;
    if (!inflate_exact(idat, raw, need)) return err = "PNG inflate failed", false;

    // samples as 16-bit values (8-bit and below are 0..255 after scaling; palette: indices)
    const int scale = ctype == 0 ? (depth == 1 ? 0xFF : depth == 2 ? 0x55 : depth == 4 ? 0x11 : 1) : 1;
    std::vector<uint16_t> smp((size_t)w * h * nc);
    size_t rp = 0;
    std::vector<uint8_t> prev, cur;
    for (int k = 0; k < npass; ++k) {
        const PassGeom& g = passes[k];
        const int pw = (w - g.x0 + g.dx - 1) / g.dx, ph = (h - g.y0 + g.dy - 1) / g.dy;
        if (pw <= 0 || ph <= 0) continue;
        const size_t rowbytes = ((size_t)pw * nc * depth + 7) / 8;
        prev.assign(rowbytes, 0);
        cur.assign(rowbytes, 0);
        for (int y = 0; y < ph; ++y) {
            const uint8_t ft = raw[rp];
            const uint8_t* src = &raw[rp + 1];
            rp += rowbytes + 1;
            for (size_t i = 0; i < rowbytes; ++i) {
                const int a = i >= (size_t)bpp ? cur[i - bpp] : 0;
                const int b = prev[i];
                const int c = i >= (size_t)bpp ? prev[i - bpp] : 0;
                int v = src[i];
                switch (ft) {
                    case 0: break;
                    case 1: v += a; break;
                    case 2: v += b; break;
                    case 3: v += (a + b) >> 1; break;
                    case 4: v += paeth(a, b, c); break;
                    default: return err = "bad PNG filter", false;
                }
                cur[i] = (uint8_t)v;
            }
            const int Y = g.y0 + y * g.dy;
            for (int x = 0; x < pw; ++x) {
                uint16_t* o = &smp[((size_t)Y * w + g.x0 + (size_t)x * g.dx) * nc];
                for (int ch = 0; ch < nc; ++ch) {
                    const size_t e = (size_t)x * nc + ch;
                    int v;
                    if (depth == 16) v = cur[2 * e] << 8 | cur[2 * e + 1];
                    else if (depth == 8) v = cur[e];
                    else v = ((cur[e * depth / 8] >> (8 - depth - (e * depth) % 8)) & ((1 << depth) - 1)) * scale;
                    o[ch] = (uint16_t)v;
                }
            }
            std::swap(prev, cur);
        }
    }

    out = Image();
    out.w = w;
    out.h = h;
    const size_t npx = (size_t)w * h;
    if (ctype == 3) {  // palette: RGB, or RGBA when a tRNS chunk is present
        const int oc = trns.empty() ? 3 : 4;
        const int np = (int)plte.size() / 3;
        out.c = oc;
        out.px8.resize(npx * oc);
        for (size_t i = 0; i < npx; ++i) {
            const int idx = smp[i];
            if (idx >= np) return err = "PNG palette index out of range", false;
            uint8_t* o = &out.px8[i * oc];
            o[0] = plte[3 * idx];
            o[1] = plte[3 * idx + 1];
            o[2] = plte[3 * idx + 2];
            if (oc == 4) o[3] = idx < (int)trns.size() ? trns[idx] : 255;
        }
        return true;
    }
    const int oc = nc + (key ? 1 : 0);
    uint16_t kc[3] = {0, 0, 0};  // the colour key in sample units (scaled like the samples)
    for (int ch = 0; key && ch < nc; ++ch) {
        const int v = trns[2 * ch] << 8 | trns[2 * ch + 1];
        kc[ch] = depth == 16 ? (uint16_t)v : (uint8_t)((v & 255) * (depth < 8 ? scale : 1));
    }
    out.c = oc;
    out.is16 = depth == 16;
    const uint16_t opaque = depth == 16 ? 65535 : 255;
    auto emit = [&](auto& dst) {
        dst.resize(npx * oc);
        for (size_t i = 0; i < npx; ++i) {
            const uint16_t* sp = &smp[i * nc];
            for (int ch = 0; ch < nc; ++ch) dst[i * oc + ch] = (typename std::decay<decltype(dst[0])>::type)sp[ch];
            if (key) {
                bool match = true;
                for (int ch = 0; ch < nc; ++ch) match = match && sp[ch] == kc[ch];
                dst[i * oc + nc] = match ? 0 : opaque;
            }
        }
    };
    if (out.is16) emit(out.px16);
    else emit(out.px8);
    return true;
}

// Binary PGM (P5) / PPM (P6) as stb_image v2.23 reads them: 8-bit samples as stored (a maxval
// below 255 is not rescaled); a maxval above 255 fails to load ("PPM image not 8-bit").
bool decode_pnm(const std::vector<uint8_t>& f, Image& out, std::string& err)
{
    if (f.size() < 3 || f[0] != 'P' || (f[1] != '5' && f[1] != '6'))
        return err = "not a binary PGM/PPM", false;
    size_t p = 2;
    long vals[3];
    for (int k = 0; k < 3; ++k) {
        while (p < f.size() && (std::isspace(f[p]) || f[p] == '#')) {
            if (f[p] == '#')
                while (p < f.size() && f[p] != '\n') ++p;
            else
                ++p;
        }
        long v = 0;
        bool any = false;
        while (p < f.size() && std::isdigit(f[p])) v = v * 10 + (f[p++] - '0'), any = true;
        if (!any) return err = "bad PNM header", false;
        vals[k] = v;
    }
    ++p;  // single whitespace after maxval
    const int w = (int)vals[0], h = (int)vals[1], nc = f[1] == '5' ? 1 : 3;
    const long maxv = vals[2];
    if (w <= 0 || h <= 0 || maxv <= 0) return err = "bad PNM header", false;
    if (maxv > 255) return err = "PPM image not 8-bit (max value > 255)", false;
    const size_t n = (size_t)w * h * nc;
    if (p + n > f.size()) return err = "truncated PNM", false;
    out = Image();
    out.w = w;
    out.h = h;
    out.c = nc;
    out.px8.assign(f.begin() + p, f.begin() + p + n);
    return true;
}

bool write_png(const std::string& fn, const uint8_t* rows, int w, int h, int nc, int depth,
               std::string& err)
{
    const size_t rowbytes = (size_t)w * nc * depth / 8;
    std::vector<uint8_t> raw((rowbytes + 1) * (size_t)h);
    for (int y = 0; y < h; ++y) {
        raw[(rowbytes + 1) * y] = 0;  // filter: none
        std::memcpy(&raw[(rowbytes + 1) * y + 1], rows + rowbytes * y, rowbytes);
    }
    uLongf zlen = compressBound((uLong)raw.size());
    std::vector<uint8_t> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 1) != Z_OK)
        return err = "PNG deflate failed", false;
    FILE* fp = std::fopen(fn.c_str(), "wb");
    if (!fp) return err = "cannot open " + fn + " for writing", false;
    auto chunk = [&](const char* type, const uint8_t* d, uint32_t len) {
        uint8_t hdr[8] = {(uint8_t)(len >> 24), (uint8_t)(len >> 16), (uint8_t)(len >> 8),
                          (uint8_t)len, (uint8_t)type[0], (uint8_t)type[1], (uint8_t)type[2],
                          (uint8_t)type[3]};
        uLong crc = crc32(0L, hdr + 4, 4);
        if (len) crc = crc32(crc, d, len);
        const uint8_t c4[4] = {(uint8_t)(crc >> 24), (uint8_t)(crc >> 16), (uint8_t)(crc >> 8),
                               (uint8_t)crc};
        std::fwrite(hdr, 1, 8, fp);
        if (len) std::fwrite(d, 1, len, fp);
        std::fwrite(c4, 1, 4, fp);
    };
    std::fwrite(kSig, 1, 8, fp);
    const uint8_t ctype = nc == 1 ? 0 : nc == 2 ? 4 : nc == 3 ? 2 : 6;
    const uint8_t ihdr[13] = {(uint8_t)(w >> 24), (uint8_t)(w >> 16), (uint8_t)(w >> 8),
                              (uint8_t)w, (uint8_t)(h >> 24), (uint8_t)(h >> 16),
                              (uint8_t)(h >> 8), (uint8_t)h, (uint8_t)depth, ctype, 0, 0, 0};
    chunk("IHDR", ihdr, 13);
    chunk("IDAT", z.data(), (uint32_t)zlen);
    chunk("IEND", nullptr, 0);
    const bool ok = std::fclose(fp) == 0;
    if (!ok) err = "write failed: " + fn;
    return ok;
}

}  // namespace

bool is_16bit(const std::string& fn)
{  // stbi_is_16_bit (stb_image v2.23): a PNG whose IHDR says 16 bits (PNM is 8-bit only there)
    std::vector<uint8_t> f;
    if (!read_file(fn, f)) return false;
    return f.size() >= 33 && !std::memcmp(f.data(), kSig, 8) && f[24] == 16;
}

bool load_image(const std::string& fn, Image& out, std::string& err)
{
    std::vector<uint8_t> f;
    if (!read_file(fn, f)) return err = "cannot open " + fn, false;
    if (f.size() >= 8 && !std::memcmp(f.data(), kSig, 8)) return decode_png(f, out, err);
    if (f.size() > 2 && f[0] == 'P' && (f[1] == '5' || f[1] == '6')) return decode_pnm(f, out, err);
    if (f.size() > 2 && f[0] == 0xFF && f[1] == 0xD8) {
        if (!decode_jpeg(f, out, err)) return err += ": " + fn, false;
        return true;
    }
    return err = "unknown image format: " + fn, false;
}

// Depth.cpp:376-452: header "PF"/"Pf", "w h", scale; scale < 0 = little-endian data (no swap
// on this little-endian host), scale >= 0 = big-endian (swap).  Rows are returned in file order.
float* load_pfm(const std::string& fn, int* w, int* h, int* c, std::string& err)
{
    FILE* fp = std::fopen(fn.c_str(), "rb");
    if (!fp) return err = "cannot open " + fn, nullptr;
    char buf[1024] = {0};
    int channels = 0, width = 0, height = 0;
    float flag = 0.0f;
    bool ok = std::fscanf(fp, "%1023s", buf) == 1;
    if (ok) channels = !std::strcmp(buf, "PF") ? 3 : (!std::strcmp(buf, "Pf") ? 1 : 0);
    ok = ok && channels && std::fscanf(fp, "%d %d", &width, &height) == 2 &&
         std::fscanf(fp, "%f", &flag) == 1 && width > 0 && height > 0;
    // the scale line ends with one whitespace byte; the reference's "%f\n" would also swallow
    // leading sample bytes that happen to be whitespace, which we do not reproduce
    ok = ok && std::fgetc(fp) != EOF;
    if (!ok) {
        std::fclose(fp);
        return err = "bad PFM header: " + fn, nullptr;
    }
    const size_t n = (size_t)width * height * channels;
    float* img = (float*)std::malloc(n * sizeof(float));
    const size_t got = img ? std::fread(img, sizeof(float), n, fp) : 0;
    std::fclose(fp);
    if (got != n) {
        std::free(img);
        return err = "truncated PFM: " + fn, nullptr;
    }
    if (!(flag < 0.0f)) {
        uint8_t* p = (uint8_t*)img;
        for (size_t i = 0; i < n; ++i, p += 4) {
            std::swap(p[0], p[3]);
            std::swap(p[1], p[2]);
        }
    }
    *w = width;
    *h = height;
    *c = channels;
    return img;
}

bool save_png16(const std::string& fn, const uint16_t* data, int w, int h, std::string& err)
{
    std::vector<uint8_t> be((size_t)w * h * 2);
    for (size_t i = 0; i < (size_t)w * h; ++i) {
        be[2 * i] = (uint8_t)(data[i] >> 8);
        be[2 * i + 1] = (uint8_t)data[i];
    }
    return write_png(fn, be.data(), w, h, 1, 16, err);
}

bool save_png8(const std::string& fn, const uint8_t* data, int w, int h, int c, std::string& err)
{
    if (c < 1 || c > 4) return err = "save_png8: channels must be 1..4", false;
    return write_png(fn, data, w, h, c, 8, err);
}

}  // namespace pfio
