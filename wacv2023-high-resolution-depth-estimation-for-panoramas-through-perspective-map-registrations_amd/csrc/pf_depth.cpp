// pf_depth.cpp -- DepthNamespace facade (include/pf_depth.h) over the panofuse C-ABI.
//
// The reference's MergeDepthMaps (Depth.cpp:754-1041) loads the baseline and the tiles, runs
// SolveDepthToDepth + Depth2DepthTransform per tile, SolveDepthAll, writes the u16 PNG and, with
// a ground truth, ErrorEmap/ErrorData plus the .res.png/.giv.png masks.  Here the loads and the
// file writes stay on the host (they are file formats), every per-pixel computation of the path
// (registration, transform, fusion, quantisation, metrics) is a libpanofuse HIP kernel.
#include "../../include/pf_depth.h"
#include "../../include/panofuse.h"
#include "pf_geom.hpp"
#include "pf_image.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <future>
#include <iostream>
#include <map>
#include <mutex>

Vec2f g_zenith_range((float)PF_D2R(26), (float)PF_D2R(154));  // Depth.cpp:22

namespace {

// One context per device, created on first use (the reference is single-threaded and not
// re-entrant; so is this facade per device).
pf_ctx* facade_ctx()
{
    static std::mutex mu;
    static std::map<int, pf_ctx*> ctxs;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    std::lock_guard<std::mutex> lk(mu);
    auto it = ctxs.find(dev);
    if (it != ctxs.end()) return it->second;
    pf_ctx* c = nullptr;
    if (pf_create(dev, &c) != PF_OK) {
        std::cout << "[panofuse] pf_create(" << dev << ") failed: no usable HIP device" << std::endl;
        return nullptr;
    }
    // ErrorData / ErrorEmap summation order: the facade mirrors Depth.cpp, so by default it sums
    // in the reference's row-major float order (the means the reference prints, bit for bit;
    // ~7.4 ms per 64-panorama call, well under a millisecond more at the facade's batch 1).
    // PF_METRICS_ORDER=tree (panofuse_main --metrics-order tree) opts into the fp64 tree.
    const char* mo = std::getenv("PF_METRICS_ORDER");
    pf_set_metrics_order(c, mo && std::strcmp(mo, "tree") == 0 ? PF_METRICS_TREE
                                                                : PF_METRICS_SEQUENTIAL);
    ctxs[dev] = c;
    return c;
}

struct DevMem {
    void* p = nullptr;
    bool ok = true;
    explicit DevMem(size_t bytes) { ok = bytes == 0 || hipMalloc(&p, bytes) == hipSuccess; }
    ~DevMem()
    {
        if (p) (void)hipFree(p);
    }
    DevMem(const DevMem&) = delete;
    DevMem& operator=(const DevMem&) = delete;
    template <class T>
    T* as() const { return (T*)p; }
};

bool hip_ok(hipError_t e, const char* what)
{
    if (e == hipSuccess) return true;
    std::cout << "[panofuse] " << what << ": " << hipGetErrorString(e) << std::endl;
    return false;
}

bool pf_ok(pf_ctx* c, int rc, const char* what)
{
    if (rc == PF_OK) return true;
    std::cout << "[panofuse] " << what << " failed (" << rc << "): " << pf_last_error(c)
              << std::endl;
    return false;
}

// MergeDepthMaps stores MIN2(range, D2R(359.9)) (Depth.cpp:783-784: a float against a double,
// the double result rounded back to float).
float cap_range(float r)
{
    const double cap = PF_D2R(359.9);
    return (float)((double)r < cap ? (double)r : cap);
}

// Layout of the given maps on the facade context: windows, ranges (as stored in the maps) and
// sizes; channel 0 of every map is packed into `tiles` (host), tile after tile.
bool set_layout(pf_ctx* c, std::vector<DepthNamespace::PerspectiveMap*>& pm,
                std::vector<float>& packed)
{
    std::vector<pf_window> fov(pm.size()), rng(pm.size());
    std::vector<int> tw(pm.size()), th(pm.size());
    size_t total = 0;
    for (size_t i = 0; i < pm.size(); ++i) {
        const DepthNamespace::PerspectiveMap& p = *pm[i];
        if (!p.data || !p.window_set) {
            std::cout << "[panofuse] perspective map " << i << " has no data or no window"
                      << std::endl;
            return false;
        }
        fov[i] = pf_window{p.azimuth_left, p.azimuth_right, p.zenith_top, p.zenith_down};
        rng[i] = pf_window{p.ranges[0], p.ranges[1], p.ranges[2], p.ranges[3]};
        tw[i] = p.width;
        th[i] = p.height;
        total += (size_t)p.width * p.height;
    }
    packed.resize(total);
    size_t off = 0;
    for (auto* p : pm) {
        const size_t n = (size_t)p->width * p->height;
        for (size_t k = 0; k < n; ++k) packed[off + k] = p->data[k * p->channels];
        off += n;
    }
    return pf_ok(c, pf_set_tiles(c, fov.data(), rng.data(), (int)pm.size(), tw.data(), th.data(),
                                 1, 0),
                 "pf_set_tiles");
}

template <class T>
bool upload(DevMem& d, const T* h, size_t n)
{
    return d.ok && hip_ok(hipMemcpy(d.p, h, n * sizeof(T), hipMemcpyHostToDevice), "upload");
}

bool run_metrics(DepthNamespace::EquirectangularMap& gt, const float* given_f,
                 const uint16_t* given16, int w, int h, int given_c, int align_way,
                 bool cap_depth, pf_metrics& m)
{
    pf_ctx* c = facade_ctx();
    if (!c || !gt.data) return false;
    const size_t ng = (size_t)gt.width * gt.height * gt.channels;
    DevMem dg(ng * sizeof(float)), dv(given16 ? (size_t)w * h * 2 : (size_t)w * h * given_c * 4),
        dm(sizeof(pf_metrics));
    if (!upload(dg, gt.data, ng)) return false;
    if (given16 ? !upload(dv, given16, (size_t)w * h) : !upload(dv, given_f, (size_t)w * h * given_c))
        return false;
    if (!dm.ok) return false;
    if (!pf_ok(c, pf_error_metrics(c, dg.as<float>(), gt.width, gt.height, gt.channels,
                                   given16 ? nullptr : dv.as<float>(),
                                   given16 ? dv.as<uint16_t>() : nullptr, w, h, given_c, 1,
                                   g_zenith_range[0], g_zenith_range[1], align_way,
                                   cap_depth ? 1 : 0, dm.as<pf_metrics>()),
               "pf_error_metrics"))
        return false;
    return hip_ok(hipMemcpy(&m, dm.p, sizeof(m), hipMemcpyDeviceToHost), "metrics download");
}

void fill(const pf_metrics& m, float& mse, float& mae, float& mre, float& mselog, float& d1,
          float& d2, float& d3, Vec2f* ls, float* shift)
{
    mse = m.mse;
    mae = m.mae;
    mre = m.mre;
    mselog = m.mselog;
    d1 = m.delta1;
    d2 = m.delta2;
    d3 = m.delta3;
    if (ls) *ls = Vec2f(m.ls_s, m.ls_o);
    if (shift) *shift = m.median_shift;
}

int elapsed_ms(std::chrono::steady_clock::time_point t0)
{
    return (int)std::chrono::duration_cast<std::chrono::milliseconds>(
               std::chrono::steady_clock::now() - t0)
        .count();
}

}  // namespace

bool Save16BitPNG(unsigned short* data, int width, int height, const char* filename)
{
    std::string err;
    if (!pfio::save_png16(filename, data, width, height, err)) {
        std::cout << "[Save16BitPNG] " << err << std::endl;
        return false;
    }
    return true;
}

namespace DepthNamespace {

// ---- EquirectangularMap (Depth.cpp:277-575) ----
EquirectangularMap::~EquirectangularMap() { delete[] data; }

bool EquirectangularMap::Load(std::string& filename, bool mono360)
{
    if (filename.size() >= 3 && filename.compare(filename.size() - 3, 3, "pfm") == 0)
        return LoadPfm(filename, mono360, mono360);
    delete[] data;
    data = nullptr;
    pfio::Image im;
    std::string err;
    if (!pfio::load_image(filename, im, err)) {
        std::cout << "[EquirectangularMap::Load] failed: " << err << std::endl;
        return false;
    }
    width = im.w;
    height = im.h;
    channels = im.c;
    const size_t n = (size_t)width * height * channels;
    data = new float[n];
    if (im.is16)
        for (size_t i = 0; i < n; ++i) data[i] = (float)im.px16[i] / 65535.0f;
    else
        for (size_t i = 0; i < n; ++i) data[i] = (float)im.px8[i] / 255.0f;
    return true;
}

bool EquirectangularMap::LoadPfm(std::string& filename, bool flip_vertical, bool normalize,
                                 const char* save_png_filename)
{
    std::string err;
    float* img = pfio::load_pfm(filename, &width, &height, &channels, err);
    if (!img) {
        std::cout << "load_pfm() failed? " << err << std::endl;
        return false;
    }
    float mn = FLT_MAX, mx = -FLT_MAX;  // Depth.cpp:468-486
    const size_t n = (size_t)width * height * channels;
    for (size_t i = 0; i < n; ++i) {
        if (img[i] < mn) mn = img[i];
        if (img[i] > mx) mx = img[i];
    }
    delete[] data;
    data = new float[n];
    for (int y = 0; y < height; y++)
        for (int x = 0; x < width; x++)
            for (int c = 0; c < channels; c++) {
                const int sy = flip_vertical ? height - 1 - y : y;
                float val = img[((size_t)sy * width + x) * channels + c];
                if (normalize) {
                    val = (val - mn) / (mx - mn);
                } else {  // cap to 0~10 (Depth.cpp:515-520)
                    if (val < 0) val = 0;
                    val = std::min(val / 10.0f, 10.0f);
                }
                data[((size_t)y * width + x) * channels + c] = val;
            }
    std::free(img);
    if (save_png_filename) {
        std::vector<uint8_t> d((size_t)width * height);
        for (size_t i = 0; i < d.size(); ++i) d[i] = (uint8_t)(data[i * channels] * 255.0f);
        if (!pfio::save_png8(save_png_filename, d.data(), width, height, 1, err))
            std::cout << "[LoadPfm] " << err << std::endl;
    }
    return true;
}

float EquirectangularMap::ValueAtCoord(float azi, float zen)  // Depth.cpp:551-556
{
    const int x = (int)(azi / (PF_MYPI_D * 2) * (float)(width - 1));
    const int y = (int)(zen / PF_MYPI_D * (float)(height - 1));
    return data[((size_t)y * width + x) * channels];
}

float EquirectangularMap::ValueAtXY(int x, int y) { return data[((size_t)y * width + x) * channels]; }

double EquirectangularMap::Avg()  // Depth.cpp:563-583
{
    double avg = 0;
    int count = 0;
    for (int y = 0; y < height; y++)
        for (int x = 0; x < width; x++) {
            const float val = data[((size_t)y * width + x) * channels];
            if (val > 0) {
                avg += val;
                count++;
            }
        }
    if (count == 0) return 0;
    avg /= (float)count;
    return avg;
}

// ---- PerspectiveMap (Depth.cpp:45-274) ----
PerspectiveMap::~PerspectiveMap() { delete[] data; }

PerspectiveMap::PerspectiveMap(PerspectiveMap&& o) noexcept { *this = std::move(o); }

PerspectiveMap& PerspectiveMap::operator=(PerspectiveMap&& o) noexcept
{
    if (this != &o) {
        delete[] data;
        width = o.width;
        height = o.height;
        channels = o.channels;
        data = o.data;
        o.data = nullptr;
        azimuth_left = o.azimuth_left;
        azimuth_right = o.azimuth_right;
        zenith_top = o.zenith_top;
        zenith_down = o.zenith_down;
        ranges = o.ranges;
        middle = o.middle;
        hedge = o.hedge;
        vedge = o.vedge;
        corner0 = o.corner0;
        corner1 = o.corner1;
        corner2 = o.corner2;
        corner3 = o.corner3;
        window_set = o.window_set;
    }
    return *this;
}

bool PerspectiveMap::Load(std::string& filename)
{
    delete[] data;
    data = nullptr;
    pfio::Image im;
    std::string err;
    if (!pfio::load_image(filename, im, err)) {
        std::cout << "[PerspectiveMap::Load] failed! " << err << std::endl;
        return false;
    }
    width = im.w;
    height = im.h;
    channels = im.c;
    const size_t n = (size_t)width * height * channels;
    data = new float[n];
    if (im.is16)
        for (size_t i = 0; i < n; ++i) data[i] = (float)im.px16[i] / 65535.0f;
    else
        for (size_t i = 0; i < n; ++i) data[i] = (float)im.px8[i] / 255.0f;
    return true;
}

namespace {
Vec3f vec(const pfgeom::V3& v) { return Vec3f(v.x, v.y, v.z); }
pfgeom::V3 v3(const Vec3f& v) { return pfgeom::V3{v.x, v.y, v.z}; }
pfgeom::Window window_of(const PerspectiveMap& p)
{
    pfgeom::Window w;
    w.middle = v3(p.middle);
    w.hedge = v3(p.hedge);
    w.vedge = v3(p.vedge);
    w.corner0 = v3(p.corner0);
    w.corner1 = v3(p.corner1);
    w.corner2 = v3(p.corner2);
    w.corner3 = v3(p.corner3);
    return w;
}
}  // namespace

// The window geometry (Depth.cpp:120-155) on the host, bit-identical to the reference's (and to
// pf_set_tiles, which recomputes it when the map is handed to the library).
void PerspectiveMap::SetWindow(float aL, float aR, float zT, float zD)
{
    azimuth_left = aL;
    azimuth_right = aR;
    zenith_top = zT;
    zenith_down = zD;
    const pfgeom::Window w = pfgeom::set_window(aL, aR, zT, zD);
    middle = vec(w.middle);
    hedge = vec(w.hedge);
    vedge = vec(w.vedge);
    corner0 = vec(w.corner0);
    corner1 = vec(w.corner1);
    corner2 = vec(w.corner2);
    corner3 = vec(w.corner3);
    window_set = true;
}

Vec2f PerspectiveMap::ToSphericalCoord(float x, float y)  // Depth.cpp:157-166
{
    float az, zen;
    pfgeom::to_spherical_coord(window_of(*this), x, y, az, zen);
    return Vec2f(az, zen);
}

Vec2f PerspectiveMap::SphericalTo2D(float azimuth, float zenith)  // Depth.cpp:168-182
{
    float x, y;
    pfgeom::sph_to_2d(window_of(*this), azimuth, zenith, x, y);
    return Vec2f(x, y);
}

bool PerspectiveMap::Contain(float azimuth, float zenith)  // Depth.cpp:184-207
{
    const Vec2f xy = SphericalTo2D(azimuth, zenith);
    const float threshold = 1e-3f;
    return xy.x >= 0 - threshold && xy.x <= 1 + threshold && xy.y >= 0 - threshold &&
           xy.y <= 1 + threshold;
}

float PerspectiveMap::ValueAtXY(int x, int y) { return data[((size_t)y * width + x) * channels]; }

float PerspectiveMap::Value(float x, float y)  // Depth.cpp:111-118
{
    const int X = (int)(x * (float)(width - 1));
    const int Y = (int)(y * (float)(height - 1));
    return data[((size_t)Y * width + X) * channels];
}

void PerspectiveMap::Depth2DepthTransform(Vec4f& abcd)
{
    pf_ctx* c = facade_ctx();
    if (!c || !data) return;
    const size_t n = (size_t)width * height * channels;
    DevMem d(n * sizeof(float));
    if (!upload(d, data, n)) return;
    const float k[4] = {abcd[0], abcd[1], abcd[2], abcd[3]};
    if (!pf_ok(c, pf_depth_transform(c, d.as<float>(), (long long)width * height, channels, k),
               "pf_depth_transform") ||
        !pf_ok(c, pf_synchronize(c), "pf_synchronize"))
        return;
    hip_ok(hipMemcpy(data, d.p, n * sizeof(float), hipMemcpyDeviceToHost), "download");
}

// ---- free projection functions (Depth.cpp:2955-2971) ----
Vec3f SphericalToWorld(float azimuth, float zenith) { return vec(pfgeom::sph_to_world(azimuth, zenith)); }

Vec2f WorldToSpherical(Vec3f& p)
{
    pfgeom::V3 q = v3(p);
    float az, zen;
    pfgeom::world_to_sph(q, az, zen);
    p = vec(q);
    return Vec2f(az, zen);
}

// ---- Metrics (Depth.h:161-258) ----
bool Metrics::Save(const char* filename)
{
    FILE* fp = std::fopen(filename, "w+");
    if (!fp) {
        std::cout << "fopen failed?" << std::endl;
        return false;
    }
    auto row = [&](const char* name, float g, float r, bool rel_guard) {
        std::fprintf(fp, "%s_given: %f\n", name, g);
        std::fprintf(fp, "%s_result: %f\n", name, r);
        if (rel_guard) std::fprintf(fp, "%s diff: %f\n", name, (r - g) / g);
    };
    row("mse", mse_given, mse_result, mse_given != 0);
    row("mae", mae_given, mae_result, mae_given != 0);
    row("mre", mre_given, mre_result, mre_given != 0);
    row("mselog", mselog_given, mselog_result, mselog_given != 0);
    row("delta1", delta1_given, delta1_result, delta1_given != 0);
    row("delta2", delta2_given, delta2_result, delta2_given != 0);
    row("delta3", delta3_given, delta3_result, delta1_given != 0);  // sic, Depth.h:238
    std::fclose(fp);
    return true;
}

void Metrics::Print()
{
    std::cout << "RMSE " << std::sqrt(mse_given) << "->" << std::sqrt(mse_result) << " ("
              << (std::sqrt(mse_result) - std::sqrt(mse_given)) / std::sqrt(mse_given)
              << ") MAE " << mae_given << "->" << mae_result << " ("
              << (mae_result - mae_given) / mae_given << ") MRE " << mre_given << "->"
              << mre_result << " (" << (mre_result - mre_given) / mre_given << ") RMSElog "
              << std::sqrt(mselog_given) << "->" << std::sqrt(mselog_result) << " ("
              << (std::sqrt(mselog_result) - std::sqrt(mselog_given)) / std::sqrt(mselog_given)
              << ") deltas:" << delta1_given << "->" << delta1_result << "("
              << (delta1_result - delta1_given) << ") , " << delta2_given << "->"
              << delta2_result << "(" << (delta2_result - delta2_given) << ") , "
              << delta3_given << "->" << delta3_result << "(" << (delta3_result - delta3_given)
              << std::endl;
}

// ---- solvers ----
bool SolveDepthToDepth(EquirectangularMap& emap, std::vector<PerspectiveMap>& pmaps,
                       std::vector<bool>& actives, Vec2f& zr, Vec4f& abcd)
{
    // every active map's sample grid in one least-squares problem (Depth.cpp:1274-1376)
    std::vector<PerspectiveMap*> pm;
    for (size_t i = 0; i < actives.size() && i < pmaps.size(); ++i)
        if (actives[i]) pm.push_back(&pmaps[i]);
    if (pm.empty()) {
        std::cout << "[SolveDepthToDepth] no active map" << std::endl;
        return false;
    }
    pf_ctx* c = facade_ctx();
    if (!c || !emap.data) return false;
    std::vector<float> packed;
    if (!set_layout(c, pm, packed)) return false;
    const size_t ne = (size_t)emap.width * emap.height * emap.channels;
    DevMem de(ne * 4), dt(packed.size() * 4), dc(4 * sizeof(float));
    if (!upload(de, emap.data, ne) || !upload(dt, packed.data(), packed.size()) || !dc.ok)
        return false;
    const std::vector<int> all(pm.size(), 1);
    if (!pf_ok(c, pf_register_joint(c, de.as<float>(), emap.width, emap.height, emap.channels,
                                    dt.as<float>(), 1, zr[0], zr[1], 3, all.data(),
                                    dc.as<float>(), nullptr),
               "pf_register_joint"))
        return false;
    float k[4];
    if (!hip_ok(hipMemcpy(k, dc.p, sizeof(k), hipMemcpyDeviceToHost), "download")) return false;
    abcd = Vec4f(k[0], k[1], k[2], k[3]);
    return true;
}

bool SolveDepthAll(EquirectangularMap& emap, std::vector<PerspectiveMap>& pmaps,
                   unsigned short* data, int& out_width, int& out_height, Vec2f& zr,
                   const char* Laplacian_filename)
{
    (void)Laplacian_filename;  // debug dump of the targets in the reference; not produced
    pf_ctx* c = facade_ctx();
    if (!c || !emap.data) return false;
    std::vector<PerspectiveMap*> pm;
    for (auto& p : pmaps) pm.push_back(&p);
    std::vector<float> packed;
    if (!set_layout(c, pm, packed)) return false;
    const size_t ne = (size_t)emap.width * emap.height * emap.channels;
    const size_t no = (size_t)out_width * out_height;
    DevMem de(ne * 4), dt(packed.size() * 4), dout(no * 2);
    if (!upload(de, emap.data, ne) || !upload(dt, packed.data(), packed.size()) || !dout.ok)
        return false;
    if (!pf_ok(c, pf_fuse(c, de.as<float>(), emap.width, emap.height, emap.channels,
                          dt.as<float>(), nullptr, 1, out_width, out_height, zr[0], zr[1],
                          dout.as<uint16_t>()),
               "pf_fuse") ||
        !pf_ok(c, pf_synchronize(c), "pf_synchronize"))  // PF_ETIMEOUT: invalid output
        return false;
    return hip_ok(hipMemcpy(data, dout.p, no * 2, hipMemcpyDeviceToHost), "download");
}

bool SolveDepthBySmoothing(std::vector<PerspectiveMap>& pmaps, unsigned short* data,
                           int& out_width, int& out_height, Vec2f& zr)
{  // Depth.cpp:1773-1878 on the GPU (pf_solve_smoothing)
    pf_ctx* c = facade_ctx();
    if (!c) return false;
    std::vector<PerspectiveMap*> pm;
    for (auto& p : pmaps) pm.push_back(&p);
    std::vector<float> packed;
    if (!set_layout(c, pm, packed)) return false;
    const size_t no = (size_t)out_width * out_height;
    DevMem dt(packed.size() * 4), dout(no * 2);
    if (!upload(dt, packed.data(), packed.size()) || !dout.ok) return false;
    if (!pf_ok(c, pf_solve_smoothing(c, dt.as<float>(), nullptr, 1, out_width, out_height, zr[0],
                                     zr[1], dout.as<uint16_t>()),
               "pf_solve_smoothing"))
        return false;
    // a row-band hand-off that timed out makes the result invalid: report it here, on this
    // call (PF_ETIMEOUT), as SolveDepthAll does for the fusion
    if (!pf_ok(c, pf_synchronize(c), "SolveDepthBySmoothing")) return false;
    return hip_ok(hipMemcpy(data, dout.p, no * 2, hipMemcpyDeviceToHost), "download");
}

bool ErrorData(EquirectangularMap& gt, unsigned short* data, int w, int h, float& mse,
               float& mae, float& mre, float& mselog, float& d1, float& d2, float& d3,
               int align_way, bool cap_depth, Vec2f* ls, float* shift)
{
    pf_metrics m;
    if (!run_metrics(gt, nullptr, data, w, h, 1, align_way, cap_depth, m)) return false;
    fill(m, mse, mae, mre, mselog, d1, d2, d3, ls, shift);
    return true;
}

bool ErrorEmap(EquirectangularMap& gt, EquirectangularMap& given, float& mse, float& mae,
               float& mre, float& mselog, float& d1, float& d2, float& d3, int align_way,
               bool cap_depth, Vec2f* ls, float* shift)
{
    pf_metrics m;
    if (!run_metrics(gt, given.data, nullptr, given.width, given.height, given.channels,
                     align_way, cap_depth, m))
        return false;
    fill(m, mse, mae, mre, mselog, d1, d2, d3, ls, shift);
    return true;
}

bool MergeDepthMaps(std::string& emap_fn, std::vector<std::string>& pmap_fns,
                    std::string& out_fn, std::vector<Vec4f>& fovs, std::vector<Vec4f>& ranges,
                    int out_width, Vec2f& zr, std::string* gt_fn, Metrics* metrics,
                    int* time_Reg, int* time_Laplacian)
{
    const auto t_begin = std::chrono::steady_clock::now();
    EquirectangularMap emap;
    std::vector<PerspectiveMap> pmaps;
    // the ground truth decodes on a host thread while the tiles load and the GPU fuses
    EquirectangularMap gt;
    std::future<bool> gt_loaded;
    if (gt_fn) gt_loaded = std::async(std::launch::async, [&] { return gt.Load(*gt_fn); });
    struct Join {  // never leave with the loader still writing into `gt`
        std::future<bool>& f;
        ~Join()
        {
            if (f.valid()) f.wait();
        }
    } join{gt_loaded};
    if (!emap.Load(emap_fn)) return false;
    const int out_height = out_width / 2;
    if (fovs.size() < pmap_fns.size() || ranges.size() < pmap_fns.size()) {
        std::cout << "[MergeDepthMaps] fewer FOVs/ranges than maps" << std::endl;
        return false;
    }
    pmaps.resize(pmap_fns.size());
    {  // the tiles decode in parallel host threads (zlib inflate is the host-side cost)
        std::vector<std::future<bool>> loads;
        for (size_t i = 0; i < pmap_fns.size(); i++)
            loads.push_back(std::async(std::launch::async,
                                       [&, i] { return pmaps[i].Load(pmap_fns[i]); }));
        bool ok = true;
        for (auto& f : loads) ok = f.get() && ok;
        if (!ok) return false;
    }
    for (size_t i = 0; i < pmap_fns.size(); i++) {  // Depth.cpp:773-787
        PerspectiveMap& p = pmaps[i];
        p.SetWindow(fovs[i][0], fovs[i][1], fovs[i][2], fovs[i][3]);
        p.ranges[0] = cap_range(ranges[i][0]);
        p.ranges[1] = cap_range(ranges[i][1]);
        p.ranges[2] = ranges[i][2];
        p.ranges[3] = ranges[i][3];
    }
    pf_ctx* c = facade_ctx();
    if (!c) return false;
    std::vector<PerspectiveMap*> pm;
    for (auto& p : pmaps) pm.push_back(&p);
    std::vector<float> packed;
    if (!set_layout(c, pm, packed)) return false;
    const size_t ne = (size_t)emap.width * emap.height * emap.channels;
    const size_t no = (size_t)out_width * out_height;
    DevMem de(ne * 4), dt(packed.size() * 4), dc(sizeof(float) * 4 * pmaps.size()),
        dout(no * 2);
    if (!upload(de, emap.data, ne) || !upload(dt, packed.data(), packed.size()) || !dc.ok ||
        !dout.ok)
        return false;
    // registration (Depth.cpp:789-808): every tile alone, cubic, transform fused into fusion
    auto t = std::chrono::steady_clock::now();
    if (!pf_ok(c, pf_register(c, de.as<float>(), emap.width, emap.height, emap.channels,
                              dt.as<float>(), 1, zr[0], zr[1], 3, 0, dc.as<float>(), nullptr),
               "pf_register") ||
        !pf_ok(c, pf_synchronize(c), "pf_synchronize"))
        return false;
    if (time_Reg) *time_Reg = elapsed_ms(t);
    // fusion (Depth.cpp:904-913)
    t = std::chrono::steady_clock::now();
    if (!pf_ok(c, pf_fuse(c, de.as<float>(), emap.width, emap.height, emap.channels,
                          dt.as<float>(), dc.as<float>(), 1, out_width, out_height, zr[0],
                          zr[1], dout.as<uint16_t>()),
               "pf_fuse") ||
        !pf_ok(c, pf_synchronize(c), "pf_synchronize"))
        return false;
    if (time_Laplacian) *time_Laplacian = elapsed_ms(t);
    std::vector<unsigned short> data(no);
    if (!hip_ok(hipMemcpy(data.data(), dout.p, no * 2, hipMemcpyDeviceToHost), "download"))
        return false;
    if (!Save16BitPNG(data.data(), out_width, out_height, out_fn.c_str())) return false;
    std::cout << "...All done! @" << elapsed_ms(t_begin) << std::endl;

    if (gt_fn) {  // Depth.cpp:920-1037
        const int align_way = 1;
        const bool cap_depth = true;
        if (gt_loaded.get()) {
            Metrics local;
            Metrics& M = metrics ? *metrics : local;
            ErrorEmap(gt, emap, M.mse_given, M.mae_given, M.mre_given, M.mselog_given,
                      M.delta1_given, M.delta2_given, M.delta3_given, align_way, cap_depth);
            ErrorData(gt, data.data(), out_width, out_height, M.mse_result, M.mae_result,
                      M.mre_result, M.mselog_result, M.delta1_result, M.delta2_result,
                      M.delta3_result, align_way, cap_depth);
            M.Print();
            // result and baseline masked by the gt's invalid (0) / saturated pixels
            auto mask = [&](int w, int h, auto value_at, const std::string& fn) {
                const int h0 = (int)std::floor(h * zr[0] / PF_MYPI_D);
                const int h1 = (int)std::ceil(h * zr[1] / PF_MYPI_D);
                std::vector<unsigned short> o((size_t)w * h);
                for (int y = 0; y < h; y++)
                    for (int x = 0; x < w; x++) {
                        unsigned short& d = o[(size_t)y * w + x];
                        if (y < h0 || y > h1) {
                            d = 0;
                            continue;
                        }
                        const int X = (int)((float)x * (float)gt.width / (float)w);
                        const int Y = (int)((float)y * (float)gt.height / (float)h);
                        const float g = gt.ValueAtXY(X, Y);
                        d = g == 0 ? 0 : ((double)g >= 1 - 1e-4 ? 65535 : value_at(x, y));
                    }
                Save16BitPNG(o.data(), w, h, fn.c_str());
            };
            auto res = std::async(std::launch::async, [&] {
                mask(out_width, out_height,
                     [&](int x, int y) { return data[(size_t)y * out_width + x]; },
                     out_fn + ".res.png");
            });
            mask(emap.width, emap.height,
                 [&](int x, int y) {
                     return (unsigned short)(emap.ValueAtXY(x, y) * 65535.0f);
                 },
                 out_fn + ".giv.png");
            res.get();
        }
    }
    return true;
}

}  // namespace DepthNamespace

// ---- mode-0 driver (Main.cpp:331-687) ----
void pf_leres_layout(std::vector<Vec4f>& fovs, std::vector<Vec4f>& ranges)
{
    // Main.cpp:788-843, the active "5-fold for LeReS" block
    const float margin = (float)PF_D2R(3);
    float a0[5], a1[5];
    for (int i = 0; i < 5; ++i) {
        a0[i] = (float)(PF_D2R(72.0 * i) - margin);
        a1[i] = (float)(PF_D2R(72.0 * (i + 1)) + margin);
    }
    const double fz[3][2] = {{18, 94}, {52, 128}, {86, 162}};
    const double rz[3][2] = {{25, 60}, {60, 120}, {120, 155}};
    fovs.clear();
    ranges.clear();
    for (int b = 0; b < 3; ++b)
        for (int i = 0; i < 5; ++i)
            fovs.push_back(Vec4f(a0[i], a1[i], (float)PF_D2R(fz[b][0]), (float)PF_D2R(fz[b][1])));
    for (int b = 0; b < 3; ++b)
        for (int i = 0; i < 5; ++i)
            ranges.push_back(Vec4f(a1[i] - margin, a0[i] + margin, (float)PF_D2R(rz[b][0]),
                                   (float)PF_D2R(rz[b][1])));
}

int pf_create_depth_panoramas(const std::string& rgb_folder, const std::string& gt_folder,
                              const std::string& baseline_folder,
                              const std::string& result_folder, const std::string& tile_dir,
                              const std::string& tile_ext, int out_width, int shard,
                              int nshards)
{
    namespace fs = std::filesystem;
    std::vector<Vec4f> fovs, ranges;
    pf_leres_layout(fovs, ranges);
    std::vector<std::string> rgb;  // AllFilesInFolder (Main.cpp:50-83): files only
    std::error_code ec;
    for (const auto& e : fs::directory_iterator(rgb_folder, ec))
        if (!e.is_directory()) rgb.push_back(e.path().filename().string());
    if (ec) {
        std::cout << "[CreateDepthPanoramas] cannot list " << rgb_folder << std::endl;
        return 1;
    }
    std::sort(rgb.begin(), rgb.end());
    if (nshards > 1) {  // panorama sharding over processes / GPUs
        std::vector<std::string> mine;
        for (size_t i = (size_t)shard; i < rgb.size(); i += (size_t)nshards) mine.push_back(rgb[i]);
        rgb.swap(mine);
    }
    std::cout << "[CreateDepthPanormas] #RGB_filenames:" << rgb.size() << std::endl;
    auto join = [](const std::string& dir, const std::string& name) {
        return (fs::path(dir) / name).string();
    };
    std::vector<DepthNamespace::Metrics> all;
    for (size_t i = 0; i < rgb.size(); i++) {
        const std::string rawname = rgb[i].substr(0, rgb[i].find_last_of('.'));
        // baseline naming by result folder (Main.cpp:499-517)
        std::string base = join(baseline_folder, rawname + ".jpg");
        if (result_folder.find("Slicenet") != std::string::npos ||
            result_folder.find("slicenet") != std::string::npos)
            base = join(baseline_folder, rawname + ".jpg.slicenet.png");
        else if (result_folder.find("unifuse") != std::string::npos)
            base = join(baseline_folder, rawname + ".unifuse.jpg");
        else if (result_folder.find("hohonet") != std::string::npos)
            base = join(baseline_folder, rawname + ".depth.png");
        std::string gt = join(gt_folder, rawname + ".png");  // Main.cpp:520-530
        const size_t k = gt.find("_rgb");
        if (k != std::string::npos) gt.replace(k, 4, "_depth");
        std::string out = join(result_folder, rawname + ".png");
        if (fs::exists(out)) {  // Main.cpp:552-561
            std::cout << i << "/" << rgb.size() << " skip!" << std::endl;
            continue;
        }
        std::cout << i << "/" << rgb.size() << " baseline:" << base << std::endl;
        std::cout << "gt:" << gt << std::endl << "output_filename:" << out << std::endl;
        std::vector<std::string> tiles;  // Main.cpp:563-587
        for (const Vec4f& f : fovs) {
            char name[512];
            std::snprintf(name, sizeof(name), "%s.%d_%d_%d_%d.", rawname.c_str(),
                          (int)std::round(f[0] / PF_MYPI_D * 180.0),
                          (int)std::round(f[1] / PF_MYPI_D * 180.0),
                          (int)std::round(f[2] / PF_MYPI_D * 180.0),
                          (int)std::round(f[3] / PF_MYPI_D * 180.0));
            std::string fn = join(tile_dir, std::string(name) + (tile_ext == "auto" ? "jpg" : tile_ext));
            if (tile_ext == "auto" && !fs::exists(fn)) fn = join(tile_dir, std::string(name) + "png");
            tiles.push_back(fn);
        }
        DepthNamespace::Metrics m;
        int tr = 0, tl = 0;
        if (!DepthNamespace::MergeDepthMaps(base, tiles, out, fovs, ranges, out_width,
                                            g_zenith_range, &gt, &m, &tr, &tl)) {
            std::cout << "[CreateDepthPanorma] MergeDepthMaps #" << i << " failed!" << std::endl;
            return 1;
        }
        m.Save((join(result_folder, rawname) + ".aligned.txt").c_str());
        all.push_back(m);
        std::cout << "time_Reg:" << tr << " time_Laplacian:" << tl << std::endl;
    }
    if (!all.empty()) {  // averages (Main.cpp:612-676)
        double rg = 0, rr = 0, mg = 0, mr = 0, d1g = 0, d1r = 0;
        for (auto& m : all) {
            rg += std::sqrt(m.mse_given);
            rr += std::sqrt(m.mse_result);
            mg += m.mae_given;
            mr += m.mae_result;
            d1g += m.delta1_given;
            d1r += m.delta1_result;
        }
        const double n = (double)all.size();
        std::cout << "RMSE_given:" << rg / n << " RMSE_result:" << rr / n
                  << " MAE_given:" << mg / n << " MAE_result_avg:" << mr / n
                  << " delta1_given:" << d1g / n << " delta1_result:" << d1r / n << std::endl;
    }
    return 0;
}

// ---- RGB tile export (Main.cpp:242-326 SaveCubeMap, called for every panorama by
// CreateDepthPanoramas, Main.cpp:399-430) ----
// Tile size as SaveCubeMap sizes its viewport: width 1024, height round(1024 / aspect) with
// aspect = tan(fovx/2) / tan(fovy/2) (the window-size clamps of a small screen do not apply).
static void rgb_tile_size(const Vec4f& f, int& w, int& h)
{
    const float fovx = (float)((f[1] - f[0]) / PF_MYPI_D * 180.0);
    const float fovy = (float)((f[3] - f[2]) / PF_MYPI_D * 180.0);
    const float aspect = (float)(std::tan(PF_D2R(fovx) / 2) / std::tan(PF_D2R(fovy) / 2));
    w = 1024;
    h = (int)std::round((float)w / aspect);
}

int pf_export_rgb_tiles(const std::string& rgb_folder, const std::string& tile_dir)
{
    namespace fs = std::filesystem;
    std::vector<Vec4f> fovs, ranges;
    pf_leres_layout(fovs, ranges);
    pf_ctx* c = facade_ctx();
    if (!c) return 1;
    const int n = (int)fovs.size();
    std::vector<pf_window> fw(n), rw(n);
    std::vector<int> tw(n), th(n);
    size_t total = 0;
    for (int i = 0; i < n; ++i) {
        fw[i] = pf_window{fovs[i][0], fovs[i][1], fovs[i][2], fovs[i][3]};
        rw[i] = pf_window{ranges[i][0], ranges[i][1], ranges[i][2], ranges[i][3]};
        rgb_tile_size(fovs[i], tw[i], th[i]);
        total += (size_t)tw[i] * th[i] * 3;
    }
    if (!pf_ok(c, pf_set_tiles(c, fw.data(), rw.data(), n, tw.data(), th.data(), 1, 1),
               "pf_set_tiles"))
        return 1;
    std::vector<std::string> rgb;
    std::error_code ec;
    for (const auto& e : fs::directory_iterator(rgb_folder, ec))
        if (!e.is_directory()) rgb.push_back(e.path().string());
    if (ec) {
        std::cout << "[SaveCubeMap] cannot list " << rgb_folder << std::endl;
        return 1;
    }
    std::sort(rgb.begin(), rgb.end());
    fs::create_directories(tile_dir, ec);
    std::vector<uint8_t> tiles(total);
    for (const std::string& fn : rgb) {
        pfio::Image im;
        std::string err;
        if (!pfio::load_image(fn, im, err)) {
            std::cout << "[SaveCubeMap] " << err << std::endl;
            return 1;
        }
        // the GL texture is RGB8: gray replicated, alpha dropped, 16-bit reduced to the top byte
        std::vector<uint8_t> pano((size_t)im.w * im.h * 3);
        for (size_t p = 0; p < (size_t)im.w * im.h; ++p)
            for (int k = 0; k < 3; ++k) {
                const int ch = im.c >= 3 ? k : 0;
                pano[p * 3 + k] = im.is16 ? (uint8_t)(im.px16[p * im.c + ch] >> 8)
                                          : im.px8[p * im.c + ch];
            }
        DevMem dp(pano.size()), dt(total);
        if (!upload(dp, pano.data(), pano.size()) || !dt.ok) return 1;
        if (!pf_ok(c, pf_warp_rgb(c, dp.as<uint8_t>(), im.w, im.h, 1, dt.as<uint8_t>()),
                   "pf_warp_rgb") ||
            !hip_ok(hipMemcpy(tiles.data(), dt.p, total, hipMemcpyDeviceToHost), "download"))
            return 1;
        const std::string base = fs::path(fn).filename().string();
        const std::string rawname = base.substr(0, base.find_last_of('.'));
        size_t off = 0;
        for (int i = 0; i < n; ++i) {
            char name[512];
            std::snprintf(name, sizeof(name), "%s.%d_%d_%d_%d.jpg", rawname.c_str(),
                          (int)std::round(fovs[i][0] / PF_MYPI_D * 180.0),
                          (int)std::round(fovs[i][1] / PF_MYPI_D * 180.0),
                          (int)std::round(fovs[i][2] / PF_MYPI_D * 180.0),
                          (int)std::round(fovs[i][3] / PF_MYPI_D * 180.0));
            // stbi_write_jpg(filename, w, h, 3, data, w * 3): the reference passes the row stride
            // as the quality, which stb clamps to 100 (no chroma subsampling), Main.cpp:319-320
            if (!pfio::save_jpeg((fs::path(tile_dir) / name).string(), tiles.data() + off, tw[i],
                                 th[i], 3, tw[i] * 3, err)) {
                std::cout << "[SaveCubeMap] " << err << std::endl;
                return 1;
            }
            off += (size_t)tw[i] * th[i] * 3;
        }
        std::cout << "[SaveCubeMap] " << fn << ": " << n << " tiles" << std::endl;
    }
    return 0;
}

// ---- C-ABI helpers for bindings and tests (include/pf_depth.h) ----
extern "C" int pfd_load_map(const char* fn, int is_emap, float* out, long long cap, int* w, int* h,
                            int* c)
{
    std::string f(fn);
    DepthNamespace::EquirectangularMap e;
    DepthNamespace::PerspectiveMap p;
    const bool ok = is_emap ? e.Load(f) : p.Load(f);
    if (!ok) return -1;
    const int W = is_emap ? e.width : p.width, H = is_emap ? e.height : p.height,
              C = is_emap ? e.channels : p.channels;
    *w = W;
    *h = H;
    *c = C;
    const long long n = (long long)W * H * C;
    if (out && cap >= n) std::memcpy(out, is_emap ? e.data : p.data, sizeof(float) * n);
    return 0;
}

extern "C" int pfd_decode_image(const char* fn, void* out, long long cap, int* w, int* h, int* c,
                                int* is16)
{
    pfio::Image im;
    std::string err;
    if (!pfio::load_image(fn, im, err)) {
        std::cout << "[pfd_decode_image] " << err << std::endl;
        return -1;
    }
    *w = im.w;
    *h = im.h;
    *c = im.c;
    *is16 = im.is16 ? 1 : 0;
    const long long n = (long long)im.w * im.h * im.c * (im.is16 ? 2 : 1);
    if (!out || cap < n) return -2;
    std::memcpy(out, im.is16 ? (const void*)im.px16.data() : (const void*)im.px8.data(), n);
    return 0;
}

extern "C" int pfd_is_16_bit(const char* fn) { return pfio::is_16bit(fn) ? 1 : 0; }

extern "C" int pfd_save_jpeg(const char* fn, const uint8_t* px, int w, int h, int c, int quality,
                             int flip)
{
    std::string err;
    if (!pfio::save_jpeg(fn, px, w, h, c, quality, err, flip != 0)) {
        std::cout << "[pfd_save_jpeg] " << err << std::endl;
        return -1;
    }
    return 0;
}

extern "C" int pfd_save_png16(const char* fn, const uint16_t* data, int w, int h)
{
    return Save16BitPNG(const_cast<unsigned short*>(data), w, h, fn) ? 0 : -1;
}

extern "C" void pfd_leres_layout(float* fovs, float* ranges)
{
    std::vector<Vec4f> f, r;
    pf_leres_layout(f, r);
    for (size_t i = 0; i < f.size(); ++i)
        for (int k = 0; k < 4; ++k) {
            fovs[4 * i + k] = f[i][k];
            ranges[4 * i + k] = r[i][k];
        }
}
