// pf_api.hip -- C-ABI of libpanofuse (include/panofuse.h): context, layout preparation and the
// stream-ordered launch sequences of the drop-in entry points.
//
// Host-side preparation done once per layout / fusion level (all tiny): the tile windows
// (PerspectiveMap::SetWindow, Depth.cpp:120-155), the per-level tile boxes (Depth.cpp:1497-1562)
// and the separable trig tables of the fusion and registration grids, computed with glibc's
// sincosf/tanf exactly as the reference calls them.  Everything per panorama runs on the GPU.
#include "../../include/panofuse.h"
#include "pf_geom.hpp"
#include "pf_internal.hpp"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

using namespace pf;

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

struct LevelCache {
    int out_w = 0, out_h = 0;
    uint32_t zr0 = 0, zr1 = 0;
    int nlevels = 0;
    LevelDims dims[4];
    DevBuf box[4], cols[4], rows[4], tapbox[4], tapmap[4], hcol[4];
    DevBuf tmask[4];  // per targets patch, the tiles whose box meets it (k_targets_multi)
    // (pixel, tile) pairs of the pixels covered by three or more tiles, sorted by pixel then
    // tile (the sharded fusion recomputes their sums in tile order: pf_fuse_multicover)
    DevBuf mcpairs[4];
    int nmc[4] = {0, 0, 0, 0};
    std::vector<TileBox> box_h[4];
    // separable-coverage certificate of each level: a band pixel is covered iff it lies in rows
    // h0+1..h1-1 and in a column of a fixed set that excludes column 0.  Enables the packed
    // Jacobi form (pf_jacobi.hip), with hcol[l][X] = 0.5 on covered columns, 0 elsewhere.
    bool full[4] = {false, false, false, false};
    // tap-grid points of each level (one tile texel gathered per point): the targets stage's
    // algorithmic read count
    long long taps[4] = {0, 0, 0, 0};
    // the one-launch targets of every level (k_targets_multi): (level, patch) gather order
    DevBuf tgt_order;
    int tgt_nentries = 0;
};

}  // namespace

struct pf_ctx {
    int device = 0;
    int num_cu = 256;
    hipStream_t stream = nullptr;
    std::string err;
    // layout
    int ntiles = 0, tile_c = 1;
    int solver = PF_SOLVER_LM;  // degree-3 registration solver (pf_set_solver)
    int metrics_order = PF_METRICS_TREE;  // pf_set_metrics_order
    std::vector<pf_window> fov, rng;
    std::vector<int> tw_h, th_h;
    bool layout_ok = false;  // the stored layout was set completely
    std::vector<TileGeom> geom_h;
    std::vector<RegGrid> reg_h;
    long long tile_elems = 0, npix_max = 0, rgb_elems = 0;
    DevBuf geom, reg, rcols, rrows, rgb_off;
    DevBuf reg_sidx;                       // registration sample indices (k_regidx), for the
    int reg_sidx_key[3] = {-1, -1, -1};    // (ew, eh, ec) of the baseline they were built for
    std::vector<RgbCam> cams_h;  // GL cameras of the RGB warp (SaveCubeMap), host only
    // RGB warp taps for one panorama size (rgb_taps_host), built on first use
    int rgb_pw = 0, rgb_ph = 0;
    DevBuf rgbtap;
    // LDS-staged RGB warp (k_warp_rgb_box): patch boxes, per-pixel box index and weights
    DevBuf rgbpatch, rgbunits, rgbloc, rgbw;
    int n_rgbpatch = 0;
    bool rgb_staged = false;
    LevelCache lc;
    bool reg_valid = false;
    uint32_t reg_zr0 = 0, reg_zr1 = 0;
    // E->P depth warp for one panorama size (pf_warp.hip): tile patches with their panorama
    // boxes, per tile pixel the corner index in its box and the (fx, fy) weights; built on
    // first use
    int wmap_pw = 0, wmap_ph = 0, npatch = 0;
    DevBuf wmap, wfxy, wpatch, wunits;  // wunits: the ragged footprints' unit table
    std::vector<WarpPatch> wpatch_grid_h;  // the layout's plain 32x32 patch grid
    // workspace
    DevBuf buf[3], lnorm, coeffs, lsum_ws, metrics_ws, reg_sums, reg_active;
    // SolveDepthBySmoothing (pf_smooth.hip): boxes, grid tables, per-pixel source and mask
    DevBuf sm_box, sm_cols, sm_rows, sm_src, sm_mask;
    // its compacted pixel list (k_smooth_iter_list), cached for one (boxes, size, band) key
    DevBuf sm_list, sm_off;
    std::vector<SmoothBox> sm_key_boxes;
    int sm_key[4] = {0, 0, 0, 0}, sm_nk = 0, sm_nb = 0, sm_smin = 0, sm_smax = -1;
    // row-band smoothing (k_smooth_band): ticket, timeouts, per-block step flags
    DevBuf sm_sync;
    uint32_t sm_tk = 0, sm_fb = 1;
    // level-0 seed index tables of the streaming Jacobi (run_jacobi), keyed by level and emap
    DevBuf seed_ecol, seed_erow;
    // resident level kernel (pf_jres.hip): hand-off rows, and the sync words ([0] ticket
    // counter, [1] spin timeouts, [2..] one flag per row block); tickets and flags are
    // monotone across launches (jres_tk, jres_fb), so nothing is reset between launches
    DevBuf jres_x, jres_sync;
    uint32_t jres_tk = 0, jres_fb = 1;
    int jres_mode = -1, jres_nb = 0;  // pf_set_jacobi_engine (-1: not set, PF_JRES decides)
    double jacobi_share = 1.0;  // pf_set_jacobi_share: the chip share the pass plans assume
    // timeout reporting: a resident launch whose wait times out also raises this flag in
    // coherent pinned host memory (a system-scope store from the kernel, no extra stream work);
    // jres_check reports a raised flag once as PF_ETIMEOUT and lowers it
    uint32_t* jres_err_h = nullptr;
    int jres_fault = 0;  // pf_debug_jres_fault: spin_log2 for the next resident launch (0: off)
    int smooth_fault = 0;  // pf_debug_smooth_fault: spin_log2 for the next row-band smoothing
    int seed_key[5] = {0, 0, 0, 0, 0};
    // stage profiling
    struct Span {
        int stage;
        hipEvent_t a, b;
        double bytes;
        long long launches;
    };
    bool prof_on = false;
    std::vector<Span> spans;
    std::vector<hipEvent_t> event_pool;
    // side stream for the finer levels' target planes (fuse_range), created on first use
    hipStream_t aux = nullptr;
    hipEvent_t ev_fork = nullptr, ev_tgt[4] = {};
    // end of each level's sweeps in the last fusion (pf_stream_wait_level), created on first use
    hipEvent_t ev_level[4] = {};
    int nlev_recorded = 0;
};

namespace {
hipEvent_t take_event(pf_ctx* c)
{
    if (!c->event_pool.empty()) {
        hipEvent_t e = c->event_pool.back();
        c->event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

// Records an event pair around a stage when profiling is on (RAII: end on scope exit).
struct StageTimer {
    pf_ctx* c;
    long idx = -1;
    StageTimer(pf_ctx* c_, int stage, double bytes, long long launches) : c(c_)
    {
        if (!c->prof_on) return;
        pf_ctx::Span s{stage, take_event(c), take_event(c), bytes, launches};
        (void)hipEventRecord(s.a, c->stream);
        c->spans.push_back(s);
        idx = (long)c->spans.size() - 1;
    }
    ~StageTimer()
    {
        if (idx >= 0) (void)hipEventRecord(c->spans[idx].b, c->stream);
    }
    void set_launches(long long n)
    {
        if (idx >= 0) c->spans[idx].launches = n;
    }
};
}  // namespace

// ---------------------------------------------------------------------------------------------
static int fail(pf_ctx* c, int code, const char* fmt, ...)
{
    char msg[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(msg, sizeof(msg), fmt, ap);
    va_end(ap);
    if (c) c->err = msg;
    return code;
}

#define HIPCHK(ctx, expr)                                                                    \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return fail(ctx, PF_EHIP, "%s: %s", #expr, hipGetErrorString(e_));               \
    } while (0)

static int ensure(pf_ctx* c, DevBuf& b, size_t bytes)
{
    if (b.bytes >= bytes) return PF_OK;
    if (b.p) {
        (void)hipStreamSynchronize(c->stream);
        (void)hipFree(b.p);
        b.p = nullptr;
        b.bytes = 0;
    }
    if (bytes == 0) return PF_OK;
    if (hipMalloc(&b.p, bytes) != hipSuccess)
        return fail(c, PF_ENOMEM, "hipMalloc(%zu) failed", bytes);
    b.bytes = bytes;
    return PF_OK;
}

static void release(DevBuf& b)
{
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
}

template <class T>
static int upload(pf_ctx* c, DevBuf& b, const std::vector<T>& v)
{
    int rc = ensure(c, b, v.size() * sizeof(T) + 16);
    if (rc) return rc;
    if (!v.empty())
        HIPCHK(c, hipMemcpyAsync(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice,
                                 c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));  // host vector may die after return
    return PF_OK;
}

// ---------------------------------------------------------------------------------------------
// Host geometry: PerspectiveMap::SetWindow in Imath Vec3<float> semantics (pf_geom.hpp).
namespace {
TileGeom set_window(const pf_window& f, int w, int h, int ch)
{  // PerspectiveMap::SetWindow, Depth.cpp:120-155
    using namespace pfgeom;
    const Window win = pfgeom::set_window(f.az_left, f.az_right, f.zen_top, f.zen_down);
    TileGeom g{};
    g.middle[0] = win.middle.x; g.middle[1] = win.middle.y; g.middle[2] = win.middle.z;
    g.hedge[0] = win.hedge.x; g.hedge[1] = win.hedge.y; g.hedge[2] = win.hedge.z;
    g.vedge[0] = win.vedge.x; g.vedge[1] = win.vedge.y; g.vedge[2] = win.vedge.z;
    g.corner0[0] = win.corner0.x; g.corner0[1] = win.corner0.y; g.corner0[2] = win.corner0.z;
    const V3 p0mp = {win.middle.x - 0.0f, win.middle.y - 0.0f, win.middle.z - 0.0f};  // p0 - p
    g.mm = dot(p0mp, win.middle);
    g.hl = length(win.hedge);
    g.vl = length(win.vedge);
    g.w = w;
    g.h = h;
    g.c = ch;
    return g;
}

// RGB camera of SaveCubeMap (Main.cpp:246-269: gluLookAt toward the window centre, up = z;
// gluPerspective fovy / aspect), in double.
RgbCam rgb_cam(const pf_window& f)
{
    float azc = (f.az_right + f.az_left) / 2, zenc = (f.zen_down + f.zen_top) / 2;
    float fovx = (float)((f.az_right - f.az_left) / PF_MYPI * 180.0);
    float fovy = (float)((f.zen_down - f.zen_top) / PF_MYPI * 180.0);
    float aspect = (float)(tan(fovx / 180.0 * PF_MYPI / 2) / tan(fovy / 180.0 * PF_MYPI / 2));
    RgbCam cam{};
    double fv[3] = {cos((double)azc) * sin((double)zenc), sin((double)azc) * sin((double)zenc),
                    cos((double)zenc)};
    double fl = sqrt(fv[0] * fv[0] + fv[1] * fv[1] + fv[2] * fv[2]);
    for (int k = 0; k < 3; k++) cam.f[k] = fv[k] / fl;
    double sv[3] = {cam.f[1], -cam.f[0], 0.0};
    double sl = sqrt(sv[0] * sv[0] + sv[1] * sv[1]);
    cam.s[0] = sv[0] / sl; cam.s[1] = sv[1] / sl; cam.s[2] = 0.0;
    cam.u[0] = cam.s[1] * cam.f[2] - cam.s[2] * cam.f[1];
    cam.u[1] = cam.s[2] * cam.f[0] - cam.s[0] * cam.f[2];
    cam.u[2] = cam.s[0] * cam.f[1] - cam.s[1] * cam.f[0];
    cam.ty = tan((double)fovy / 180.0 * PF_MYPI / 2);
    cam.tx = cam.ty * (double)aspect;
    return cam;
}

LevelDims level_dims(int out_w, int out_h, float zr0, float zr1, int level)
{  // Depth.cpp:1420-1437, 1650-1675
    LevelDims L{};
    int max_level = out_w >= 4096 ? 4 : 3;
    L.nlevels = max_level;
    L.w = (int)(out_w / pow(2, max_level - 1 - level));
    L.h = (int)(out_h / pow(2, max_level - 1 - level));
    L.h0 = (int)floor((double)((float)L.h * zr0) / PF_MYPI);
    L.h1 = (int)ceil((double)((float)L.h * zr1) / PF_MYPI);
    static const int it3[3] = {200, 100, 50};
    static const int it4[4] = {200, 150, 100, 50};
    L.iters = max_level == 3 ? it3[level] : it4[level];
    return L;
}

TileBox tile_box(const pf_window& r, const LevelDims& L)
{  // Depth.cpp:1497-1562 (enlargement disabled at :1522/:1543; the clamps stay)
    int w = L.w, h = L.h;
    int x0 = (int)round((double)r.az_left / (2 * PF_MYPI) * (double)(w - 1));
    int x1 = (int)round((double)r.az_right / (2 * PF_MYPI) * (double)(w - 1));
    int y0 = (int)round((double)r.zen_top / PF_MYPI * (double)(h - 1));
    int y1 = (int)round((double)r.zen_down / PF_MYPI * (double)(h - 1));
    int xs = x1 >= x0 ? 1 : -1;
    x0 = x0 < 0 ? 0 : (x0 >= w ? w - 1 : x0);
    x1 = x1 < 0 ? 0 : (x1 >= w ? w - 1 : x1);
    y0 = y0 < 0 ? 0 : (y0 >= h ? h - 1 : y0);
    y1 = y1 < 0 ? 0 : (y1 >= h ? h - 1 : y1);
    if (y0 <= L.h0) y0 = L.h0 + 1;
    if (y1 >= L.h1) y1 = L.h1 - 1;
    TileBox b{};
    b.x0 = x0; b.x1 = x1; b.y0 = y0; b.y1 = y1; b.xs = xs;
    return b;
}

// Fusion grid coordinates (Depth.cpp:1456,1591): az = (float)xx/(float)(w-1)*2*MYPI and
// zen = (float)yy/(float)(h-1)*MYPI, rounded to float by the Vec2f; xx in [-1, w], yy in [-1, h].
void grid_tables(const LevelDims& L, std::vector<GridCol>& cols, std::vector<GridRow>& rows)
{
    cols.resize(L.w + 2);
    rows.resize(L.h + 2);
    for (int xx = -1; xx <= L.w; xx++) {
        float az = (float)((double)((float)xx / (float)(L.w - 1) * 2.0f) * PF_MYPI);
        GridCol c{};
        c.az = az;
        sincosf(az, &c.sa, &c.ca);
        cols[xx + 1] = c;
    }
    for (int yy = -1; yy <= L.h; yy++) {
        float zen = (float)((double)((float)yy / (float)(L.h - 1)) * PF_MYPI);
        GridRow r{};
        r.zen = zen;
        sincosf(zen, &r.sz, &r.cz);
        rows[yy + 1] = r;
    }
}
}  // namespace

// ---------------------------------------------------------------------------------------------
extern "C" {

const char* pf_version(void) { return "panofuse 0.1 (gfx950)"; }

int pf_create(int device, pf_ctx** out)
{
    if (!out) return PF_EINVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return PF_EHIP;
    if (hipSetDevice(device) != hipSuccess) return PF_EHIP;
    pf_ctx* c = new pf_ctx();
    c->device = device;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
        c->num_cu = prop.multiProcessorCount;
    *out = c;
    return PF_OK;
}

void pf_destroy(pf_ctx* c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    DevBuf* all[] = {&c->geom, &c->reg, &c->reg_sidx, &c->rcols, &c->rrows, &c->rgbtap, &c->rgb_off, &c->rgbpatch, &c->rgbunits, &c->rgbloc, &c->rgbw,
                     &c->buf[0], &c->buf[1], &c->buf[2], &c->lnorm, &c->coeffs, &c->lsum_ws,
                     &c->wmap, &c->wfxy, &c->wpatch, &c->wunits, &c->metrics_ws, &c->reg_sums,
                     &c->reg_active, &c->sm_box, &c->sm_cols, &c->sm_rows, &c->sm_src,
                     &c->sm_mask, &c->seed_ecol, &c->seed_erow, &c->jres_x, &c->jres_sync,
                     &c->sm_sync, &c->sm_list, &c->sm_off};
    for (DevBuf* b : all) release(*b);
    for (int l = 0; l < 4; l++) {
        release(c->lc.box[l]);
        release(c->lc.cols[l]);
        release(c->lc.rows[l]);
        release(c->lc.tapbox[l]);
        release(c->lc.tmask[l]);
        release(c->lc.tapmap[l]);
        release(c->lc.hcol[l]);
        release(c->lc.mcpairs[l]);
    }
    release(c->lc.tgt_order);

    for (auto& s : c->spans) {
        (void)hipEventDestroy(s.a);
        (void)hipEventDestroy(s.b);
    }
    for (hipEvent_t e : c->event_pool) (void)hipEventDestroy(e);
    if (c->aux) {
        (void)hipStreamSynchronize(c->aux);
        (void)hipStreamDestroy(c->aux);
        (void)hipEventDestroy(c->ev_fork);
        for (hipEvent_t e : c->ev_tgt) (void)hipEventDestroy(e);
    }
    for (hipEvent_t e : c->ev_level)
        if (e) (void)hipEventDestroy(e);
    if (c->jres_err_h) (void)hipHostFree(c->jres_err_h);
    delete c;
}

const char* pf_last_error(const pf_ctx* c) { return c ? c->err.c_str() : "null context"; }

int pf_stream_wait_level(pf_ctx* c, int level, void* hip_stream)
{
    if (!c || level < 0 || level >= c->nlev_recorded || !c->ev_level[level]) return PF_EINVAL;
    HIPCHK(c, hipStreamWaitEvent((hipStream_t)hip_stream, c->ev_level[level], 0));
    return PF_OK;
}

int pf_set_jacobi_share(pf_ctx* c, double share)
{
    if (!c || !(share > 0.0 && share <= 1.0)) return PF_EINVAL;
    c->jacobi_share = share;
    return PF_OK;
}

// SIMDs the pass plans of this context count on: the chip times the context's share
static int plan_simds(const pf_ctx* c)
{
    const int n = (int)(4.0 * c->num_cu * c->jacobi_share + 0.5);
    return n < 4 ? 4 : n;
}

int pf_set_jacobi_engine(pf_ctx* c, int mode, int row_blocks)
{
    if (!c || mode < 0 || mode > 1 || row_blocks < 0) return PF_EINVAL;
    c->jres_mode = mode;
    c->jres_nb = row_blocks;
    return PF_OK;
}

// PF_ETIMEOUT once for every new batch of timed-out resident-kernel waits whose count has
// reached the host (the copy queued behind each resident launch); never blocks.
static int jres_check(pf_ctx* c)
{
    if (!c->jres_err_h || !__atomic_load_n(c->jres_err_h, __ATOMIC_ACQUIRE)) return PF_OK;
    __atomic_store_n(c->jres_err_h, 0u, __ATOMIC_RELEASE);
    return fail(c, PF_ETIMEOUT, "resident kernel (Jacobi level or row-band smoothing): "
                "hand-off wait(s) timed out (%d resident-Jacobi timeouts so far on this context, "
                "pf_jres_errors); the output of that call is invalid", pf_jres_errors(c));
}

// The coherent pinned PF_ETIMEOUT flag shared by the resident Jacobi kernel and the row-band
// smoothing kernel: allocated and zeroed once (hipHostMalloc does not promise zeroed memory);
// PF_JRES_ERRHOST=0 leaves it out (timeouts then only count into pf_jres_errors).
static int ensure_err_host(pf_ctx* c)
{
    static const bool errhost = !(getenv("PF_JRES_ERRHOST") && atoi(getenv("PF_JRES_ERRHOST")) == 0);
    if (c->jres_err_h || !errhost) return PF_OK;
    HIPCHK(c, hipHostMalloc((void**)&c->jres_err_h, sizeof(uint32_t),
                            hipHostMallocMapped | hipHostMallocCoherent));
    __atomic_store_n(c->jres_err_h, 0u, __ATOMIC_RELEASE);
    return PF_OK;
}

int pf_debug_smooth_fault(pf_ctx* c, int spin_log2)
{
    if (!c || spin_log2 < 4 || spin_log2 > 24) return PF_EINVAL;
    c->smooth_fault = spin_log2;
    return PF_OK;
}

int pf_debug_jres_fault(pf_ctx* c, int spin_log2)
{
    if (!c || spin_log2 < 4 || spin_log2 > 24) return PF_EINVAL;
    c->jres_fault = spin_log2;
    return PF_OK;
}

int pf_jres_errors(pf_ctx* c)
{
    if (!c) return PF_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (!c->jres_sync.p) return 0;
    uint32_t n = 0;
    HIPCHK(c, hipMemcpy(&n, (const uint32_t*)c->jres_sync.p + 1, sizeof(n), hipMemcpyDeviceToHost));
    return (int)(n & 0x7FFFFFFF);
}

int pf_set_solver(pf_ctx* c, int solver)
{
    if (!c) return PF_EINVAL;
    if (solver != PF_SOLVER_LM && solver != PF_SOLVER_NORMAL)
        return fail(c, PF_EINVAL, "pf_set_solver: unknown solver %d", solver);
    c->solver = solver;
    return PF_OK;
}

int pf_set_stream(pf_ctx* c, void* s)
{
    if (!c) return PF_EINVAL;
    c->stream = (hipStream_t)s;
    return PF_OK;
}

int pf_profile_enable(pf_ctx* c, int on)
{
    if (!c) return PF_EINVAL;
    double ms[PF_NSTAGES], by[PF_NSTAGES];
    long long ln[PF_NSTAGES];
    int rc = pf_profile_read(c, ms, by, ln);  // drains and recycles pending spans
    c->prof_on = on != 0;
    return rc;
}

int pf_profile_read(pf_ctx* c, double* ms, double* bytes, long long* launches)
{
    if (!c) return PF_EINVAL;
    for (int s = 0; s < PF_NSTAGES; s++) {
        if (ms) ms[s] = 0;
        if (bytes) bytes[s] = 0;
        if (launches) launches[s] = 0;
    }
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (auto& s : c->spans) {
        float t = 0.0f;
        HIPCHK(c, hipEventElapsedTime(&t, s.a, s.b));
        if (ms) ms[s.stage] += t;
        if (bytes) bytes[s.stage] += s.bytes;
        if (launches) launches[s.stage] += s.launches;
        c->event_pool.push_back(s.a);
        c->event_pool.push_back(s.b);
    }
    c->spans.clear();
    return PF_OK;
}

int pf_synchronize(pf_ctx* c)
{
    if (!c) return PF_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return jres_check(c);
}

int pf_level_info(int out_w, int out_h, float zr0, float zr1, int level, int* w, int* h,
                  int* h0, int* h1, int* iters, int* nlevels)
{
    if (out_w < 8 || out_h < 4) return PF_EINVAL;
    int nl = out_w >= 4096 ? 4 : 3;
    if (level < 0 || level >= nl) return PF_EINVAL;
    LevelDims L = level_dims(out_w, out_h, zr0, zr1, level);
    if (w) *w = L.w;
    if (h) *h = L.h;
    if (h0) *h0 = L.h0;
    if (h1) *h1 = L.h1;
    if (iters) *iters = L.iters;
    if (nlevels) *nlevels = L.nlevels;
    return PF_OK;
}

int pf_probe_warp_coords(const pf_window* fov, int tile_w, int tile_h, int pw, int ph,
                         uint32_t* wxy, float* wfxy)
{
    if (!fov || !wxy || !wfxy || tile_w < 2 || tile_h < 2 || pw < 2 || ph < 2 || pw >= 65536 ||
        ph >= 65536)
        return PF_EINVAL;
    const TileGeom g = set_window(*fov, tile_w, tile_h, 1);
    warp_coords_host(g, pw, ph, wxy, wfxy);
    return PF_OK;
}

int pf_probe_rgb_taps(const pf_window* fov, int tile_w, int tile_h, int pw, int ph,
                      uint32_t* taps)
{
    static_assert(sizeof(RgbTap) == 16, "RgbTap is 4 words");
    if (!fov || !taps || tile_w < 1 || tile_h < 1 || pw < 2 || ph < 2 || pw >= 65536 ||
        ph >= 65536)
        return PF_EINVAL;
    rgb_taps_host(rgb_cam(*fov), tile_w, tile_h, pw, ph, reinterpret_cast<RgbTap*>(taps));
    return PF_OK;
}

int pf_set_tiles(pf_ctx* c, const pf_window* fovs, const pf_window* ranges, int ntiles,
                 const int* tile_w, const int* tile_h, int tile_c, int cap_ranges)
{
    if (!c) return PF_EINVAL;
    if (!fovs || !ranges || !tile_w || !tile_h || ntiles <= 0 || ntiles > 4096 || tile_c <= 0)
        return fail(c, PF_EINVAL, "pf_set_tiles: bad arguments (ntiles=%d, tile_c=%d)", ntiles,
                    tile_c);
    HIPCHK(c, hipSetDevice(c->device));
    const double cap = 359.9 / 180.0 * PF_MYPI;  // D2R(359.9), MergeDepthMaps :783-784
    {
        // The same layout again (a per-panorama caller such as the DepthNamespace facade):
        // keep the per-layout caches (level boxes, tap maps, registration grids, warp maps).
        bool same = c->layout_ok && c->ntiles == ntiles && c->tile_c == tile_c &&
                    (int)c->tw_h.size() == ntiles && (int)c->th_h.size() == ntiles;
        for (int i = 0; same && i < ntiles; i++) {
            pf_window r = ranges[i];
            if (cap_ranges) {
                r.az_left = (float)((double)r.az_left < cap ? (double)r.az_left : cap);
                r.az_right = (float)((double)r.az_right < cap ? (double)r.az_right : cap);
            }
            same = !memcmp(&c->fov[i], &fovs[i], sizeof(pf_window)) &&
                   !memcmp(&c->rng[i], &r, sizeof(pf_window)) && c->tw_h[i] == tile_w[i] &&
                   c->th_h[i] == tile_h[i];
        }
        if (same) return PF_OK;
    }
    c->layout_ok = false;
    c->ntiles = ntiles;
    c->tile_c = tile_c;
    c->fov.assign(fovs, fovs + ntiles);
    c->rng.assign(ranges, ranges + ntiles);
    c->tw_h.assign(tile_w, tile_w + ntiles);
    c->th_h.assign(tile_h, tile_h + ntiles);
    c->geom_h.resize(ntiles);
    c->reg_h.resize(ntiles);
    std::vector<RgbCam> cams(ntiles);
    std::vector<long long> rgb_off(ntiles);
    long long off = 0, roff = 0, npmax = 0;
    for (int i = 0; i < ntiles; i++) {
        if (tile_w[i] < 2 || tile_h[i] < 2)
            return fail(c, PF_EINVAL, "tile %d: size %dx%d (need >= 2x2)", i, tile_w[i], tile_h[i]);
        pf_window& r = c->rng[i];
        if (cap_ranges) {
            r.az_left = (float)((double)r.az_left < cap ? (double)r.az_left : cap);
            r.az_right = (float)((double)r.az_right < cap ? (double)r.az_right : cap);
        }
        TileGeom g = set_window(fovs[i], tile_w[i], tile_h[i], tile_c);
        if (!(g.hl > 0.0f) || !(g.vl > 0.0f))
            return fail(c, PF_EINVAL, "tile %d: degenerate window (pole or zero FOV)", i);
        g.off = off;
        g.pix_off = (int)(off / tile_c);
        off += (long long)tile_w[i] * tile_h[i] * tile_c;
        if (off / tile_c > INT32_MAX)
            return fail(c, PF_EINVAL, "layout has more than 2^31 tile pixels");
        rgb_off[i] = roff;
        roff += (long long)tile_w[i] * tile_h[i] * 3;
        long long np = (long long)tile_w[i] * tile_h[i];
        if (np > npmax) npmax = np;
        c->geom_h[i] = g;
        cams[i] = rgb_cam(fovs[i]);
    }
    c->tile_elems = off;
    c->rgb_elems = roff;
    c->npix_max = npmax;
    c->lc.out_w = 0;  // boxes and registration grids depend on the ranges: rebuild lazily
    c->reg_valid = false;
    c->wmap_pw = c->wmap_ph = 0;
    c->rgb_pw = c->rgb_ph = 0;
    c->cams_h = cams;
    std::vector<WarpPatch> patches;
    const int pe = warp_patch_edge(), peh = warp_patch_height();
    for (int i = 0; i < ntiles; i++)
        for (int y = 0; y < tile_h[i]; y += peh)
            for (int x = 0; x < tile_w[i]; x += pe) patches.push_back(WarpPatch{i, x, y, 0, 0, 0, 0, 0, 0, 0});
    c->npatch = (int)patches.size();
    c->wpatch_grid_h = patches;
    int rc;
    if ((rc = upload(c, c->wpatch, patches))) return rc;
    if ((rc = upload(c, c->geom, c->geom_h))) return rc;
    if ((rc = upload(c, c->rgb_off, rgb_off))) return rc;
    c->layout_ok = true;
    return PF_OK;
}

}  // extern "C"

// Registration tables depend on the zenith range; built per call (tiny, cached by value).
static int prepare_registration(pf_ctx* c, float zr0, float zr1)
{
    uint32_t b0, b1;
    memcpy(&b0, &zr0, 4);
    memcpy(&b1, &zr1, 4);
    if (c->reg_valid && b0 == c->reg_zr0 && b1 == c->reg_zr1) return PF_OK;
    const float subd = (float)(1 / 180.0 * PF_MYPI);
    std::vector<GridCol> rcols;
    std::vector<GridRow> rrows;
    int nsamp_total = 0;
    for (int i = 0; i < c->ntiles; i++) {
        const pf_window& r = c->rng[i];
        RegGrid rg{};
        rg.cols = (int)roundf(fabsf(r.az_right - r.az_left) / subd);
        float top = zr0 > r.zen_top ? zr0 : r.zen_top;      // MAX2 (:1301)
        float down = zr1 < r.zen_down ? zr1 : r.zen_down;   // MIN2 (:1302)
        rg.rows = (int)roundf(fabsf(down - top) / subd);
        // an empty grid (the reference divides by 0 there) is an error only for a tile that is
        // solved (check_reg_grids); an inactive tile of a joint solve may have one
        if (rg.cols < 0) rg.cols = 0;
        if (rg.rows < 0) rg.rows = 0;
        rg.col_off = (int)rcols.size();
        rg.row_off = (int)rrows.size();
        rg.soff = nsamp_total;
        for (int k = 0; k <= rg.cols; k++) {  // :1334
            GridCol e{};
            e.az = r.az_left + (r.az_right - r.az_left) * (float)k / (float)rg.cols;
            sincosf(e.az, &e.sa, &e.ca);
            rcols.push_back(e);
        }
        for (int k = 0; k <= rg.rows; k++) {  // :1335
            GridRow e{};
            e.zen = top + (down - top) * (float)k / (float)rg.rows;
            sincosf(e.zen, &e.sz, &e.cz);
            rrows.push_back(e);
        }
        c->reg_h[i] = rg;
        nsamp_total += (rg.cols + 1) * (rg.rows + 1);
    }
    int rc;
    if ((rc = upload(c, c->reg, c->reg_h))) return rc;
    if ((rc = upload(c, c->rcols, rcols))) return rc;
    if ((rc = upload(c, c->rrows, rrows))) return rc;
    c->reg_valid = true;
    c->reg_sidx_key[0] = -1;  // the sample indices follow the grids
    c->reg_zr0 = b0;
    c->reg_zr1 = b1;
    return PF_OK;
}

// The tiles that will be solved must have a non-empty sample grid (Depth.cpp:1334-1335 divides
// by cols and rows); active == nullptr means every tile.
// The registration samples' indices for this baseline size (k_regidx), rebuilt when the grids
// or the baseline size change; stream-ordered before the k_register launches that read them.
static const int2* reg_sample_index(pf_ctx* c, int ew, int eh, int ec)
{
    if (c->reg_sidx_key[0] == ew && c->reg_sidx_key[1] == eh && c->reg_sidx_key[2] == ec)
        return (const int2*)c->reg_sidx.p;
    long long n = 0;
    int maxn = 0;
    for (const RegGrid& g : c->reg_h) {
        const int k = (g.cols + 1) * (g.rows + 1);
        n += k;
        maxn = k > maxn ? k : maxn;
    }
    if (n <= 0 || ensure(c, c->reg_sidx, sizeof(int2) * (size_t)n) != PF_OK) return nullptr;
    launch_regidx(c->stream, (const TileGeom*)c->geom.p, (const RegGrid*)c->reg.p,
                  (const GridCol*)c->rcols.p, (const GridRow*)c->rrows.p, c->ntiles, maxn, ew,
                  eh, ec, (int2*)c->reg_sidx.p);
    if (hipGetLastError() != hipSuccess) return nullptr;
    c->reg_sidx_key[0] = ew;
    c->reg_sidx_key[1] = eh;
    c->reg_sidx_key[2] = ec;
    return (const int2*)c->reg_sidx.p;
}

static int check_reg_grids(pf_ctx* c, const int* active)
{
    for (int i = 0; i < c->ntiles; i++) {
        if (active && !active[i]) continue;
        const RegGrid& rg = c->reg_h[i];
        if (rg.cols <= 0 || rg.rows <= 0)
            return fail(c, PF_EINVAL,
                        "tile %d: registration grid %dx%d is empty (the reference divides by 0)",
                        i, rg.cols, rg.rows);
    }
    return PF_OK;
}

static int prepare_levels(pf_ctx* c, int out_w, int out_h, float zr0, float zr1)
{
    uint32_t b0, b1;
    memcpy(&b0, &zr0, 4);
    memcpy(&b1, &zr1, 4);
    LevelCache& lc = c->lc;
    if (lc.out_w == out_w && lc.out_h == out_h && lc.zr0 == b0 && lc.zr1 == b1) return PF_OK;
    if (out_w < 8 || out_h < 8)
        return fail(c, PF_EINVAL, "output %dx%d too small", out_w, out_h);
    if ((long long)out_w * out_h >= (1LL << 31))  // per-panorama pixel indices are 32-bit
        return fail(c, PF_EINVAL, "output %dx%d too large", out_w, out_h);
    int nl = out_w >= 4096 ? 4 : 3;
    for (int l = 0; l < nl; l++) {
        LevelDims L = level_dims(out_w, out_h, zr0, zr1, l);
        if (L.w < 4 || L.h < 4 || L.h0 < 1 || L.h1 > L.h - 2 || L.h0 >= L.h1)
            return fail(c, PF_EINVAL,
                        "level %d: %dx%d with band [%d,%d] (zenith range must stay inside "
                        "(0, pi) by a row)",
                        l, L.w, L.h, L.h0, L.h1);
        if (l > 0 && (L.w != 2 * lc.dims[l - 1].w || L.h != 2 * lc.dims[l - 1].h))
            return fail(c, PF_EINVAL, "output %dx%d is not divisible by 2^%d", out_w, out_h,
                        nl - 1);
        lc.dims[l] = L;
        std::vector<TileBox> boxes(c->ntiles);
        std::vector<int> cover((size_t)L.w * L.h, 0);
        for (int p = 0; p < c->ntiles; p++) {
            boxes[p] = tile_box(c->rng[p], L);
            const TileBox& b = boxes[p];
            if (b.x0 == b.x1)
                return fail(c, PF_EDEGENERATE,
                            "tile %d at level %d: box x0 == x1 == %d (the reference never "
                            "terminates here)",
                            p, l, b.x0);
            for (int X = b.x0; X != b.x1; X += b.xs)
                for (int Y = b.y0; Y <= b.y1; Y++)
                    if (++cover[(size_t)Y * L.w + X] > PF_MAX_COVER)
                        return fail(c, PF_EINVAL, "pixel (%d,%d) covered by more than %d tiles",
                                    X, Y, PF_MAX_COVER);
        }
        lc.box_h[l] = boxes;
        {
            std::vector<int2> mc;
            for (size_t o = 0; o < cover.size(); o++) {
                if (cover[o] <= 2) continue;
                const int Y = (int)(o / L.w), X = (int)(o % L.w);
                for (int p = 0; p < c->ntiles; p++) {
                    const TileBox& b = boxes[p];
                    const bool in = Y >= b.y0 && Y <= b.y1 &&
                                    (b.xs > 0 ? (X >= b.x0 && X < b.x1) : (X <= b.x0 && X > b.x1));
                    if (in) mc.push_back(make_int2((int)o, p));
                }
            }
            lc.nmc[l] = (int)mc.size();
            int rc2;
            if ((rc2 = upload(c, lc.mcpairs[l], mc))) return rc2;
        }
        std::vector<float> hcol(L.w, 0.0f);
        bool full = L.h0 + 1 < L.h1;
        for (int X = 0; X < L.w && full; X++)
            hcol[X] = cover[(size_t)(L.h0 + 1) * L.w + X] > 0 ? 0.5f : 0.0f;
        full = full && hcol[0] == 0.0f;
        for (int Y = L.h0; Y <= L.h1 && full; Y++)
            for (int X = 0; X < L.w; X++)
                if ((cover[(size_t)Y * L.w + X] > 0) != (hcol[X] != 0.0f && Y > L.h0 && Y < L.h1)) {
                    full = false;
                    break;
                }
        lc.full[l] = full;
        std::vector<GridCol> cols;
        std::vector<GridRow> rows;
        grid_tables(L, cols, rows);
        int rc;
        {   // per targets patch of this level, mask words of the tiles whose box meets it (the
            // device's box_meets on the patch rectangle targets_patch uses)
            const int pw_ = targets_patch_w(), ph_ = targets_patch_h();
            const int npx = (L.w + pw_ - 1) / pw_, npy = (L.h1 - L.h0 + 1 + ph_ - 1) / ph_;
            const int nmw = (c->ntiles + 31) / 32;
            std::vector<uint32_t> tm((size_t)npx * npy * nmw, 0u);
            for (int pid = 0; pid < npx * npy; pid++) {
                const int X0 = (pid % npx) * pw_, Y0 = L.h0 + (pid / npx) * ph_;
                const int X1 = std::min(X0 + pw_ - 1, L.w - 1), Y1 = std::min(Y0 + ph_ - 1, L.h1);
                for (int p = 0; p < c->ntiles; p++)
                    if (box_meets(boxes[p], X0, X1, Y0, Y1))
                        tm[(size_t)pid * nmw + p / 32] |= 1u << (p % 32);
            }
            if ((rc = upload(c, lc.tmask[l], tm))) return rc;
        }
        if ((rc = upload(c, lc.box[l], boxes))) return rc;
        if ((rc = upload(c, lc.hcol[l], hcol))) return rc;
        if ((rc = upload(c, lc.cols[l], cols))) return rc;
        if ((rc = upload(c, lc.rows[l], rows))) return rc;
        // tap-index maps: every tile's box plus a one-pixel ring (pf_targets.hip)
        std::vector<TapBox> tbs(c->ntiles);
        long long moff = 0, maxpts = 0;
        for (int p = 0; p < c->ntiles; p++) {
            const TileBox& b = boxes[p];
            TapBox t{};
            if (b.y0 <= b.y1) {
                int xlo = b.xs > 0 ? b.x0 : b.x1 + 1, xhi = b.xs > 0 ? b.x1 - 1 : b.x0;
                t.xmin = xlo - 1;
                t.ymin = b.y0 - 1;
                t.nx = xhi - xlo + 3;
                t.ny = b.y1 - b.y0 + 3;
            }
            t.off = moff;
            long long np = (long long)t.nx * t.ny;
            moff += np;
            if (np > maxpts) maxpts = np;
            tbs[p] = t;
        }
        if ((rc = upload(c, lc.tapbox[l], tbs))) return rc;
        if ((rc = ensure(c, lc.tapmap[l], sizeof(int32_t) * (moff + 1)))) return rc;
        lc.taps[l] = moff;
        launch_tapmap(c->stream, (const TileGeom*)c->geom.p, (const TapBox*)lc.tapbox[l].p,
                      c->ntiles, maxpts, (const GridCol*)lc.cols[l].p,
                      (const GridRow*)lc.rows[l].p, (int32_t*)lc.tapmap[l].p);
        HIPCHK(c, hipGetLastError());
    }
    {
        // gather order of k_targets_multi: zenith bands = the coarsest level's patch rows; per
        // band the finest level's patches first, then each coarser level's patches of that band
        const int pw_ = targets_patch_w(), ph_ = targets_patch_h();
        int npy[4], npx[4];
        for (int l = 0; l < nl; l++) {
            npx[l] = (lc.dims[l].w + pw_ - 1) / pw_;
            npy[l] = (lc.dims[l].h1 - lc.dims[l].h0 + 1 + ph_ - 1) / ph_;
        }
        std::vector<int2> order;
        for (int j = 0; j < npy[0]; j++)
            for (int l = nl - 1; l >= 0; l--)
                for (int r = 0; r < npy[l]; r++) {
                    const int band = std::min(npy[0] - 1, (int)((long long)r * npy[0] / npy[l]));
                    if (band != j) continue;
                    for (int x = 0; x < npx[l]; x++) order.push_back(make_int2(l, r * npx[l] + x));
                }
        int rc;
        if ((rc = upload(c, lc.tgt_order, order))) return rc;
        lc.tgt_nentries = (int)order.size();
    }
    lc.nlevels = nl;
    lc.out_w = out_w;
    lc.out_h = out_h;
    lc.zr0 = b0;
    lc.zr1 = b1;
    return PF_OK;
}

static int check_common(pf_ctx* c, int batch)
{
    if (!c) return PF_EINVAL;
    if (c->ntiles <= 0) return fail(c, PF_ESTATE, "no tile layout: call pf_set_tiles first");
    if (batch <= 0 || batch > 65535) return fail(c, PF_EINVAL, "batch %d out of range", batch);
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, PF_EHIP, "hipSetDevice failed");
    return PF_OK;
}

static int check_emap(pf_ctx* c, const float* emap, int ew, int eh, int ec)
{
    if (!emap || ew < 2 || eh < 2 || ec < 1)
        return fail(c, PF_EINVAL, "bad emap %p %dx%dx%d", (const void*)emap, ew, eh, ec);
    if ((long long)ew * eh * ec >= (1LL << 31))  // 32-bit emap indices (run_jacobi's seed tables)
        return fail(c, PF_EINVAL, "emap %dx%dx%d too large", ew, eh, ec);
    return PF_OK;
}

// Jacobi pass geometry: lanes own C columns, strips carry a Tp-column halo (Tp >= T, rounded to
// C so vector rows stay aligned); the sweep depth and row chunking of every pass come from the
// cost model of plan_level().  Env overrides for tuning runs: PF_JT (largest T), PF_JOVH (per-step
// overhead in update units), PF_JC=4 (4 columns per lane, builds with PF_JACOBI_C4 only).
struct JacobiTuning {
    // columns per lane: 2 (default); PF_JC=3 / 4 force those forms, PF_JC=0 lets the cost model
    // pick per level.  Round 6 measured C = 3 (192-column strips, 10 % less halo at level 1, 5 %
    // at level 2, but its L ring in LDS and 224 VGPRs: two waves per SIMD) slower on MI355X: T10
    // passes 100-103 / 343-355 us at levels 1 / 2 against 92 / 296 us for C = 2 (serial C3 trace),
    // and the cost model, which does not see that, would pick it (with T8 / T5 passes: 4.2 ms)
    int C = 2, Tmax = 10;
    double step_overhead = 3.0, lone_cycles = 4.0;  // swept on MI355X (profiles/r02/jacobi; recipe: tools/gpu_round.sh ab)
    double c4_eff = 23.0 / 26.0;  // packed C=4 issue per pixel-update relative to C=2
    double pipe_overhead = 1.0;   // pipelined engine: barrier + exchange per step, update units
    // per pass, in the cost units of best_chunks (~10 ns each at C3): a launch's fixed cost
    // (dispatch, ramp, drain; a few us).  Without it the planner cut the batch-1 levels into
    // hundreds of tiny passes (C5 on one GPU: 173 passes, Jacobi 2.11 ms; with it 63 passes,
    // 1.60 ms; C2 latency 0.97 -> 0.82 ms; the batch-64 plans are unchanged).  PF_JLAUNCH=...
    double launch_cost = 300.0;
};

static JacobiTuning jacobi_tuning()
{
    JacobiTuning t;
    if (const char* e = getenv("PF_JC")) t.C = atoi(e) == 4 ? 4 : (atoi(e) == 3 ? 3 : (atoi(e) == 0 ? 0 : 2));
    if (const char* e = getenv("PF_JC4EFF")) t.c4_eff = atof(e);
    if (const char* e = getenv("PF_JT")) t.Tmax = atoi(e);
    if (const char* e = getenv("PF_JOVH")) t.step_overhead = atof(e);
    if (const char* e = getenv("PF_JC1")) t.lone_cycles = atof(e);
    if (const char* e = getenv("PF_JPOVH")) t.pipe_overhead = atof(e);
    if (const char* e = getenv("PF_JLAUNCH")) t.launch_cost = atof(e);
    if (t.Tmax < 1) t.Tmax = 1;
    return t;
}

// One pass: depth T, nchunks row chunks.  Its nstrips*batch*nchunks waves each run
// rows_per_chunk + 3T + ~4 steps of T*C updates (lagged levels, halo, 6-step alignment), and
// they run in ceil(waves / resident) rounds, so the pass costs ~ rounds * steps * (T + o) with o
// the per-step overhead (loads, LDS ring, store) in update units.  Whole rounds matter: at the
// small levels a "one wave per slot" grid left the last round 20-80% empty.
// The halo columns of a strip on each side: T, rounded up to C for the even forms so each lane's
// C-vector (and the one vector store per lane) stays aligned; the C == 3 form stores per column.
static int strip_halo(int T, int C) { return C == 3 ? T : (T + C - 1) / C * C; }

struct PassPlan {
    int T = 1, nchunks = 1;
    int stages = 1;  // > 1: the pipelined engine (k_jpipe), T/stages levels per wave
    double cost = 0;
};

static PassPlan best_chunks(int T, int C, int band_rows, int w, int batch, int per_simd,
                            int nsimd, double ovh, double c1, double c4_eff, int stages = 1)
{
    // VALU work of one step of one wave in update units: T/stages levels of C updates, per-update
    // issue of the C form
    const double lv = (double)T / stages;
    const double work = C == 4 ? lv * 2.0 * c4_eff : (C == 3 ? lv * 1.5 : lv);
    PassPlan best;
    best.T = T;
    best.stages = stages;
    best.cost = 1e300;
    const int Tp = strip_halo(T, C);
    const long long per = (long long)((w + 64 * C - 2 * Tp - 1) / (64 * C - 2 * Tp)) * batch;
    const long long slots = (long long)per_simd * nsimd;
    for (int n = 1; n <= band_rows; n++) {
        const int rows = (band_rows + n - 1) / n;
        if (n > 1 && (band_rows + rows - 1) / rows < n) continue;  // same as a smaller n
        // rounds of resident waves; in each, a SIMD holding W waves issues one VALU
        // instruction per 2 cycles shared among them, and a lone wave one per ~c1 cycles
        const long long waves = per * n * stages;
        double cyc = 0;
        for (long long left = waves; left > 0; left -= slots) {
            const long long in_round = left < slots ? left : slots;
            const double W = (double)((in_round + nsimd - 1) / nsimd);
            cyc += (2.0 * W > c1 ? 2.0 * W : c1);
        }
        const double cost = cyc * (rows + 3.0 * T + 4.0) * (work + ovh);
        if (cost < best.cost) {
            best.cost = cost;
            best.nchunks = n;
        }
    }
    return best;
}

// Sweep depths for a level: a shortest-path split of `iters` into passes from the supported
// menu (<= tcap), each with its best chunking.
static std::vector<PassPlan> plan_level(pf_ctx* c, const LevelDims& L, int C, int tcap, int batch,
                                        bool fast, int band_rows = 0)
{
    static const JacobiTuning tune = jacobi_tuning();
    static const int menu[] = {10, 8, 5, 4, 2, 1};
    if (band_rows <= 0) band_rows = L.h1 - L.h0 + 1;
    PassPlan opt[11];
    for (int T : menu)
        if (T <= tcap && jstream_supported_T(T))
            opt[T] = best_chunks(T, C, band_rows, L.w, batch,
                                 jstream_waves_per_cu(C, T, fast) / 4, 4 * c->num_cu,
                                 tune.step_overhead, tune.lone_cycles, tune.c4_eff);
    // the pipelined engine (2 waves per strip-chunk), packed form only; PF_JPIPE=0 disables it,
    // PF_JPIPE=1 takes it wherever it exists, otherwise the cost model decides
    static const char* pe = getenv("PF_JPIPE");
    const int pmode = pe ? atoi(pe) : 2;
    if (fast && C == 2 && pmode != 0)
        for (int T : menu) {
            if (T > tcap || T % 2 || !jpipe_supported(2, T / 2)) continue;
            PassPlan pp = best_chunks(T, C, band_rows, L.w, batch,
                                      jpipe_waves_per_cu(2, T / 2) / 4, 4 * c->num_cu,
                                      tune.step_overhead + tune.pipe_overhead, tune.lone_cycles,
                                      tune.c4_eff, 2);
            if (pmode == 1 || pp.cost < opt[T].cost || !jstream_supported_T(T)) opt[T] = pp;
        }
    if (fast && C == 2 && pmode == 1)  // forced: the single-wave engine only where no pipe fits
        for (int T : menu)
            if (opt[T].stages == 1) opt[T].cost *= 1e6;
    // tuning runs: PF_JTONLY<w>=T restricts the level of width w to depth-T passes (and depths 1
    // and 2 for a remainder)
    char tkey[32];
    snprintf(tkey, sizeof(tkey), "PF_JTONLY%d", L.w);
    const int tonly = getenv(tkey) ? atoi(getenv(tkey)) : 0;
    std::vector<double> dp(L.iters + 1, 1e300);
    std::vector<int> choice(L.iters + 1, 1);
    dp[0] = 0;
    for (int r = 1; r <= L.iters; r++)
        for (int T : menu) {
            if (T > r || T > tcap || !jstream_supported_T(T)) continue;
            if (tonly && T != tonly && T > 2) continue;
            const double v = dp[r - T] + opt[T].cost + tune.launch_cost;
            if (v < dp[r]) {
                dp[r] = v;
                choice[r] = T;
            }
        }
    std::vector<PassPlan> plan;
    for (int r = L.iters; r > 0; r -= choice[r]) plan.push_back(opt[choice[r]]);
    // a context that shares the chip with concurrent fusions (pf_set_jacobi_share) keeps the
    // depths and engines chosen for the whole chip and re-chunks its streaming passes for its
    // share: fewer, longer row chunks
    if (c->jacobi_share < 1.0)
        for (PassPlan& pp : plan)
            if (pp.stages == 1)
                pp.nchunks = best_chunks(pp.T, C, band_rows, L.w, batch,
                                         jstream_waves_per_cu(C, pp.T, fast) / 4, plan_simds(c),
                                         tune.step_overhead, tune.lone_cycles, tune.c4_eff).nchunks;
    // tuning runs: PF_JN<w> forces the row chunking of the level of width w
    char key[32];
    snprintf(key, sizeof(key), "PF_JN%d", L.w);
    if (const char* e = getenv(key))
        for (PassPlan& pp : plan) pp.nchunks = atoi(e) > 0 ? atoi(e) : pp.nchunks;
    return plan;
}

// Runs L.iters sweeps.  The first pass reads `first` (SRC_SEED: emap, SRC_UPSAMPLE: prev level,
// SRC_BUF: buffer a); passes ping-pong between a and b.  With out != nullptr the last pass stores
// the u16 quantisation instead of floats.  Returns the buffer holding the result (unused when
// out is given).
// Largest sweep depth the streaming engine may use on this level: its halo rows must stay inside
// [1, h-2] (loads clamp rows into that range) and a strip (plus halo) must fit in a row.
static int jacobi_tcap(const LevelDims& L)
{
    static const JacobiTuning tune = jacobi_tuning();
    int cap = tune.Tmax;
    char key[32];  // tuning runs: PF_JT<w> caps the sweep depth of the level of width w
    snprintf(key, sizeof(key), "PF_JT%d", L.w);
    if (const char* e = getenv(key)) cap = atoi(e) > 0 ? atoi(e) : cap;
    if (L.h0 - 1 < cap) cap = L.h0 - 1;
    if (L.h - 2 - L.h1 < cap) cap = L.h - 2 - L.h1;
    while (cap >= 1) {
        int Tp = (cap + 3) / 4 * 4;
        if (128 - Tp <= L.w && L.w % 2 == 0) break;
        cap--;
    }
    return cap;
}

// SRC_SEED passes: ValueAtCoord's index (emap_index) split into its column term x * ec and row
// term y * ew * ec over the level's grid (the az / zen of grid_tables, then emap_index's fp64
// expression), cached per (level size, emap size).  Built by fuse_range before the level's
// timed Jacobi stage (the upload synchronises the stream); returns PF_OK or the upload's error.
static int seed_tables(pf_ctx* c, const LevelDims& L, int ew, int eh, int ec)
{
    const int key[5] = {L.w, L.h, ew, eh, ec};
    if (memcmp(key, c->seed_key, sizeof(key)) != 0) {
        std::vector<int> ecol(L.w + 2), erow(L.h + 2);
        for (int xx = -1; xx <= L.w; xx++) {
            const float az = (float)((double)((float)xx / (float)(L.w - 1) * 2.0f) * PF_MYPI);
            ecol[xx + 1] = (int)((double)az / (PF_MYPI * 2) * (double)(float)(ew - 1)) * ec;
        }
        for (int yy = -1; yy <= L.h; yy++) {
            const float zen = (float)((double)((float)yy / (float)(L.h - 1)) * PF_MYPI);
            erow[yy + 1] = (int)((double)zen / PF_MYPI * (double)(float)(eh - 1)) * ew * ec;
        }
        int rc;
        if ((rc = upload(c, c->seed_ecol, ecol)) || (rc = upload(c, c->seed_erow, erow))) return rc;
        memcpy(c->seed_key, key, sizeof(key));
    }
    return PF_OK;
}

// The resident level kernel (pf_jres.hip): one launch for all of a level's sweeps, for the
// widths it is built for (a wave holds whole rows) and levels with the packed-form certificate.
// nb row blocks per panorama of `core` rows; every K sweeps the blocks trade K halo rows.
struct JresPlan {
    bool on = false;
    int nb = 0, core = 0, K = 0, rounds = 0;
    bool half = false;  // half-height regions (jres_region_rows)
};

static JresPlan jres_plan(pf_ctx* c, const LevelDims& L, int batch, bool fast)
{
    JresPlan jp;
    static const char* env = getenv("PF_JRES");  // "0": streaming passes only (A/B runs)
    const int mode = c->jres_mode >= 0 ? c->jres_mode : (env && atoi(env) == 0 ? 0 : 1);
    if (mode == 0 || !fast || batch < 1) return jp;
    const int rows = jres_region_rows(L.w);  // region rows of one workgroup
    if (rows <= 0 || L.iters < 1) return jp;
    // resident blocks per CU at widths 256, 512, 1024, for the full and the half-height region
    static int bpc_w[3][2] = {{-1, -1}, {-1, -1}, {-1, -1}};
    const int wi = L.w == 256 ? 0 : (L.w == 512 ? 1 : 2);
    const int band = L.h1 - L.h0 + 1;
    // cost in sweep units: the blocks run in ceil(blocks / resident) rounds of residency, each
    // sweep costs one unit (fixed region size), each K-sweep hand-off ~2.5 units (measured
    // hand-off latency on MI355X is 2-3 us against ~1.2 us per sweep)
    static const double xcost = getenv("PF_JRES_X") ? atof(getenv("PF_JRES_X")) : 2.5;
    static const int nb_env = getenv("PF_JRES_NB") ? atoi(getenv("PF_JRES_NB")) : 0;
    const int nb_force = c->jres_nb > 0 ? c->jres_nb : nb_env;
    // a sweep of the half-height region costs each wave ~half the updates, plus the fixed
    // barrier / edge exchange (PF_JRES_HALFCOST: its cost in full-region sweeps)
    static const double hcost = getenv("PF_JRES_HALFCOST") ? atof(getenv("PF_JRES_HALFCOST")) : 0.6;
    double best = 1e300;
    for (int hv = 0; hv < 2; hv++) {
        const int rows_h = hv ? jres_region_rows(L.w, true) : rows;
        if (rows_h <= 0) continue;
        if (bpc_w[wi][hv] < 0) bpc_w[wi][hv] = jres_blocks_per_cu(L.w, hv == 1);
        const int bpc = bpc_w[wi][hv];  // of the instantiation this choice launches
        if (bpc < 1) continue;
        const double sweep = hv ? hcost : 1.0;
        for (int nb = 1; nb <= band && nb <= 64; nb++) {
            if (nb_force > 0 && nb != nb_force) continue;
            const int core = (band + nb - 1) / nb;
            if ((band + core - 1) / core != nb) continue;
            int K;
            if (nb == 1) {
                if (core > rows_h) continue;
                K = L.iters;
            } else {
                K = (rows_h - core) / 2;
                if (K > core) K = core;
                if (K > L.iters) K = L.iters;
                if (K < 1) continue;
            }
            const int rounds = (L.iters + K - 1) / K;
            const long long resident = (long long)c->num_cu * bpc;
            const long long waves = ((long long)batch * nb + resident - 1) / resident;
            // 1024 wide (one workgroup per CU, two waves per SIMD): only where every block of
            // the launch is resident at once -- the latency-bound one-panorama levels (C5); at
            // C3's batch its passes are not measured against the streaming engine's
            // (PF_JRES1024_ANY=1: allow)
            static const bool any1024 = getenv("PF_JRES1024_ANY") && atoi(getenv("PF_JRES1024_ANY"));
            if (L.w == 1024 && waves > 1 && !any1024) continue;
            const double cost = (double)waves * (L.iters * sweep + (rounds - 1) * xcost);
            if (cost < best) {
                best = cost;
                jp.on = true;
                jp.nb = nb;
                jp.core = core;
                jp.K = K;
                jp.rounds = rounds;
                jp.half = hv == 1;
            }
        }
    }
    return jp;
}

// The resident kernel's buffers (outside the timed stage: a first allocation synchronises).
static int jres_prepare(pf_ctx* c, const LevelDims& L, int batch, const JresPlan& jp)
{
    int rc;
    const size_t xb = sizeof(float) * jres_words_per_value() * (size_t)batch * jp.nb * 4 *
                      (size_t)jp.K * L.w;
    if ((rc = ensure(c, c->jres_x, xb))) return rc;
    const size_t sb = sizeof(uint32_t) * (2 + (size_t)batch * jp.nb * jres_flags_per_block(jp.K));
    if ((rc = ensure_err_host(c))) return rc;
    if (c->jres_sync.bytes < sb) {
        if ((rc = ensure(c, c->jres_sync, sb))) return rc;
        HIPCHK(c, hipMemsetAsync(c->jres_sync.p, 0, sb, c->stream));
        c->jres_tk = 0;
        c->jres_fb = 1;
    }
    return PF_OK;
}

static float* run_jacobi(pf_ctx* c, const LevelDims& L, int first, const float* emap, int ew,
                         int eh, int ec, long long estride, const GridCol* cols,
                         const GridRow* rows, const float* prev, long long pstride,
                         const float* lnorm, float* a, float* b, uint16_t* out,
                         long long ostride, int batch, int* npasses, const float* hcol,
                         const JresPlan* jp = nullptr)
{
    static const JacobiTuning tune = jacobi_tuning();
    if (jp && jp->on) {
        JresArgs A{};
        A.src_mode = first;
        if (first == 2) {
            const int key[5] = {L.w, L.h, ew, eh, ec};
            if (!emap || memcmp(key, c->seed_key, sizeof(key)) != 0) return nullptr;
            A.ecol = (const int*)c->seed_ecol.p;
            A.erow = (const int*)c->seed_erow.p;
        }
        const long long st = (long long)L.w * L.h;
        A.src = a; A.sstride = st;
        A.prev = prev; A.pstride = pstride;
        A.emap = emap; A.estride = estride;
        A.lnorm = lnorm; A.lstride = st;
        A.hcol = hcol;
        float* dst = first == 0 ? b : a;
        A.dst = dst; A.dstride = st;
        A.out = out; A.ostride = ostride;
        A.w = L.w; A.h = L.h; A.h0 = L.h0; A.h1 = L.h1; A.iters = L.iters; A.batch = batch;
        A.nb = jp->nb; A.core = jp->core; A.K = jp->K; A.half = jp->half ? 1 : 0;
        uint32_t* sync = (uint32_t*)c->jres_sync.p;
        A.xbuf = (float*)c->jres_x.p;
        A.ticket = sync;
        A.err = sync + 1;
        A.flags = sync + 2;
        A.err_host = c->jres_err_h;  // mapped + coherent: the device pointer is the host one
        static const int dbg = getenv("PF_JRES_DBG") ? atoi(getenv("PF_JRES_DBG")) : 0;
        A.dbg = dbg;
        A.spin_log2 = 24;
        if (c->jres_fault) {  // pf_debug_jres_fault: this launch only
            A.dbg |= 16;
            A.spin_log2 = c->jres_fault;
            c->jres_fault = 0;
        }
        A.tbase = c->jres_tk;
        A.fbase = c->jres_fb;
        c->jres_tk += (uint32_t)(batch * jp->nb);
        c->jres_fb += (uint32_t)(jp->rounds + 1);
        static const bool show = getenv("PF_JPLAN") != nullptr;
        if (show)
            fprintf(stderr, "jacobi plan %dx%d band %d iters %d batch %d resident: nb %d core %d K %d rounds %d\n",
                    L.w, L.h, L.h1 - L.h0 + 1, L.iters, batch, jp->nb, jp->core, jp->K, jp->rounds);
        launch_jres(c->stream, A);
        // the error word, stream-ordered into pinned memory: jres_check reports it
        if (npasses) *npasses = 1;
        return dst;
    }
    static const bool slow = getenv("PF_JSLOW") != nullptr;  // force the general (scalar) form
    const long long st = (long long)L.w * L.h;
    // packed form: the level's separable-coverage certificate (pf_jacobi.hip)
    const bool fast = hcol && !slow;
    // 4 columns per lane (packed form only): fewer DPP moves and pair assemblies per pixel and a
    // wider strip per halo; 2 keeps more waves resident.  The cost model picks per level.
    const bool c4ok = jstream_supported_C(4, fast) && L.w % 4 == 0 && L.w >= 512;
    // 3 columns per lane (packed form): a 192-column strip, so the 2T-column halo is a smaller
    // share than in the 128-column strips of C = 2 (L.w >= 192 + 2T: jacobi_tcap's bound)
    const bool c3ok = jstream_supported_C(3, fast) && L.w >= 256;
    int C = 2;
    std::vector<PassPlan> plan = plan_level(c, L, 2, jacobi_tcap(L), batch, fast);
    double cbest = 0;
    for (const PassPlan& pp : plan) cbest += pp.cost;
    for (int cc : {3, 4}) {
        if (!(cc == 3 ? c3ok : c4ok) || (tune.C != 0 && tune.C != cc)) continue;
        std::vector<PassPlan> pc = plan_level(c, L, cc, jacobi_tcap(L), batch, fast);
        double cost = 0;
        for (const PassPlan& pp : pc) cost += pp.cost;
        if (tune.C == cc || cost < cbest) {
            C = cc;
            cbest = cost;
            plan.swap(pc);
        }
    }
    JacobiPass P{};
    if (first == 2 && emap) {  // the tables seed_tables() built for this level and emap
        const int key[5] = {L.w, L.h, ew, eh, ec};
        if (memcmp(key, c->seed_key, sizeof(key)) != 0) return nullptr;
        P.ecol = (const int*)c->seed_ecol.p;
        P.erow = (const int*)c->seed_erow.p;
    }
    P.prev = prev; P.pstride = pstride;
    P.emap = emap; P.estride = estride; P.ew = ew; P.eh = eh; P.ec = ec;
    P.cols = cols; P.rows = rows;
    P.lnorm = lnorm; P.lstride = st;
    P.sstride = st; P.dstride = st;
    P.out = out; P.ostride = ostride;
    P.w = L.w; P.h = L.h; P.h0 = L.h0; P.h1 = L.h1;
    P.hcol = hcol;
    P.row_lo = L.h0;
    P.row_hi = L.h1 + 1;
    const int band_rows = L.h1 - L.h0 + 1;
    float* src = (first == 0) ? a : nullptr;
    float* dst = (first == 0) ? b : a;
    static const bool show = getenv("PF_JPLAN") != nullptr;
    if (show) {
        fprintf(stderr, "jacobi plan %dx%d band %d iters %d batch %d %s C%d:", L.w, L.h,
                band_rows, L.iters, batch, fast ? "packed" : "general", C);
        for (const PassPlan& pp : plan)
            fprintf(stderr, " T%d/n%d%s", pp.T, pp.nchunks, pp.stages > 1 ? "p" : "");
        fprintf(stderr, "\n");
    }
    int pass = 0;
    for (const PassPlan& pp : plan) {
        const int T = pp.T;
        P.Tp = strip_halo(T, C);
        P.V = 64 * C - 2 * P.Tp;
        P.nstrips = (L.w + P.V - 1) / P.V;
        P.rows_per_chunk = (band_rows + pp.nchunks - 1) / pp.nchunks;
        P.nchunks = (band_rows + P.rows_per_chunk - 1) / P.rows_per_chunk;
        P.src_mode = pass == 0 ? first : 0;
        P.src = src;
        P.dst = dst;
        P.out_mode = (pass + 1 == (int)plan.size() && out) ? 1 : 0;
        if (pp.stages > 1) launch_jpipe(c->stream, P, pp.stages, T / pp.stages, batch);
        else launch_jstream(c->stream, P, C, T, batch, fast);
        src = dst;
        dst = (dst == a) ? b : a;
        pass++;
    }
    if (npasses) *npasses = pass;
    return src;
}

// Side stream (lowest priority) and its fork/join events, created once per context.
static int ensure_aux(pf_ctx* c)
{
    if (c->aux) return PF_OK;
    int least = 0, greatest = 0;
    HIPCHK(c, hipDeviceGetStreamPriorityRange(&least, &greatest));
    const char* pr = getenv("PF_AUXPRIO");  // A/B runs: "high" | "default" (else lowest)
    const int prio = pr && !strcmp(pr, "high") ? greatest : (pr && !strcmp(pr, "default") ? 0 : least);
    HIPCHK(c, hipStreamCreateWithPriority(&c->aux, hipStreamNonBlocking, prio));
    HIPCHK(c, hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
    for (hipEvent_t& e : c->ev_tgt) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return PF_OK;
}

// Floats of the per-level target planes of one panorama (fuse_range's lnorm workspace).
static long long target_planes(const LevelCache& lc)
{
    long long n = 0;
    for (int l = 0; l < lc.nlevels; l++) n += (long long)lc.dims[l].w * lc.dims[l].h;
    return n;
}

// The fusion levels of panoramas [0, batch) of the given pointers, on c->stream.  ws are the
// level-buffer bases (pano b of a level with stride st at base + b*st); lnorm_ws holds one target
// plane per level (level l at lnorm_ws + batch * sum_{k<l} st_k), target_planes() * batch floats.
//
// The target planes depend only on the tiles and the coefficients, not on any Jacobi result, so
// the finer levels' planes are gathered on a low-priority side stream while the coarse levels
// sweep: the level-0 and level-1 passes fill ~2 waves per SIMD (a 512- or 1024-wide band per
// panorama), leaving room for the gathers.  With the stage timers on, everything stays on
// c->stream so that every stage's time is its own.
static int fuse_range(pf_ctx* c, const float* emap, int ew, int eh, int ec, const float* tiles,
                      const float* coeffs, int batch, int out_w, int out_h, uint16_t* out,
                      float* const ws[3], float* lnorm_ws)
{
    const long long plane = (long long)out_w * out_h;
    const long long estride = (long long)ew * eh * ec;
    float* bufs[3] = {ws[0], ws[1], ws[2]};
    float* prev = nullptr;
    LevelCache& lc = c->lc;
    static const bool naive = getenv("PF_JACOBI") && strcmp(getenv("PF_JACOBI"), "naive") == 0;
    static const bool noside = getenv("PF_NOSIDE") != nullptr;  // A/B runs
    float* lnl[4] = {};
    {
        long long off = 0;
        for (int l = 0; l < lc.nlevels; l++) {
            lnl[l] = lnorm_ws + off;
            off += (long long)lc.dims[l].w * lc.dims[l].h * batch;
        }
    }
    auto targets = [&](int l, hipStream_t s) {
        const LevelDims& L = lc.dims[l];
        const long long st = (long long)L.w * L.h;
        const GridCol* cols = (const GridCol*)lc.cols[l].p;
        const GridRow* rows = (const GridRow*)lc.rows[l].p;
        // PF_TARGETS=direct|map selects the older per-pixel gathers (A/B tuning runs)
        static const char* tsel = getenv("PF_TARGETS");
        static const bool direct = tsel && strcmp(tsel, "direct") == 0;
        static const bool permap = tsel && strcmp(tsel, "map") == 0;
        if (direct)
            launch_targets(s, (const TileGeom*)c->geom.p, (const TileBox*)lc.box[l].p, 0,
                           c->ntiles, cols, rows, tiles, c->tile_elems, coeffs, c->ntiles, L,
                           lnl[l], st, batch);
        else if (!permap)
            launch_targets_patch(s, (const TileGeom*)c->geom.p, (const TileBox*)lc.box[l].p,
                                 (const TapBox*)lc.tapbox[l].p, c->ntiles,
                                 (const int32_t*)lc.tapmap[l].p, tiles, c->tile_elems, coeffs, L,
                                 lnl[l], st, batch);
        else
            launch_targets_map(s, (const TileGeom*)c->geom.p, (const TileBox*)lc.box[l].p,
                               (const TapBox*)lc.tapbox[l].p, c->ntiles,
                               (const int32_t*)lc.tapmap[l].p, tiles, c->tile_elems, coeffs, L,
                               lnl[l], st, batch);
    };
    // PF_TGT_MULTI=0: the per-level target launches (levels 1+ on the side stream) -- A/B runs
    static const bool multi = !(getenv("PF_TGT_MULTI") && atoi(getenv("PF_TGT_MULTI")) == 0) &&
                              !naive && !(getenv("PF_TARGETS"));
    if (multi) {
        TgtMulti M{};
        M.nlev = lc.nlevels;
        M.nentries = lc.tgt_nentries;
        const int pw_ = targets_patch_w(), ph_ = targets_patch_h();
        double bytes = 0;
        for (int l = 0; l < lc.nlevels; l++) {
            const LevelDims& L = lc.dims[l];
            TgtLevel& T = M.lv[l];
            T.tmask = (const uint32_t*)lc.tmask[l].p;
            T.nmw = (c->ntiles + 31) / 32;
            T.L = L;
            T.box = (const TileBox*)lc.box[l].p;
            T.tb = (const TapBox*)lc.tapbox[l].p;
            T.map = (const int32_t*)lc.tapmap[l].p;
            T.lnorm = lnl[l];
            T.lstride = (long long)L.w * L.h;
            T.npx = (L.w + pw_ - 1) / pw_;
            T.npy = (L.h1 - L.h0 + 1 + ph_ - 1) / ph_;
            bytes += (double)batch * (4.0 * L.w * (L.h1 - L.h0 + 1) + 4.0 * (double)lc.taps[l]);
        }
        StageTimer t(c, PF_STAGE_TARGETS, bytes, 1);
        launch_targets_multi(c->stream, (const TileGeom*)c->geom.p, c->ntiles, tiles,
                             c->tile_elems, coeffs, M, (const int2*)lc.tgt_order.p, batch);
    }
    const bool side = !multi && !c->prof_on && !noside && lc.nlevels > 1;
    if (side) {
        int rc;
        if ((rc = ensure_aux(c))) return rc;
        // the side stream starts after everything queued so far on c->stream (tiles, coeffs,
        // and the previous call's reads of these planes)
        HIPCHK(c, hipEventRecord(c->ev_fork, c->stream));
        HIPCHK(c, hipStreamWaitEvent(c->aux, c->ev_fork, 0));
        for (int l = 1; l < lc.nlevels; l++) {
            targets(l, c->aux);
            HIPCHK(c, hipEventRecord(c->ev_tgt[l], c->aux));
        }
    }
    for (int l = 0; l < lc.nlevels; l++) {
        const LevelDims& L = lc.dims[l];
        const long long st = (long long)L.w * L.h;
        const bool last = l == lc.nlevels - 1;
        const long long pst = l > 0 ? (long long)lc.dims[l - 1].w * lc.dims[l - 1].h : 0;
        float* a = nullptr;
        float* b = nullptr;
        for (int k = 0; k < 3; k++) {
            if (bufs[k] == prev) continue;
            if (!a) a = bufs[k];
            else if (!b) b = bufs[k];
        }
        const double B = (double)batch;
        const double band = (double)L.w * (L.h1 - L.h0 + 1);
        const GridCol* cols = (const GridCol*)lc.cols[l].p;
        const GridRow* rows = (const GridRow*)lc.rows[l].p;
        float* const lnorm_l = lnl[l];
        if (multi) {
            // gathered above, for every level
        } else if (side && l > 0) {
            HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_tgt[l], 0));
        } else {
            // algorithmic bytes: one 4-B tile texel per tap-grid point (k_targets_patch gathers
            // each once; coarse levels touch a fraction of the tiles) + the 4-B L plane write
            StageTimer t(c, PF_STAGE_TARGETS, B * (4.0 * band + 4.0 * (double)lc.taps[l]), 1);
            targets(l, c->stream);
        }
        float* res = nullptr;
        if (naive || jacobi_tcap(L) < 1) {
            {
                double srcb = l == 0 ? band * 4.0 : (double)st;
                StageTimer t(c, PF_STAGE_SEED, B * (4.0 * st + srcb), 1);
                if (l == 0)
                    launch_seed0(c->stream, emap, ew, eh, ec, estride, cols, rows, L, a, st, batch);
                else
                    launch_upsample(c->stream, prev, pst, L, a, st, batch);
            }
            HIPCHK(c, hipMemcpyAsync(b, a, sizeof(float) * st * batch, hipMemcpyDeviceToDevice,
                                     c->stream));
            {
                StageTimer t(c, PF_STAGE_JACOBI, B * 12.0 * band * L.iters, L.iters);
                launch_jacobi(c->stream, a, b, (const float*)lnorm_l, st, L, L.iters, batch,
                              &res);
            }
            if (last) {
                StageTimer t(c, PF_STAGE_QUANTIZE, B * 6.0 * st, 1);
                launch_quantize(c->stream, res, st, (int)st, out, plane, batch);
            }
        } else {
            {
                // out-of-band rows: zero / upsampled copy (u16 on the last level)
                double nb = (double)st - band;
                StageTimer t(c, PF_STAGE_SEED, B * nb * (last ? 3.0 : 9.0), 1);
                launch_border(c->stream, l == 0 ? nullptr : prev, pst, L, a, b, st,
                              last ? out : nullptr, plane, batch);
            }
            if (l == 0) {  // outside the timed stage: the first call per emap size uploads
                int rc;
                if ((rc = seed_tables(c, L, ew, eh, ec))) return rc;
            }
            const JresPlan jp = jres_plan(c, L, batch, lc.full[l]);
            if (jp.on) {  // outside the timed stage too (first allocation synchronises)
                int rc;
                if ((rc = jres_prepare(c, L, batch, jp))) return rc;
            }
            {
                // 12 B per pixel-update (read b, read L, write b'), SURVEY.md 8d
                StageTimer t(c, PF_STAGE_JACOBI, B * 12.0 * band * L.iters, L.iters);
                int passes = 0;
                res = run_jacobi(c, L, l == 0 ? 2 : 1, emap, ew, eh, ec, estride, cols, rows,
                                 prev, pst, (const float*)lnorm_l, a, b, last ? out : nullptr,
                                 plane, batch, &passes,
                                 lc.full[l] ? (const float*)lc.hcol[l].p : nullptr, &jp);
                t.set_launches(passes);  // k_jlag launches (rocprof's count for that kernel)
            }
            if (!res) return fail(c, PF_EINVAL, "level-0 seed tables missing");
        }
        prev = res;
        if (!c->ev_level[l]) HIPCHK(c, hipEventCreateWithFlags(&c->ev_level[l], hipEventDisableTiming));
        HIPCHK(c, hipEventRecord(c->ev_level[l], c->stream));
    }
    c->nlev_recorded = lc.nlevels;
    HIPCHK(c, hipGetLastError());
    return PF_OK;
}

// SolveDepthAll for a batch, on c->stream.  (Running the batch as two staggered halves on two
// streams, so that one half's coarse levels overlap the other's fine levels, was measured slower:
// 10.4-10.6k vs 11.6k panoramas/s at batch 64 -- the half-size passes lose more than the
// overlap wins.)
static int fuse_impl(pf_ctx* c, const float* emap, int ew, int eh, int ec, const float* tiles,
                     const float* coeffs, int batch, int out_w, int out_h, float zr0,
                     float zr1, uint16_t* out)
{
    int rc;
    if ((rc = prepare_levels(c, out_w, out_h, zr0, zr1))) return rc;
    const long long plane = (long long)out_w * out_h;
    for (int k = 0; k < 3; k++)
        if ((rc = ensure(c, c->buf[k], sizeof(float) * plane * batch))) return rc;
    if ((rc = ensure(c, c->lnorm, sizeof(float) * target_planes(c->lc) * batch))) return rc;
    float* ws[3] = {(float*)c->buf[0].p, (float*)c->buf[1].p, (float*)c->buf[2].p};
    return fuse_range(c, emap, ew, eh, ec, tiles, coeffs, batch, out_w, out_h, out, ws,
                      (float*)c->lnorm.p);
}

// Once per (layout, panorama size): order the warp patches by panorama footprint -- 32-row bands
// of the box centre, then its azimuth -- instead of tile by tile.  The blocks resident on one XCD
// then stage overlapping boxes (neighbouring patches of a tile and the overlapping patches of the
// neighbouring tiles) at about the same time, so a panorama line is fetched from HBM once and
// re-read from that XCD's L2 instead of once per box that holds it (the boxes hold each panorama
// pixel ~3 times at the C2 layout).  Patches are self-describing, so the permutation is free.
static int sort_warp_patches(pf_ctx* c, int pw)
{
    std::vector<WarpPatch> p(c->npatch);
    HIPCHK(c, hipMemcpyAsync(p.data(), c->wpatch.p, sizeof(WarpPatch) * p.size(),
                             hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    auto key = [pw](const WarpPatch& w) {
        const long long band = (w.gy0 + w.bh / 2) / 32;
        const long long col = (w.gx0 + w.bw / 2) % pw;
        return band * 65536 + col;
    };
    std::stable_sort(p.begin(), p.end(),
                     [&](const WarpPatch& a, const WarpPatch& b) { return key(a) < key(b); });
    return upload(c, c->wpatch, p);
}

extern "C" {

int pf_register(pf_ctx* c, const float* emap, int ew, int eh, int ec, float* tiles, int batch,
                float zr0, float zr1, int degree, int apply, float* coeffs, double* coeffs64)
{
    int rc;
    if ((rc = check_common(c, batch))) return rc;
    if ((rc = check_emap(c, emap, ew, eh, ec))) return rc;
    if (!tiles) return fail(c, PF_EINVAL, "tiles is NULL");
    if (degree < 0 || degree > 3) return fail(c, PF_EINVAL, "degree %d not in [0,3]", degree);
    if ((rc = prepare_registration(c, zr0, zr1))) return rc;
    if ((rc = check_reg_grids(c, nullptr))) return rc;
    float* cf = coeffs;
    if (!cf) {
        if ((rc = ensure(c, c->coeffs, sizeof(float) * 4 * c->ntiles * batch))) return rc;
        cf = (float*)c->coeffs.p;
    }
    double nsamp = 0;
    for (const RegGrid& g : c->reg_h) nsamp += (double)(g.cols + 1) * (g.rows + 1);
    const int2* sidx = reg_sample_index(c, ew, eh, ec);  // before the stage timer: built once
    {
        StageTimer t(c, PF_STAGE_REGISTER,
                     batch * (8.0 * nsamp + (apply ? 8.0 * (double)c->tile_elems / c->tile_c : 0.0)),
                     apply ? 2 : 1);
        launch_register(c->stream, (const TileGeom*)c->geom.p, (const RegGrid*)c->reg.p,
                        (const GridCol*)c->rcols.p, (const GridRow*)c->rrows.p, c->ntiles, emap,
                        ew, eh, ec, (long long)ew * eh * ec, tiles, c->tile_elems, degree,
                        c->solver, cf, coeffs64, batch, nullptr, nullptr, sidx);
        if (apply)
            launch_apply_cubic(c->stream, (const TileGeom*)c->geom.p, c->ntiles,
                               c->tile_elems / c->tile_c, tiles, c->tile_elems, cf, batch);
    }
    HIPCHK(c, hipGetLastError());
    return PF_OK;
}

int pf_fuse(pf_ctx* c, const float* emap, int ew, int eh, int ec, const float* tiles,
            const float* coeffs, int batch, int out_w, int out_h, float zr0, float zr1,
            uint16_t* out)
{
    int rc;
    if ((rc = check_common(c, batch))) return rc;
    if ((rc = check_emap(c, emap, ew, eh, ec))) return rc;
    if (!tiles || !out) return fail(c, PF_EINVAL, "tiles/out is NULL");
    if ((rc = jres_check(c))) return rc;  // an earlier fusion's timeout, once it has landed
    return fuse_impl(c, emap, ew, eh, ec, tiles, coeffs, batch, out_w, out_h, zr0, zr1, out);
}

int pf_merge(pf_ctx* c, const float* emap, int ew, int eh, int ec, const float* tiles, int batch,
             int out_w, float zr0, float zr1, float* coeffs, uint16_t* out)
{
    int rc;
    if ((rc = check_common(c, batch))) return rc;
    if ((rc = check_emap(c, emap, ew, eh, ec))) return rc;
    if (!tiles || !out) return fail(c, PF_EINVAL, "tiles/out is NULL");
    if ((rc = jres_check(c))) return rc;  // an earlier fusion's timeout, once it has landed
    float* cf = coeffs;
    if (!cf) {
        if ((rc = ensure(c, c->coeffs, sizeof(float) * 4 * c->ntiles * batch))) return rc;
        cf = (float*)c->coeffs.p;
    }
    if ((rc = pf_register(c, emap, ew, eh, ec, const_cast<float*>(tiles), batch, zr0, zr1, 3, 0,
                          cf, nullptr)))
        return rc;
    return fuse_impl(c, emap, ew, eh, ec, tiles, cf, batch, out_w, out_w / 2, zr0, zr1, out);
}

int pf_solve_smoothing(pf_ctx* c, const float* tiles, const float* coeffs, int batch, int out_w,
                       int out_h, float zr0, float zr1, uint16_t* out)
{  // SolveDepthBySmoothing (Depth.cpp:1773-1878)
    int rc;
    if ((rc = check_common(c, batch))) return rc;
    if ((rc = jres_check(c))) return rc;  // an earlier call's timeout, once it has landed
    if (!tiles || !out) return fail(c, PF_EINVAL, "tiles/out is NULL");
    if (out_w < 3 || out_h < 3 || (long long)out_w * out_h >= (1LL << 31))
        return fail(c, PF_EINVAL, "output %dx%d out of range", out_w, out_h);
    LevelDims L{};
    L.w = out_w;
    L.h = out_h;
    L.h0 = (int)floor((double)((float)out_h * zr0) / PF_MYPI);  // height0/height1 (:1781-1782)
    L.h1 = (int)ceil((double)((float)out_h * zr1) / PF_MYPI);
    if (L.h0 < 1 || L.h1 > out_h - 2 || L.h0 > L.h1)
        return fail(c, PF_EINVAL, "rows [%d, %d] of %d: the smoothing stencil would leave the "
                    "buffer (the reference reads out of bounds)", L.h0, L.h1, out_h);
    std::vector<SmoothBox> boxes(c->ntiles);
    for (int p = 0; p < c->ntiles; p++) {  // :1795-1805, no clamps
        const pf_window& r = c->rng[p];
        SmoothBox b{};
        b.x0 = (int)round((double)r.az_left / (2 * PF_MYPI) * (double)(out_w - 1));
        b.x1 = (int)round((double)r.az_right / (2 * PF_MYPI) * (double)(out_w - 1));
        b.y0 = (int)round((double)r.zen_top / PF_MYPI * (double)(out_h - 1));
        b.y1 = (int)round((double)r.zen_down / PF_MYPI * (double)(out_h - 1));
        b.xs = b.x1 >= b.x0 ? 1 : -1;
        if (b.x0 == b.x1)
            return fail(c, PF_EDEGENERATE, "tile %d: box x0 == x1 == %d (the reference never "
                        "terminates here)", p, b.x0);
        if (b.x0 < 0 || b.x0 >= out_w || b.x1 < 0 || b.x1 >= out_w || b.y0 < 0 || b.y1 >= out_h)
            return fail(c, PF_EINVAL, "tile %d: box (%d..%d, %d..%d) leaves the %dx%d output (the "
                        "reference writes out of bounds)", p, b.x0, b.x1, b.y0, b.y1, out_w, out_h);
        boxes[p] = b;
    }
    std::vector<GridCol> cols;
    std::vector<GridRow> rows;
    grid_tables(L, cols, rows);
    const long long n = (long long)out_w * out_h;
    if ((rc = upload(c, c->sm_box, boxes))) return rc;
    if ((rc = upload(c, c->sm_cols, cols))) return rc;
    if ((rc = upload(c, c->sm_rows, rows))) return rc;
    if ((rc = ensure(c, c->sm_src, sizeof(int2) * n))) return rc;
    if ((rc = ensure(c, c->sm_mask, n))) return rc;
    if ((rc = ensure(c, c->buf[0], sizeof(float) * n * batch))) return rc;
    launch_smooth_map(c->stream, (const TileGeom*)c->geom.p, (const SmoothBox*)c->sm_box.p,
                      c->ntiles, (const GridCol*)c->sm_cols.p, (const GridRow*)c->sm_rows.p,
                      out_w, out_h, (int2*)c->sm_src.p, (uint8_t*)c->sm_mask.p);
    const int iters = 500;  // :1838
    static const bool scan = getenv("PF_SMOOTH_SCAN") && atoi(getenv("PF_SMOOTH_SCAN"));
    if (scan) {  // every (X, Y) of the diagonal tested against the mask (the first form)
        launch_smooth(c->stream, (const TileGeom*)c->geom.p, c->ntiles, (const int2*)c->sm_src.p,
                      (const uint8_t*)c->sm_mask.p, tiles, c->tile_elems, coeffs, out_w, out_h,
                      L.h0, L.h1, iters, (float*)c->buf[0].p, batch);
    } else {
        // row blocks per panorama (k_smooth_band): a panorama's steps spread over nb CUs;
        // PF_SMOOTH_BAND=0 keeps one workgroup per panorama (k_smooth_iter_list, nb = 1)
        const char* be = getenv("PF_SMOOTH_BAND");  // read per call (tests vary it)
        const int band_mode = be ? atoi(be) : 1;
        int nb = 1;
        if (band_mode != 0) {
            nb = band_mode > 1 ? band_mode : std::max(1, std::min(64, 1024 / batch));
            nb = std::max(1, std::min(nb, (L.h1 - L.h0 + 1) / 4));
        }
        const bool same = c->sm_key_boxes.size() == boxes.size() && c->sm_key[0] == out_w &&
                          c->sm_key[1] == out_h && c->sm_key[2] == L.h0 && c->sm_key[3] == L.h1 &&
                          c->sm_nb == nb &&
                          std::equal(boxes.begin(), boxes.end(), c->sm_key_boxes.begin(),
                                     [](const SmoothBox& a, const SmoothBox& b) {
                                         return a.x0 == b.x0 && a.x1 == b.x1 && a.y0 == b.y0 &&
                                                a.y1 == b.y1 && a.xs == b.xs;
                                     });
        if (!same) {  // per row block, the masked pixels by parity of d = X + Y, sorted by d
            std::vector<uint8_t> mask(n);
            HIPCHK(c, hipMemcpyAsync(mask.data(), c->sm_mask.p, n, hipMemcpyDeviceToHost,
                                     c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
            const int nk = (out_w + out_h) / 2 + 1;  // d = 2k + p < w + h
            // row blocks of about equal masked-pixel counts
            std::vector<long long> rowcnt(out_h, 0);
            long long total = 0;
            for (int Y = L.h0; Y <= L.h1; Y++) {
                for (int X = 1; X <= out_w - 2; X++) rowcnt[Y] += mask[(long long)Y * out_w + X];
                total += rowcnt[Y];
            }
            std::vector<int> blk_of(out_h, 0);
            {
                long long acc = 0;
                int b = 0, rows_in = 0;
                for (int Y = L.h0; Y <= L.h1; Y++) {
                    const int rows_left = L.h1 - Y + 1;
                    if (b < nb - 1 && rows_in > 0 &&
                        (acc >= total * (b + 1) / nb || rows_left <= nb - 1 - b)) {
                        b++;
                        rows_in = 0;
                    }
                    blk_of[Y] = b;
                    acc += rowcnt[Y];
                    rows_in++;
                }
            }
            const size_t per = (size_t)(nk + 1);
            std::vector<int> cnt((size_t)nb * 2 * per, 0);
            int dmin = INT32_MAX, dmax = -1;
            for (int Y = L.h0; Y <= L.h1; Y++)
                for (int X = 1; X <= out_w - 2; X++)
                    if (mask[(long long)Y * out_w + X]) {
                        const int d = X + Y;
                        cnt[((size_t)blk_of[Y] * 2 + (d & 1)) * per + (d >> 1) + 1]++;
                        dmin = std::min(dmin, d);
                        dmax = std::max(dmax, d);
                    }
            std::vector<int> off(cnt.size());
            int acc = 0;
            for (size_t q = 0; q < (size_t)nb * 2; q++)
                for (size_t k = 0; k < per; k++) {
                    acc += cnt[q * per + k];
                    off[q * per + k] = acc;  // k = 0 holds the zero count: start of d = p
                }
            std::vector<int> fill(off), list(std::max(acc, 1));
            for (int Y = L.h0; Y <= L.h1; Y++)
                for (int X = 1; X <= out_w - 2; X++)
                    if (mask[(long long)Y * out_w + X]) {
                        const int d = X + Y;
                        list[fill[((size_t)blk_of[Y] * 2 + (d & 1)) * per + (d >> 1)]++] =
                            Y * out_w + X;
                    }
            if ((rc = upload(c, c->sm_list, list))) return rc;
            if ((rc = upload(c, c->sm_off, off))) return rc;
            c->sm_nk = nk;
            c->sm_nb = nb;
            c->sm_smin = dmin;
            c->sm_smax = dmax < 0 ? -1 : dmax + 2 * (iters - 1);
            c->sm_key_boxes = boxes;
            c->sm_key[0] = out_w; c->sm_key[1] = out_h; c->sm_key[2] = L.h0; c->sm_key[3] = L.h1;
        }
        launch_smooth_seed(c->stream, (const TileGeom*)c->geom.p, c->ntiles,
                           (const int2*)c->sm_src.p, tiles, c->tile_elems, coeffs, out_w, out_h,
                           (float*)c->buf[0].p, batch);
        if (c->sm_smax >= c->sm_smin) {
            if (nb == 1) {
                launch_smooth_list(c->stream, (const int*)c->sm_list.p, (const int*)c->sm_off.p,
                                   c->sm_nk, out_w, out_h, c->sm_smin, c->sm_smax, iters,
                                   (float*)c->buf[0].p, batch);
            } else {
                // sync words: [0] ticket, [1] timeouts, [2..] one step flag per (panorama, block);
                // tickets and flags are monotone across launches (sm_tk, sm_fb)
                const size_t sb = sizeof(uint32_t) * (2 + (size_t)batch * nb);
                if (c->sm_sync.bytes < sb) {
                    if ((rc = ensure(c, c->sm_sync, sb))) return rc;
                    HIPCHK(c, hipMemsetAsync(c->sm_sync.p, 0, sb, c->stream));
                    c->sm_tk = 0;
                    c->sm_fb = 1;
                }
                if ((rc = ensure_err_host(c))) return rc;
                SmoothSync S{};
                uint32_t* w32 = (uint32_t*)c->sm_sync.p;
                S.ticket = w32;
                S.err = w32 + 1;
                S.flags = w32 + 2;
                S.err_host = c->jres_err_h;
                S.tbase = c->sm_tk;
                S.fbase = c->sm_fb;
                S.spin_log2 = 22;
                if (c->smooth_fault) {  // pf_debug_smooth_fault: this launch only
                    S.fault = 1;
                    S.spin_log2 = c->smooth_fault;
                    c->smooth_fault = 0;
                }
                c->sm_tk += (uint32_t)(batch * nb);
                c->sm_fb += (uint32_t)(c->sm_smax - c->sm_smin + 2);
                launch_smooth_band(c->stream, (const int*)c->sm_list.p, (const int*)c->sm_off.p,
                                   c->sm_nk, nb, out_w, out_h, c->sm_smin, c->sm_smax, iters,
                                   (float*)c->buf[0].p, batch, S);
            }
        }
    }
    launch_quantize(c->stream, (const float*)c->buf[0].p, n, (int)n, out, n, batch);
    HIPCHK(c, hipGetLastError());
    return PF_OK;
}

int pf_warp_depth(pf_ctx* c, const float* pano, int pw, int ph, int batch,
                  const pf_response* resp, float* tiles)
{
    int rc;
    if ((rc = check_common(c, batch))) return rc;
    if (!pano || !tiles || pw < 2 || ph < 2)
        return fail(c, PF_EINVAL, "bad pano %p %dx%d", (const void*)pano, pw, ph);
    static_assert(sizeof(pf_response) == sizeof(Resp), "pf_response layout");
    if ((long long)pw * ph >= (1ll << 30) || pw >= 65536 || ph >= 65536)
        return fail(c, PF_EINVAL, "pano %dx%d: too large (< 2^30 pixels, sides < 65536)", pw, ph);
    if (c->tile_elems >= (1ll << 29))  // the warp addresses a panorama's tile block with 32-bit
        return fail(c, PF_EINVAL, "tile block of %lld floats: too large for the depth warp "
                    "(< 2^29)", c->tile_elems);      // byte offsets (buffer stores)
    const long long npix = c->tile_elems / c->tile_c;
    if (c->wmap_pw != pw || c->wmap_ph != ph) {
        if ((rc = ensure(c, c->wmap, sizeof(uint32_t) * npix))) return rc;
        if ((rc = ensure(c, c->wfxy, sizeof(float) * 2 * npix))) return rc;
        // corners and weights on the host (glibc atan2f: the reference's bits).  Tiles are
        // built into one host staging run of up to kStagePix pixels (C3's whole layout; C5 in
        // 6 runs), uploaded with one copy per array and one synchronisation per run.  This first
        // call per panorama size blocks the host (the staging memory is reused).
        const size_t kStagePix = (size_t)1 << 24;
        const size_t cap = std::max((size_t)c->npix_max, std::min((size_t)npix, kStagePix));
        std::vector<uint32_t> wxy(cap), loc;
        std::vector<float> wf(2 * cap);
        // ragged footprints (host, warp_patches_host) unless PF_WARP_RAGGED=0 or pw % 4 != 0;
        // else the bounding boxes of k_patch_box / k_warp_local
        const char* rg = getenv("PF_WARP_RAGGED");
        const bool ragged = (pw % 4) == 0 && !(rg && atoi(rg) == 0);
        std::vector<WarpPatch> patches;
        std::vector<uint32_t> units;
        if (ragged) loc.resize(cap);
        for (int p0 = 0; p0 < c->ntiles;) {
            const size_t off0 = (size_t)c->geom_h[p0].pix_off;
            size_t n = 0;
            int p1 = p0;
            for (; p1 < c->ntiles; p1++) {
                const TileGeom& g = c->geom_h[p1];
                const size_t m = (size_t)g.w * g.h;
                if (p1 > p0 && n + m > cap) break;
                warp_coords_host(g, pw, ph, wxy.data() + n, wf.data() + 2 * n);
                if (ragged)
                    warp_patches_host(g, p1, wxy.data() + n, pw, ph, patches, units,
                                      loc.data() + n);
                n += m;
            }
            HIPCHK(c, hipMemcpyAsync((uint32_t*)c->wmap.p + off0, ragged ? loc.data() : wxy.data(),
                                     4 * n, hipMemcpyHostToDevice, c->stream));
            HIPCHK(c, hipMemcpyAsync((float*)c->wfxy.p + 2 * off0, wf.data(), 8 * n,
                                     hipMemcpyHostToDevice, c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));  // the staging run is reused
            p0 = p1;
        }
        if (ragged) {
            // footprint order, as sort_warp_patches: 32-row bands of the first staged unit, then
            // its column (a wide patch: its first corner)
            std::vector<long long> keys(patches.size());
            for (size_t q = 0; q < patches.size(); q++) {
                const WarpPatch& P = patches[q];
                long long row, col;
                if (P.units > 0) {
                    const uint32_t e = units[P.uoff] / 4u;
                    row = e / (uint32_t)pw;
                    col = e % (uint32_t)pw;
                } else {
                    const TileGeom& g = c->geom_h[P.tile];
                    row = 0;
                    col = P.X0 + (long long)g.w * P.Y0;  // keep tile order among wide patches
                }
                keys[q] = (row / 32) * (1LL << 40) + col;
            }
            std::vector<size_t> ord(patches.size());
            for (size_t q = 0; q < ord.size(); q++) ord[q] = q;
            std::stable_sort(ord.begin(), ord.end(),
                             [&](size_t a, size_t b) { return keys[a] < keys[b]; });
            std::vector<WarpPatch> sp(patches.size());
            for (size_t q = 0; q < ord.size(); q++) sp[q] = patches[ord[q]];
            if (units.empty()) units.push_back(0u);
            if ((rc = upload(c, c->wpatch, sp))) return rc;
            if ((rc = upload(c, c->wunits, units))) return rc;
            c->npatch = (int)sp.size();
        } else {
            // the plain patch grid (a ragged build for another size replaced it)
            if ((rc = upload(c, c->wpatch, c->wpatch_grid_h))) return rc;
            c->npatch = (int)c->wpatch_grid_h.size();
            launch_warp_boxes(c->stream, (const TileGeom*)c->geom.p, (WarpPatch*)c->wpatch.p,
                              c->npatch, pw, ph, (uint32_t*)c->wmap.p);
            HIPCHK(c, hipGetLastError());
            if ((rc = sort_warp_patches(c, pw))) return rc;
        }
        c->wmap_pw = pw;
        c->wmap_ph = ph;
    }
    StageTimer t(c, PF_STAGE_WARP, batch * (4.0 * pw * ph + 4.0 * (double)npix), 1);
    launch_warp_depth(c->stream, (const TileGeom*)c->geom.p, c->ntiles,
                      (const WarpPatch*)c->wpatch.p, (const uint32_t*)c->wunits.p, c->npatch,
                      (const uint32_t*)c->wmap.p,
                      (const float*)c->wfxy.p, pano, pw, ph, (long long)pw * ph,
                      (const Resp*)resp, tiles, c->tile_elems, batch);
    HIPCHK(c, hipGetLastError());
    return PF_OK;
}

int pf_warp_rgb(pf_ctx* c, const uint8_t* pano, int pw, int ph, int batch, uint8_t* tiles)
{
    int rc;
    if ((rc = check_common(c, batch))) return rc;
    if (!pano || !tiles || pw < 2 || ph < 2)
        return fail(c, PF_EINVAL, "bad pano %p %dx%d", (const void*)pano, pw, ph);
    if (pw >= 65536 || ph >= 65536)
        return fail(c, PF_EINVAL, "pano %dx%d: sides must be < 65536", pw, ph);
    if (c->rgb_pw != pw || c->rgb_ph != ph) {  // the taps of this size, on the host (glibc)
        const long long npix = c->tile_elems / c->tile_c;
        if ((rc = ensure(c, c->rgbtap, sizeof(RgbTap) * npix))) return rc;
        // the LDS-staged kernel needs 16-B units that never straddle the row wrap, 12-B
        // stores of 4 whole pixels, and 32-bit byte offsets (else the per-pixel kernel runs)
        const bool naive = getenv("PF_WARP_RGB_NAIVE") && atoi(getenv("PF_WARP_RGB_NAIVE"));
        bool staged = !naive && (3 * pw) % 16 == 0 && 3LL * pw * ph < (1LL << 31) &&
                      c->rgb_elems < (1LL << 31);
        for (int p = 0; staged && p < c->ntiles; p++) staged = c->geom_h[p].w % 4 == 0;
        if (staged) {
            if ((rc = ensure(c, c->rgbloc, sizeof(uint32_t) * npix))) return rc;
            if ((rc = ensure(c, c->rgbw, sizeof(float) * 2 * npix))) return rc;
        }
        // staged as the depth warp's corner tables: runs of up to 2^24 pixels, one copy and
        // one synchronisation per run (this first call per panorama size blocks the host)
        const size_t kStagePix = (size_t)1 << 24;
        const size_t cap = std::max((size_t)c->npix_max, std::min((size_t)npix, kStagePix));
        std::vector<RgbTap> taps(cap);
        std::vector<uint32_t> loc(staged ? cap : 0);
        std::vector<float> wts(staged ? 2 * cap : 0);
        std::vector<RgbPatch> patches;
        std::vector<uint32_t> units;
        for (int p0 = 0; p0 < c->ntiles;) {
            const size_t off0 = (size_t)c->geom_h[p0].pix_off;
            size_t n = 0;
            int p1 = p0;
            for (; p1 < c->ntiles; p1++) {
                const TileGeom& g = c->geom_h[p1];
                const size_t m = (size_t)g.w * g.h;
                if (p1 > p0 && n + m > cap) break;
                rgb_taps_host(c->cams_h[p1], g.w, g.h, pw, ph, taps.data() + n);
                if (staged)
                    rgb_patches_host(g, p1, taps.data() + n, pw, ph, patches, units,
                                     loc.data() + n, wts.data() + 2 * n);
                n += m;
            }
            HIPCHK(c, hipMemcpyAsync((RgbTap*)c->rgbtap.p + off0, taps.data(),
                                     sizeof(RgbTap) * n, hipMemcpyHostToDevice, c->stream));
            if (staged) {
                HIPCHK(c, hipMemcpyAsync((uint32_t*)c->rgbloc.p + off0, loc.data(), 4 * n,
                                         hipMemcpyHostToDevice, c->stream));
                HIPCHK(c, hipMemcpyAsync((float*)c->rgbw.p + 2 * off0, wts.data(), 8 * n,
                                         hipMemcpyHostToDevice, c->stream));
            }
            HIPCHK(c, hipStreamSynchronize(c->stream));
            p0 = p1;
        }
        if (staged) {
            // footprint order (32-row bands of the first staged unit, then azimuth), as the
            // depth warp's patches: the blocks resident on one XCD stage overlapping footprints
            // and re-read them from its L2.  Each patch carries its unit-table row along.
            const uint32_t rowb = (uint32_t)(3 * pw);
            std::vector<long long> keys(patches.size());
            for (size_t q = 0; q < patches.size(); q++) {
                const uint32_t u = units[q * kRgbUnits];
                keys[q] = (long long)(u / rowb / 32) * 65536 + (u % rowb) / 3;
            }
            std::vector<size_t> ord(patches.size());
            for (size_t q = 0; q < ord.size(); q++) ord[q] = q;
            std::stable_sort(ord.begin(), ord.end(),
                             [&](size_t a, size_t b) { return keys[a] < keys[b]; });
            std::vector<RgbPatch> sp(patches.size());
            std::vector<uint32_t> su(units.size());
            for (size_t q = 0; q < ord.size(); q++) {
                sp[q] = patches[ord[q]];
                std::copy(units.begin() + ord[q] * kRgbUnits,
                          units.begin() + (ord[q] + 1) * kRgbUnits, su.begin() + q * kRgbUnits);
            }
            if ((rc = upload(c, c->rgbpatch, sp))) return rc;
            if ((rc = upload(c, c->rgbunits, su))) return rc;
            c->n_rgbpatch = (int)patches.size();
        }
        c->rgb_staged = staged;
        c->rgb_pw = pw;
        c->rgb_ph = ph;
    }
    StageTimer t(c, PF_STAGE_WARP, batch * (3.0 * pw * ph + (double)c->rgb_elems), 1);
    if (c->rgb_staged)
        launch_warp_rgb_box(c->stream, (const TileGeom*)c->geom.p, (const RgbPatch*)c->rgbpatch.p,
                            c->n_rgbpatch, (const uint32_t*)c->rgbunits.p,
                            (const uint32_t*)c->rgbloc.p, (const float*)c->rgbw.p,
                            (const RgbTap*)c->rgbtap.p, (const long long*)c->rgb_off.p, pano, pw,
                            ph, (long long)pw * ph * 3, tiles, c->rgb_elems, batch);
    else
        launch_warp_rgb(c->stream, (const RgbTap*)c->rgbtap.p, (const TileGeom*)c->geom.p,
                        c->ntiles, c->npix_max, (const long long*)c->rgb_off.p, pano, pw, ph,
                        (long long)pw * ph * 3, tiles, c->rgb_elems, batch);
    HIPCHK(c, hipGetLastError());
    return PF_OK;
}

int pf_fuse_partial(pf_ctx* c, const float* tiles, const float* coeffs, int t0, int t1,
                    int out_w, int out_h, float zr0, float zr1, int level, float* lsum,
                    float* cnt)
{
    int rc;
    if ((rc = check_common(c, 1))) return rc;
    if (!tiles || !lsum || !cnt) return fail(c, PF_EINVAL, "NULL buffer");
    if (t0 < 0 || t1 > c->ntiles || t0 > t1)
        return fail(c, PF_EINVAL, "tile range [%d,%d) outside [0,%d)", t0, t1, c->ntiles);
    if ((rc = prepare_levels(c, out_w, out_h, zr0, zr1))) return rc;
    LevelCache& lc = c->lc;
    if (level < 0 || level >= lc.nlevels) return fail(c, PF_EINVAL, "bad level %d", level);
    const LevelDims& L = lc.dims[level];
    HIPCHK(c, hipMemsetAsync(lsum, 0, sizeof(float) * L.w * L.h, c->stream));
    HIPCHK(c, hipMemsetAsync(cnt, 0, sizeof(float) * L.w * L.h, c->stream));
    HIPCHK(c, launch_targets_partial(c->stream, (const TileGeom*)c->geom.p,
                               (const TileBox*)lc.box[level].p, (const TapBox*)lc.tapbox[level].p,
                               (const uint32_t*)lc.tmask[level].p, (c->ntiles + 31) / 32, t0, t1,
                               (const int32_t*)lc.tapmap[level].p, tiles, coeffs, L, lsum, cnt,
                               L.h0, L.h1 + 1));
    HIPCHK(c, hipGetLastError());
    return PF_OK;
}

// Row-restricted pieces of the sharded fusion (pf_dist.fuse_row_sharded): a rank computes only
// the rows it sweeps (plus halo) and the rows its tiles send to its neighbours.
static int level_rows(pf_ctx* c, int out_w, int out_h, float zr0, float zr1, int level, int& row0,
                      int& row1, const LevelDims** Lp)
{
    int rc;
    if ((rc = check_common(c, 1))) return rc;
    if ((rc = prepare_levels(c, out_w, out_h, zr0, zr1))) return rc;
    if (level < 0 || level >= c->lc.nlevels) return fail(c, PF_EINVAL, "bad level %d", level);
    const LevelDims& L = c->lc.dims[level];
    if (row0 < 0 || row1 > L.h || row0 > row1)
        return fail(c, PF_EINVAL, "rows [%d,%d) outside [0,%d)", row0, row1, L.h);
    row0 = std::max(row0, L.h0);  // the band: rows outside it are never targets
    row1 = std::min(row1, L.h1 + 1);
    *Lp = &L;
    return PF_OK;
}

int pf_fuse_partial_rows(pf_ctx* c, const float* tiles, const float* coeffs, int t0, int t1,
                         int out_w, int out_h, float zr0, float zr1, int level, int row0,
                         int row1, float* lsum, float* cnt)
{
    int rc;
    const LevelDims* L = nullptr;
    if ((rc = level_rows(c, out_w, out_h, zr0, zr1, level, row0, row1, &L))) return rc;
    if (!tiles || !lsum || !cnt) return fail(c, PF_EINVAL, "NULL buffer");
    if (t0 < 0 || t1 > c->ntiles || t0 > t1)
        return fail(c, PF_EINVAL, "tile range [%d,%d) outside [0,%d)", t0, t1, c->ntiles);
    const LevelCache& lc = c->lc;
    HIPCHK(c, launch_targets_partial(c->stream, (const TileGeom*)c->geom.p,
                               (const TileBox*)lc.box[level].p, (const TapBox*)lc.tapbox[level].p,
                               (const uint32_t*)lc.tmask[level].p, (c->ntiles + 31) / 32, t0, t1,
                               (const int32_t*)lc.tapmap[level].p, tiles, coeffs, *L, lsum, cnt,
                               row0, std::max(row0, row1)));
    HIPCHK(c, hipGetLastError());
    return PF_OK;
}

int pf_fuse_coverage_rows(pf_ctx* c, int out_w, int out_h, float zr0, float zr1, int level,
                          int row0, int row1, float* cnt)
{
    int rc;
    const LevelDims* L = nullptr;
    if ((rc = level_rows(c, out_w, out_h, zr0, zr1, level, row0, row1, &L))) return rc;
    if (!cnt) return fail(c, PF_EINVAL, "NULL buffer");
    launch_coverage_rows(c->stream, (const TileBox*)c->lc.box[level].p, c->ntiles, *L, cnt, row0,
                         row1);
    HIPCHK(c, hipGetLastError());
    return PF_OK;
}

int pf_fuse_normalize_rows(pf_ctx* c, const float* lsum, const float* cnt, int out_w, int out_h,
                           float zr0, float zr1, int level, int row0, int row1, float* lnorm)
{
    int rc;
    const LevelDims* L = nullptr;
    if ((rc = level_rows(c, out_w, out_h, zr0, zr1, level, row0, row1, &L))) return rc;
    if (!lsum || !cnt || !lnorm) return fail(c, PF_EINVAL, "NULL buffer");
    if (row1 > row0) launch_normalize(c->stream, lsum, cnt, *L, lnorm, row0, row1);
    HIPCHK(c, hipGetLastError());
    return PF_OK;
}

int pf_fuse_tile_rows(pf_ctx* c, int out_w, int out_h, float zr0, float zr1, int level, int t0,
                      int t1, int* ymin, int* ymax)
{
    int rc;
    if ((rc = check_common(c, 1))) return rc;
    if (!ymin || !ymax) return fail(c, PF_EINVAL, "NULL output");
    if ((rc = prepare_levels(c, out_w, out_h, zr0, zr1))) return rc;
    if (level < 0 || level >= c->lc.nlevels) return fail(c, PF_EINVAL, "bad level %d", level);
    if (t0 < 0 || t1 > c->ntiles || t0 > t1)
        return fail(c, PF_EINVAL, "tile range [%d,%d) outside [0,%d)", t0, t1, c->ntiles);
    const LevelDims& L = c->lc.dims[level];
    int lo = INT32_MAX, hi = INT32_MIN;
    for (int p = t0; p < t1; p++) {  // rows where k_targets_patch_partial can write a non-zero sum
        const TileBox& b = c->lc.box_h[level][p];
        const int a = std::max(std::min(b.y0, b.y1), L.h0 + 1);
        const int z = std::min(std::max(b.y0, b.y1), L.h1 - 1);
        if (a > z) continue;
        lo = std::min(lo, a);
        hi = std::max(hi, z);
    }
    *ymin = lo == INT32_MAX ? 0 : lo;
    *ymax = lo == INT32_MAX ? -1 : hi;
    return PF_OK;
}

int pf_rows_add(pf_ctx* c, float* dst, const float* src, long long n)
{
    int rc;
    if ((rc = check_common(c, 1))) return rc;
    if (n < 0 || (n > 0 && (!dst || !src))) return fail(c, PF_EINVAL, "bad rows add");
    launch_rows_add(c->stream, dst, src, n);
    HIPCHK(c, hipGetLastError());
    return PF_OK;
}

int pf_rows_add_batch(pf_ctx* c, float* const* dst, const float* const* src, const long long* n,
                      int count)
{
    int rc;
    if ((rc = check_common(c, 1))) return rc;
    if (count < 0 || (count > 0 && (!dst || !src || !n))) return fail(c, PF_EINVAL, "bad rows add batch");
    for (int k = 0; k < count; k++)  // every segment checked before any is added
        if (n[k] < 0 || (n[k] > 0 && (!dst[k] || !src[k])))
            return fail(c, PF_EINVAL, "bad rows add segment %d", k);
    // launches of up to kRowsAddBatch non-empty segments; k walks the list once (empty segments
    // are skipped, so a launch may span more than kRowsAddBatch entries)
    for (int k = 0; k < count;) {
        RowsAddBatch B{};
        int m = 0;
        long long nmax = 0;
        for (; k < count && m < kRowsAddBatch; k++) {
            if (n[k] == 0) continue;
            B.dst[m] = dst[k];
            B.src[m] = src[k];
            B.n[m] = n[k];
            nmax = std::max(nmax, n[k]);
            m++;
        }
        launch_rows_add_batch(c->stream, B, m, nmax);
        HIPCHK(c, hipGetLastError());
    }
    return PF_OK;
}

int pf_fuse_seed(pf_ctx* c, const float* emap, int ew, int eh, int ec, const float* prev,
                 int out_w, int out_h, float zr0, float zr1, int level, float* buf)
{
    int rc;
    if ((rc = check_common(c, 1))) return rc;
    if (!buf) return fail(c, PF_EINVAL, "NULL buffer");
    if ((rc = prepare_levels(c, out_w, out_h, zr0, zr1))) return rc;
    LevelCache& lc = c->lc;
    if (level < 0 || level >= lc.nlevels) return fail(c, PF_EINVAL, "bad level %d", level);
    const LevelDims& L = lc.dims[level];
    if (level == 0) {
        if ((rc = check_emap(c, emap, ew, eh, ec))) return rc;
        launch_seed0(c->stream, emap, ew, eh, ec, 0, (const GridCol*)lc.cols[0].p,
                     (const GridRow*)lc.rows[0].p, L, buf, 0, 1);
    } else {
        if (!prev) return fail(c, PF_EINVAL, "level %d needs the previous level's buffer", level);
        launch_upsample(c->stream, prev, 0, L, buf, 0, 1);
    }
    HIPCHK(c, hipGetLastError());
    return PF_OK;
}

int pf_fuse_finish_level(pf_ctx* c, const float* lsum, const float* cnt, int out_w, int out_h,
                         float zr0, float zr1, int level, float* buf, uint16_t* out)
{
    int rc;
    if ((rc = check_common(c, 1))) return rc;
    if (!lsum || !cnt || !buf) return fail(c, PF_EINVAL, "NULL buffer");
    if ((rc = prepare_levels(c, out_w, out_h, zr0, zr1))) return rc;
    LevelCache& lc = c->lc;
    if (level < 0 || level >= lc.nlevels) return fail(c, PF_EINVAL, "bad level %d", level);
    const LevelDims& L = lc.dims[level];
    const long long st = (long long)L.w * L.h;
    if ((rc = ensure(c, c->lnorm, sizeof(float) * st))) return rc;
    if ((rc = ensure(c, c->lsum_ws, sizeof(float) * st))) return rc;
    launch_normalize(c->stream, lsum, cnt, L, (float*)c->lnorm.p);
    float* other = (float*)c->lsum_ws.p;
    // every pass stores every band row [h0, h1] of the plane it writes (pf_jacobi.hip): the second
    // plane takes the rows outside the band's interior (h0, h1), and the band comes back at the end
    const size_t rowb = sizeof(float) * (size_t)L.w;
    const int ia = std::max(L.h0 + 1, 0), ib = std::min(L.h1, L.h);  // interior rows [ia, ib)
    const int ba = std::max(L.h0, 0), bb = std::min(L.h1 + 1, L.h);  // band rows [ba, bb)
    HIPCHK(c, hipMemcpyAsync(other, buf, rowb * ia, hipMemcpyDeviceToDevice, c->stream));
    if (ib < L.h)
        HIPCHK(c, hipMemcpyAsync(other + (size_t)ib * L.w, buf + (size_t)ib * L.w,
                                 rowb * (L.h - ib), hipMemcpyDeviceToDevice, c->stream));
    float* res = nullptr;
    if (jacobi_tcap(L) >= 1)
        res = run_jacobi(c, L, 0, nullptr, 0, 0, 0, 0, nullptr, nullptr, nullptr, 0,
                         (const float*)c->lnorm.p, buf, other, nullptr, 0, 1, nullptr,
                         lc.full[level] ? (const float*)lc.hcol[level].p : nullptr);
    else
        launch_jacobi(c->stream, buf, other, (const float*)c->lnorm.p, st, L, L.iters, 1, &res);
    if (res != buf && bb > ba)
        HIPCHK(c, hipMemcpyAsync(buf + (size_t)ba * L.w, res + (size_t)ba * L.w,
                                 rowb * (bb - ba), hipMemcpyDeviceToDevice, c->stream));
    if (level == lc.nlevels - 1 && out) launch_quantize(c->stream, buf, st, (int)st, out, st, 1);
    HIPCHK(c, hipGetLastError());
    return PF_OK;
}

// One level's normalised targets of one panorama from every tile (the one-GPU gather,
// k_targets_patch with one-panorama blocks): the replicated levels of a one-rank row-sharded
// fusion need no partial sums.
int pf_fuse_targets(pf_ctx* c, const float* tiles, const float* coeffs, int out_w, int out_h,
                    float zr0, float zr1, int level, float* lnorm)
{
    int rc;
    if ((rc = check_common(c, 1))) return rc;
    if (!tiles || !lnorm) return fail(c, PF_EINVAL, "NULL buffer");
    if ((rc = prepare_levels(c, out_w, out_h, zr0, zr1))) return rc;
    const LevelCache& lc = c->lc;
    if (level < 0 || level >= lc.nlevels) return fail(c, PF_EINVAL, "bad level %d", level);
    const LevelDims& L = lc.dims[level];
    launch_targets_patch(c->stream, (const TileGeom*)c->geom.p, (const TileBox*)lc.box[level].p,
                         (const TapBox*)lc.tapbox[level].p, c->ntiles,
                         (const int32_t*)lc.tapmap[level].p, tiles, c->tile_elems, coeffs, L,
                         lnorm, (long long)L.w * L.h, 1, (const uint32_t*)lc.tmask[level].p,
                         (c->ntiles + 31) / 32);
    HIPCHK(c, hipGetLastError());
    return PF_OK;
}

// One whole level of one panorama from its summed targets, seeded inside the sweeps: the
// one-call path's level (fuse_range) for a caller that gathered (lsum, cnt) itself -- the
// replicated levels of pf_dist.fuse_row_sharded.  pf_fuse_seed + pf_fuse_finish_level give the
// same planes, through a seeded full-level plane and two copies.  cnt == NULL: lsum already holds
// the normalised targets (pf_fuse_targets).
int pf_fuse_level(pf_ctx* c, const float* emap, int ew, int eh, int ec, const float* prev,
                  const float* lsum, const float* cnt, int out_w, int out_h, float zr0, float zr1,
                  int level, float* buf, uint16_t* out)
{
    int rc;
    if ((rc = check_common(c, 1))) return rc;
    if (!lsum || !buf) return fail(c, PF_EINVAL, "NULL buffer");
    if ((rc = prepare_levels(c, out_w, out_h, zr0, zr1))) return rc;
    LevelCache& lc = c->lc;
    if (level < 0 || level >= lc.nlevels) return fail(c, PF_EINVAL, "bad level %d", level);
    const LevelDims& L = lc.dims[level];
    if (level == 0) {
        if ((rc = check_emap(c, emap, ew, eh, ec))) return rc;
    } else if (!prev) {
        return fail(c, PF_EINVAL, "level %d needs the previous level's buffer", level);
    }
    const long long st = (long long)L.w * L.h;
    if ((rc = ensure(c, c->lnorm, sizeof(float) * st))) return rc;
    if ((rc = ensure(c, c->lsum_ws, sizeof(float) * st))) return rc;
    const bool last = level == lc.nlevels - 1;
    uint16_t* o = last ? out : nullptr;
    if (cnt) launch_normalize(c->stream, lsum, cnt, L, (float*)c->lnorm.p);
    const float* ln = cnt ? (const float*)c->lnorm.p : lsum;
    float* other = (float*)c->lsum_ws.p;
    const int ba = std::max(L.h0, 0), bb = std::min(L.h1 + 1, L.h);  // band rows [ba, bb)
    float* res = nullptr;
    if (jacobi_tcap(L) < 1) {  // the plain sweep form: a seeded full plane, copied, swept
        if ((rc = pf_fuse_seed(c, emap, ew, eh, ec, prev, out_w, out_h, zr0, zr1, level, buf)))
            return rc;
        HIPCHK(c, hipMemcpyAsync(other, buf, sizeof(float) * st, hipMemcpyDeviceToDevice,
                                 c->stream));
        launch_jacobi(c->stream, buf, other, ln, st, L, L.iters, 1, &res);
        if (res != buf && bb > ba)
            HIPCHK(c, hipMemcpyAsync(buf + (size_t)ba * L.w, res + (size_t)ba * L.w,
                                     sizeof(float) * (size_t)L.w * (bb - ba),
                                     hipMemcpyDeviceToDevice, c->stream));
        if (o) launch_quantize(c->stream, buf, st, (int)st, o, st, 1);
        HIPCHK(c, hipGetLastError());
        return PF_OK;
    }
    if (level == 0 && (rc = seed_tables(c, L, ew, eh, ec))) return rc;
    const JresPlan jp = jres_plan(c, L, 1, lc.full[level]);
    if (jp.on && (rc = jres_prepare(c, L, 1, jp))) return rc;
    // the rows outside the band, in both planes (the u16 rows too on the last level)
    launch_border(c->stream, level == 0 ? nullptr : prev, 0, L, buf, other, st, o, st, 1);
    res = run_jacobi(c, L, level == 0 ? 2 : 1, emap, ew, eh, ec, 0,
                     (const GridCol*)lc.cols[level].p, (const GridRow*)lc.rows[level].p, prev, 0,
                     ln, buf, other, o, st, 1, nullptr,
                     lc.full[level] ? (const float*)lc.hcol[level].p : nullptr, &jp);
    if (!res) return fail(c, PF_EINVAL, "level-0 seed tables missing");
    if (res != buf && bb > ba && !o)  // the band back into buf (its other rows are equal)
        HIPCHK(c, hipMemcpyAsync(buf + (size_t)ba * L.w, res + (size_t)ba * L.w,
                                 sizeof(float) * (size_t)L.w * (bb - ba),
                                 hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipGetLastError());
    return PF_OK;
}

// ---- row-band sharding of one level's sweeps (pf_dist.fuse_row_sharded) ----
int pf_fuse_normalize(pf_ctx* c, const float* lsum, const float* cnt, int out_w, int out_h,
                      float zr0, float zr1, int level, float* lnorm)
{
    int rc;
    if ((rc = check_common(c, 1))) return rc;
    if (!lsum || !cnt || !lnorm) return fail(c, PF_EINVAL, "NULL buffer");
    if ((rc = prepare_levels(c, out_w, out_h, zr0, zr1))) return rc;
    if (level < 0 || level >= c->lc.nlevels) return fail(c, PF_EINVAL, "bad level %d", level);
    launch_normalize(c->stream, lsum, cnt, c->lc.dims[level], lnorm);
    HIPCHK(c, hipGetLastError());
    return PF_OK;
}

int pf_fuse_multicover(pf_ctx* c, const float* tiles, const float* coeffs, int t0, int t1,
                       int out_w, int out_h, float zr0, float zr1, int level, float* contrib,
                       int* npairs)
{
    int rc;
    if ((rc = check_common(c, 1))) return rc;
    if ((rc = prepare_levels(c, out_w, out_h, zr0, zr1))) return rc;
    const LevelCache& lc = c->lc;
    if (level < 0 || level >= lc.nlevels) return fail(c, PF_EINVAL, "bad level %d", level);
    if (npairs) *npairs = lc.nmc[level];
    if (!contrib || lc.nmc[level] == 0) return PF_OK;
    if (!tiles) return fail(c, PF_EINVAL, "NULL tiles");
    if (t0 < 0 || t1 > c->ntiles || t0 > t1)
        return fail(c, PF_EINVAL, "tile range [%d,%d) outside [0,%d)", t0, t1, c->ntiles);
    launch_multicover(c->stream, (const TileGeom*)c->geom.p, (const int2*)lc.mcpairs[level].p,
                      lc.nmc[level], t0, t1, (const GridCol*)lc.cols[level].p,
                      (const GridRow*)lc.rows[level].p, tiles, coeffs, lc.dims[level], contrib);
    HIPCHK(c, hipGetLastError());
    return PF_OK;
}

int pf_fuse_multicover_patch(pf_ctx* c, int out_w, int out_h, float zr0, float zr1, int level,
                             const float* contrib, float* lsum)
{
    int rc;
    if ((rc = check_common(c, 1))) return rc;
    if ((rc = prepare_levels(c, out_w, out_h, zr0, zr1))) return rc;
    const LevelCache& lc = c->lc;
    if (level < 0 || level >= lc.nlevels) return fail(c, PF_EINVAL, "bad level %d", level);
    if (lc.nmc[level] == 0) return PF_OK;
    if (!contrib || !lsum) return fail(c, PF_EINVAL, "NULL buffer");
    launch_multicover_patch(c->stream, (const int2*)lc.mcpairs[level].p, lc.nmc[level], contrib,
                            lsum);
    HIPCHK(c, hipGetLastError());
    return PF_OK;
}

int pf_fuse_border(pf_ctx* c, const float* prev, int out_w, int out_h, float zr0, float zr1,
                   int level, float* a, float* b, uint16_t* out)
{
    int rc;
    if ((rc = check_common(c, 1))) return rc;
    if ((rc = prepare_levels(c, out_w, out_h, zr0, zr1))) return rc;
    const LevelCache& lc = c->lc;
    if (level < 0 || level >= lc.nlevels) return fail(c, PF_EINVAL, "bad level %d", level);
    if (level > 0 && !prev) return fail(c, PF_EINVAL, "level %d needs the previous level", level);
    const bool last = level == lc.nlevels - 1;
    if (last ? !out : (!a || !b)) return fail(c, PF_EINVAL, "NULL buffer");
    const LevelDims& L = lc.dims[level];
    const long long st = (long long)L.w * L.h;
    const long long pst = level > 0 ? (long long)lc.dims[level - 1].w * lc.dims[level - 1].h : 0;
    launch_border(c->stream, level == 0 ? nullptr : prev, pst, L, a, b, st, last ? out : nullptr,
                  st, 1);  // last level: a / b (if given) get the rows h0-1 and h1+1
    HIPCHK(c, hipGetLastError());
    return PF_OK;
}

int pf_fuse_band_plan(pf_ctx* c, int out_w, int out_h, float zr0, float zr1, int level,
                      int nbands, int* T, int cap)
{
    int rc;
    if ((rc = check_common(c, 1))) return rc;
    if (!T || cap < 1 || nbands < 1) return fail(c, PF_EINVAL, "pf_fuse_band_plan: bad arguments");
    if ((rc = prepare_levels(c, out_w, out_h, zr0, zr1))) return rc;
    const LevelCache& lc = c->lc;
    if (level < 0 || level >= lc.nlevels) return fail(c, PF_EINVAL, "bad level %d", level);
    const LevelDims& L = lc.dims[level];
    if (jacobi_tcap(L) < 1)
        return fail(c, PF_EINVAL, "level %d: the zenith band leaves no room for band passes", level);
    const int band = L.h1 - L.h0 + 1;
    // the sweep depths depend only on (level, nbands): every rank derives the same plan
    std::vector<PassPlan> plan = plan_level(c, L, 2, jacobi_tcap(L), 1, lc.full[level],
                                            (band + nbands - 1) / nbands);
    if ((int)plan.size() > cap) return fail(c, PF_EINVAL, "plan of %zu passes > cap %d", plan.size(), cap);
    for (size_t i = 0; i < plan.size(); i++) T[i] = plan[i].T;
    return (int)plan.size();
}

int pf_fuse_band_pass(pf_ctx* c, const float* emap, int ew, int eh, int ec, const float* prev,
                      const float* lnorm, int src_mode, const float* src, float* dst,
                      uint16_t* out, int out_w, int out_h, float zr0, float zr1, int level, int T,
                      int row0, int row1)
{
    int rc;
    if ((rc = check_common(c, 1))) return rc;
    if ((rc = prepare_levels(c, out_w, out_h, zr0, zr1))) return rc;
    const LevelCache& lc = c->lc;
    if (level < 0 || level >= lc.nlevels) return fail(c, PF_EINVAL, "bad level %d", level);
    const LevelDims& L = lc.dims[level];
    if (!lnorm || (!dst && !out)) return fail(c, PF_EINVAL, "NULL buffer");
    if (src_mode < 0 || src_mode > 2) return fail(c, PF_EINVAL, "src_mode %d", src_mode);
    if (src_mode == 0 && !src) return fail(c, PF_EINVAL, "src_mode 0 needs src");
    if (src_mode == 1 && (level == 0 || !prev)) return fail(c, PF_EINVAL, "src_mode 1 needs prev");
    if (src_mode == 2 && (level != 0 || (rc = check_emap(c, emap, ew, eh, ec))))
        return rc ? rc : fail(c, PF_EINVAL, "src_mode 2 (seed) is level 0 only");
    if (T < 1 || T > jacobi_tcap(L) || !jstream_supported_T(T))
        return fail(c, PF_EINVAL, "pass depth %d not available at level %d", T, level);
    if (row0 < L.h0 || row1 > L.h1 + 1 || row0 >= row1)
        return fail(c, PF_EINVAL, "rows [%d,%d) outside the band [%d,%d]", row0, row1, L.h0, L.h1);
    const bool fast = lc.full[level];
    static const JacobiTuning tune = jacobi_tuning();
    const int band = row1 - row0;
    PassPlan pp = best_chunks(T, 2, band, L.w, 1, jstream_waves_per_cu(2, T, fast) / 4,
                              plan_simds(c), tune.step_overhead, tune.lone_cycles, tune.c4_eff);
    const long long st = (long long)L.w * L.h;
    JacobiPass P{};
    if (src_mode == 2) {
        if ((rc = seed_tables(c, L, ew, eh, ec))) return rc;
        P.ecol = (const int*)c->seed_ecol.p;
        P.erow = (const int*)c->seed_erow.p;
    }
    P.prev = prev; P.pstride = 0;
    P.emap = emap; P.estride = 0; P.ew = ew; P.eh = eh; P.ec = ec;
    P.cols = (const GridCol*)lc.cols[level].p; P.rows = (const GridRow*)lc.rows[level].p;
    P.lnorm = lnorm; P.lstride = st;
    P.sstride = st; P.dstride = st;
    P.out = out; P.ostride = st;
    P.w = L.w; P.h = L.h; P.h0 = L.h0; P.h1 = L.h1;
    P.hcol = fast ? (const float*)lc.hcol[level].p : nullptr;
    P.row_lo = row0;
    P.row_hi = row1;
    P.Tp = (T + 1) / 2 * 2;
    P.V = 128 - 2 * P.Tp;
    P.nstrips = (L.w + P.V - 1) / P.V;
    P.rows_per_chunk = (band + pp.nchunks - 1) / pp.nchunks;
    P.nchunks = (band + P.rows_per_chunk - 1) / P.rows_per_chunk;
    P.src_mode = src_mode;
    P.src = src;
    P.dst = dst;
    P.out_mode = out ? 1 : 0;
    launch_jstream(c->stream, P, 2, T, 1, fast);
    HIPCHK(c, hipGetLastError());
    return PF_OK;
}

int pf_probe_taps(pf_ctx* c, int out_w, int out_h, float zr0, float zr1, int level,
                  int32_t* tap_index)
{
    int rc;
    if ((rc = check_common(c, 1))) return rc;
    if (!tap_index) return fail(c, PF_EINVAL, "NULL buffer");
    if ((rc = prepare_levels(c, out_w, out_h, zr0, zr1))) return rc;
    LevelCache& lc = c->lc;
    if (level < 0 || level >= lc.nlevels) return fail(c, PF_EINVAL, "bad level %d", level);
    launch_probe_taps(c->stream, (const TileGeom*)c->geom.p, (const TileBox*)lc.box[level].p,
                      c->ntiles, (const GridCol*)lc.cols[level].p, (const GridRow*)lc.rows[level].p,
                      lc.dims[level], tap_index);
    HIPCHK(c, hipGetLastError());
    return PF_OK;
}

int pf_set_metrics_order(pf_ctx* c, int order)
{
    if (!c) return PF_EINVAL;
    if (order != PF_METRICS_SEQUENTIAL && order != PF_METRICS_TREE)
        return fail(c, PF_EINVAL, "metrics order %d", order);
    c->metrics_order = order;
    return PF_OK;
}

int pf_error_metrics(pf_ctx* c, const float* gt, int gw, int gh, int gc, const float* given,
                     const uint16_t* given16, int w, int h, int given_c, int batch, float zr0,
                     float zr1, int align_way, int cap_depth, pf_metrics* out)
{
    if (!c) return PF_EINVAL;
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, PF_EHIP, "hipSetDevice failed");
    if (!gt || !out || (!given == !given16))
        return fail(c, PF_EINVAL, "pf_error_metrics: need gt, out and exactly one of given/given16");
    if (gw < 1 || gh < 1 || gc < 1 || w < 1 || h < 1 || (given && given_c < 1))
        return fail(c, PF_EINVAL, "pf_error_metrics: bad shape gt %dx%dx%d given %dx%dx%d", gw,
                    gh, gc, w, h, given_c);
    if (batch <= 0 || batch > 65535) return fail(c, PF_EINVAL, "batch %d out of range", batch);
    if (align_way < 0 || align_way > 2) return fail(c, PF_EINVAL, "align_way %d", align_way);
    if ((long long)w * h >= (1ll << 31) || (long long)gw * gh * gc >= (1ll << 31))
        return fail(c, PF_EINVAL, "pf_error_metrics: map too large");
    // Depth.cpp:1984-1985 (int)(g_zenith_range[k] / MYPI * data_height), fp64
    MetricsJob j;
    j.gt = gt;
    j.gw = gw;
    j.gh = gh;
    j.gc = gc;
    j.given = given;
    j.given16 = given16;
    j.w = w;
    j.h = h;
    j.gc_given = given16 ? 1 : given_c;
    j.batch = batch;
    j.h0 = std::max(0, (int)((double)zr0 / PF_MYPI * h));
    j.h1 = std::min(h - 1, (int)((double)zr1 / PF_MYPI * h));
    if (j.h1 < j.h0) return fail(c, PF_EINVAL, "pf_error_metrics: empty zenith band");
    j.align_way = align_way;
    j.cap_depth = cap_depth ? 1 : 0;
    j.sequential = c->metrics_order == PF_METRICS_SEQUENTIAL ? 1 : 0;
    int rc;
    if ((rc = ensure(c, c->metrics_ws, metrics_workspace_bytes(j))))
        return rc;
    // algorithmic bytes: one read of the compared band of gt (4 B, channel 0) and of the
    // result (2 B u16 / 4 B f32); the kernels make 4 passes (3 radix digits + the sums) for
    // align_way 1, 2 for align_way 2, 1 otherwise
    const double band = (double)(j.h1 - j.h0 + 1) * w;
    const int passes = align_way == 1 ? 4 : (align_way == 2 ? 2 : 1);
    StageTimer t(c, PF_STAGE_METRICS, batch * band * (4.0 + (given16 ? 2.0 : 4.0)),
                 align_way == 1 ? 9 : passes + 2);
    launch_metrics(c->stream, j, c->metrics_ws.p, out);
    HIPCHK(c, hipGetLastError());
    return PF_OK;
}

int pf_depth_transform(pf_ctx* c, float* data, long long npix, int channels, const float* abcd)
{
    if (!c) return PF_EINVAL;
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, PF_EHIP, "hipSetDevice failed");
    if (!data || !abcd || npix < 0 || channels < 1)
        return fail(c, PF_EINVAL, "pf_depth_transform: bad arguments");
    if (npix == 0) return PF_OK;
    launch_d2d_map(c->stream, data, npix, channels, abcd);
    HIPCHK(c, hipGetLastError());
    return PF_OK;
}

int pf_register_joint(pf_ctx* c, const float* emap, int ew, int eh, int ec, const float* tiles,
                      int batch, float zr0, float zr1, int degree, const int* active,
                      float* coeffs, double* coeffs64)
{
    int rc;
    if ((rc = check_common(c, batch))) return rc;
    if ((rc = check_emap(c, emap, ew, eh, ec))) return rc;
    if (!tiles || !active) return fail(c, PF_EINVAL, "tiles/active is NULL");
    if (degree < 0 || degree > 3) return fail(c, PF_EINVAL, "degree %d not in [0,3]", degree);
    if ((rc = prepare_registration(c, zr0, zr1))) return rc;
    std::vector<int> act(active, active + c->ntiles);
    int nact = 0;
    for (int v : act) nact += v != 0;
    if (nact == 0) return fail(c, PF_EINVAL, "pf_register_joint: no active tile");
    if ((rc = check_reg_grids(c, act.data()))) return rc;
    if ((rc = upload(c, c->reg_active, act))) return rc;
    if ((rc = ensure(c, c->reg_sums,
                     sizeof(double) * register_sums_per_tile() * c->ntiles * batch)))
        return rc;
    float* cf = coeffs;
    if (!cf) {
        if ((rc = ensure(c, c->coeffs, sizeof(float) * 4 * batch))) return rc;
        cf = (float*)c->coeffs.p;
    }
    launch_register(c->stream, (const TileGeom*)c->geom.p, (const RegGrid*)c->reg.p,
                    (const GridCol*)c->rcols.p, (const GridRow*)c->rrows.p, c->ntiles, emap, ew,
                    eh, ec, (long long)ew * eh * ec, tiles, c->tile_elems, degree, c->solver,
                    nullptr, nullptr, batch, (double*)c->reg_sums.p,
                    (const int*)c->reg_active.p, reg_sample_index(c, ew, eh, ec));
    launch_register_joint(c->stream, (const double*)c->reg_sums.p, (const int*)c->reg_active.p,
                          c->ntiles, batch, degree, c->solver, cf, coeffs64);
    HIPCHK(c, hipGetLastError());
    return PF_OK;
}

}  // extern "C"
