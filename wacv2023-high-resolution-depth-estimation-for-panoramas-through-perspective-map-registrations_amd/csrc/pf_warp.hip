// pf_warp.hip -- E->P depth warp as an LDS-staged gather for gfx950.
//
// For every tile pixel (X, Y) the reference mapping is ToSphericalCoord (Depth.cpp:157-166):
// corner0 + hedge*x + vedge*y -> WorldToSpherical (Depth.cpp:2960-2971) -> a bilinear sample of
// the panorama at ValueAtCoord's pixel convention (az/2pi*(pw-1), zen/pi*(ph-1)).  That mapping
// depends only on the layout and the panorama size, so it is evaluated once (cached by the
// context) and the per-call kernel does no trigonometry:
//
//  1. warp_coords_host: per tile pixel the bilinear corner (x0, y0) and weights (fx, fy), on the
//                    host with glibc atan2f as the reference calls it (bit-exact maps).
//  2. k_patch_box:   tiles are cut into 32x32-pixel patches; per patch the panorama footprint
//                    (an azimuth-unwrapped box, <= kCap floats, or "wide").
//  3. k_warp_local:  per tile pixel the corner's index inside its patch's footprint box (or the
//                    global index with edge flags for a wide patch).
//
// k_warp_depth: one block per (patch, chunk of kNB panoramas).  Per panorama the block copies the
// footprint box from HBM into LDS with plain coalesced row loads (double-buffered: the loads for
// panorama q+1 are in flight while panorama q is interpolated), then every pixel reads its four
// corners from LDS.  The box is ~0.4x the panorama's bytes per panorama (vs ~4 scattered corner
// loads per tile pixel from L2 in a direct gather), so the kernel is bound by the tile writes.
//
// Edge rule: the reference clamps x1 = min(x0+1, pw-1), y1 = min(y0+1, ph-1).  x0 == pw-1 only
// when px == pw-1 exactly (az < 2*MYPI), i.e. fx == 0, and likewise y0 == ph-1 means fy == 0; the
// neighbour's weight is then exactly zero, so the box may hold any finite value there (the box
// wraps in azimuth and clamps rows).  Inputs are depth maps, finite by contract.
#include "pf_geom.hpp"
#include "pf_internal.hpp"

#include <algorithm>
#include <cfloat>
#include <thread>
#include <type_traits>
#include <vector>

namespace pf {

#ifndef PF_WARP_WB
#define PF_WARP_WB 256
#endif
#ifndef PF_WARP_PATCH
#define PF_WARP_PATCH 64
#endif
#ifndef PF_WARP_WAVEBOX
// one 32x8 patch per WAVE with its own LDS box and no workgroup barrier (waves drift and overlap
// each other's latencies) instead of one 32x32 patch per 256-thread block with a barrier per
// panorama (SQ counters: ~20% of the block form's wave-cycles wait at barriers).  Measured
// slower on MI355X at C3 (profiles/r03/warp/wb*.log; recipe: tools/gpu_round.sh ab): 0.69 ms with 1024-float wave boxes, 0.83 with 512,
// against 0.53 for the block form (bit-identical tiles) -- the small boxes re-read more and send
// more patches to the direct-gather path.  Off.
#define PF_WARP_WAVEBOX 0
#endif
static constexpr int kWB = PF_WARP_WB;                  // threads per block
static constexpr int kPatch = PF_WARP_PATCH;            // patch width in tile pixels
#ifndef PF_WARP_PATCHH
// Round 6: 64 x 32 patches (2048 pixels, 8 per thread) instead of 32 x 32.  Their ragged
// footprints touch 37.9 cache lines per 1024 tile pixels instead of 47.4 (a host model of every
// C3 patch; the footprint rows are longer, so fewer partial lines at the row ends): serial trace
// 0.491-0.494 -> 0.478-0.481 ms per C3 launch; 64 x 16: 0.496-0.499 (46.2 lines); 64 x 32 with
// 512 threads 0.481-0.484; 128 x 16 with 512 threads 0.478-0.481 (tools/gpu_round.sh serials)
#define PF_WARP_PATCHH 32
#endif
static constexpr int kPatchH = PF_WARP_WAVEBOX ? 8 : PF_WARP_PATCHH;  // patch height
static_assert(kWB % kPatch == 0 && kPatch * kPatchH % kWB == 0, "whole patch rows per slot");
static_assert(!PF_WARP_WAVEBOX || (kPatch == 32 && kWB == 256), "wave boxes: 32x8 patches");
static constexpr int kPx = kPatch * kPatchH / kWB;      // pixels per thread (prep passes)
#ifndef PF_WARP_CAP
#define PF_WARP_CAP 4096
#endif
static constexpr int kCapB = PF_WARP_CAP;               // LDS floats per parity per block
static constexpr int kCap = PF_WARP_WAVEBOX ? kCapB / 4 : kCapB;  // per staged footprint
static constexpr int kSlots = kCap / kWB;               // staging loads per thread
static_assert(PF_WARP_WAVEBOX || kCap % (4 * kWB) == 0, "whole 16-B staging slots fill the box");
#ifndef PF_WARP_BATCH
#define PF_WARP_BATCH 16
#endif
static constexpr int kNB = PF_WARP_BATCH;               // panoramas per block
// Memory operation widths and cache policy, measured on MI355X at C3 (tools/warp_probe.py,
// profiles/r03/warp; recipe: tools/gpu_round.sh ab).  Round 2: 16-B staging loads 0.596 ms, 16-B row stores 0.600, both 0.637,
// against 0.586 for 4-B loads and stores.  Round 3, with the split LDS parities: nt tile stores
// 0.545-0.551 ms against 0.560-0.569 (written tiles no longer evict the staged boxes' lines from
// L2), and 16-B staging loads on top 0.527-0.531 (kept: the defaults below); 16-B stores through
// a wave-local LDS transpose 0.573-0.578, 16-B row stores 0.576-0.586 (not kept); 64x64 patches
// 0.75-1.4 ms (more footprints exceed the LDS box); 5 blocks per CU (3840-float box, 96 VGPRs)
// 0.539-0.541 without the 16-B loads.
#ifndef PF_WARP_V4
#define PF_WARP_V4 1     // quad-aligned footprint boxes staged with 16-B loads (pw % 4 == 0)
#endif
#ifndef PF_WARP_SPLIT
// the two staging parities in separate LDS halves (consecutive lanes read/write consecutive
// dwords: conflict-free) instead of interleaved (stride-2 dwords: 2-way bank conflicts, 64% of
// the kernel's LDS-active cycles on MI355X, profiles/r03/warp/warp_sq_summary.txt; recipe: tools/gpu_round.sh pmc-style passes)
#define PF_WARP_SPLIT 1
#endif
#ifndef PF_WARP_STPOL
#define PF_WARP_STPOL 2  // cache policy bits of the tile stores (gfx950: 2 = nt, 16 = sc1)
#endif
#ifndef PF_WARP_PFD
#define PF_WARP_PFD 2    // staging prefetch depth in panoramas (register sets in flight)
#endif
#ifndef PF_WARP_DIAG
#define PF_WARP_DIAG 0   // probes only: 1 = no tile stores, 2 = no panorama loads (wrong output)
#endif
#ifndef PF_WARP_XPOSE
// results pass through a wave-local LDS transpose so every lane stores its 4 pixels of one tile
// row with one 16-B store (the compute keeps the 32-lanes-per-row mapping the box reads want)
#define PF_WARP_XPOSE 0  // measured slower on MI355X (0.573-0.578 ms vs 0.527-0.528 at C3)
#endif
#ifndef PF_WARP_ROWPX
#define PF_WARP_ROWPX 0  // a thread's pixels consecutive in one row: one 16-B store per panorama
#endif

__device__ __forceinline__ uint32_t mix32(uint32_t x)
{  // lowbias32 finaliser (the oracle's pfo_hash32)
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    x ^= x >> 16;
    return x;
}

// Pass 1 (host, once per layout and panorama size): bilinear corner and weights of every tile
// pixel, wxy = x0 | y0 << 16.  Evaluated on the host with glibc's atan2f -- the function the
// reference's WorldToSpherical calls (Depth.cpp:2960-2971) -- through pf_geom.hpp's Imath-order
// ToSphericalCoord (Depth.cpp:157-166), so the corner indices and weights are the reference's
// bits (glibc atan2f is not correctly rounded: 16% of its results differ from a rounded fp64
// evaluation, which is what device code would give).  Rows are split over host threads.
template <class F>
static void host_rows(int h, F&& f)
{
    unsigned nt = std::thread::hardware_concurrency();
    nt = nt < 1 ? 1 : (nt > 16 ? 16 : nt);  // the GPU box grants 16 host CPUs per GPU
    if ((long long)h * 64 < 4096 || nt == 1) {
        f(0, h);
        return;
    }
    std::vector<std::thread> th;
    const int per = (h + (int)nt - 1) / (int)nt;
    for (int y0 = 0; y0 < h; y0 += per) th.emplace_back(f, y0, std::min(h, y0 + per));
    for (auto& t : th) t.join();
}

void warp_coords_host(const TileGeom& g, int pw, int ph, uint32_t* wxy, float* wfxy)
{
    pfgeom::Window win{};
    win.corner0 = {g.corner0[0], g.corner0[1], g.corner0[2]};
    win.hedge = {g.hedge[0], g.hedge[1], g.hedge[2]};
    win.vedge = {g.vedge[0], g.vedge[1], g.vedge[2]};
    host_rows(g.h, [&](int ya, int yb) {
        for (int Y = ya; Y < yb; Y++)
            for (int X = 0; X < g.w; X++) {
                const float xf = (float)X / (float)(g.w - 1), yf = (float)Y / (float)(g.h - 1);
                float az, zen;
                pfgeom::to_spherical_coord(win, xf, yf, az, zen);
                const float px = (float)((double)az / (2 * PF_MYPI) * (double)(pw - 1));
                const float py = (float)((double)zen / PF_MYPI * (double)(ph - 1));
                int x0 = (int)floorf(px), y0 = (int)floorf(py);
                float fx = px - (float)x0, fy = py - (float)y0;
                if (x0 < 0) { x0 = 0; fx = 0; }
                if (y0 < 0) { y0 = 0; fy = 0; }
                if (x0 > pw - 1) { x0 = pw - 1; fx = 0; }
                if (y0 > ph - 1) { y0 = ph - 1; fy = 0; }
                const long long i = (long long)Y * g.w + X;
                wxy[i] = (uint32_t)x0 | ((uint32_t)y0 << 16);
                wfxy[2 * i] = fx;
                wfxy[2 * i + 1] = fy;
            }
    });
}

static inline long long floor_div(long long x, long long d) { return x >= 0 ? x / d : -((d - 1 - x) / d); }
static inline int wrap_du_h(int d, int pw)
{  // the column offset d in (-pw/2, pw/2] (k_patch_box's wrap_du, host side)
    if (d > pw / 2) d -= pw;
    if (d < -(pw / 2)) d += pw;
    return d;
}

// Ragged footprints of the depth warp's 32x32 patches (round 5).  The bounding box of a patch's
// corners (k_patch_box) holds the empty corners of a rotated footprint and whole rows of
// columns no corner of that row reads; here each panorama row v of the footprint is staged only
// over the columns [xlo(v), xhi(v)] its corners use (pixels with y0 == v read their (x0, x0+1) on
// row v, pixels with y0 == v-1 on row v as y1), in whole 16-B units, the rows packed one after
// another in LDS.  Columns unwrap around the patch's first corner (the azimuth seam: staging
// wraps mod pw); rows past ph-1 (y1 clamped: fy == 0 there) stage row ph-1.
void warp_patches_host(const TileGeom& g, int tile, const uint32_t* wxy, int pw, int ph,
                       std::vector<WarpPatch>& patches, std::vector<uint32_t>& units,
                       uint32_t* loc)
{
    const int cap = kCap / 4;  // 16-B units per staged footprint
    // PF_WARP_ALIGN=n (A/B): each footprint row's units start and end on
    // n-unit boundaries (8 = whole 128-B lines), so the 64 16-B loads of a wave instruction touch
    // whole lines; the LDS box grows by the rounding
    static const int align = [] {
        const char* e = getenv("PF_WARP_ALIGN");
        const int a = e ? atoi(e) : 1;
        return a == 2 || a == 4 || a == 8 ? a : 1;
    }();
    std::vector<int> xlo, xhi, q0, off;
    for (int Y0 = 0; Y0 < g.h; Y0 += kPatchH)
        for (int X0 = 0; X0 < g.w; X0 += kPatch) {
            const int X1 = std::min(g.w, X0 + kPatch), Y1 = std::min(g.h, Y0 + kPatchH);
            const uint32_t m0 = wxy[(long long)Y0 * g.w + X0];
            const int rx = (int)(m0 & 0xFFFFu);
            int vmin = INT32_MAX, vmax = INT32_MIN;
            for (int Y = Y0; Y < Y1; Y++)
                for (int X = X0; X < X1; X++) {
                    const int y0 = (int)(wxy[(long long)Y * g.w + X] >> 16);
                    vmin = std::min(vmin, y0);
                    vmax = std::max(vmax, y0);
                }
            const int nv = vmax - vmin + 2;
            xlo.assign(nv, INT32_MAX);
            xhi.assign(nv, INT32_MIN);
            for (int Y = Y0; Y < Y1; Y++)
                for (int X = X0; X < X1; X++) {
                    const uint32_t m = wxy[(long long)Y * g.w + X];
                    const int du = wrap_du_h((int)(m & 0xFFFFu) - rx, pw);
                    const int r = (int)(m >> 16) - vmin;
                    for (int k = r; k <= r + 1; k++) {
                        xlo[k] = std::min(xlo[k], du);
                        xhi[k] = std::max(xhi[k], du + 1);
                    }
                }
            q0.resize(nv);
            off.resize(nv);
            long long nu = 0;
            bool fits = nv <= ph;
            for (int r = 0; r < nv && fits; r++) {
                if (xlo[r] > xhi[r]) {  // a row no corner reads (adjacent tile pixels jumped
                    q0[r] = 0;          // 3+ panorama rows near a pole): no units, no arithmetic
                    off[r] = (int)nu;   // on the untouched INT32_MAX / INT32_MIN bounds
                    continue;
                }
                fits = xhi[r] - xlo[r] + 1 <= pw / 2;
                long long a = floor_div(rx + xlo[r], 4), b = floor_div(rx + xhi[r] + 4, 4);
                if (align > 1 && pw % (4 * align) == 0) {  // whole aligned groups of units
                    a = floor_div(a, align) * align;
                    b = floor_div(b + align - 1, align) * align;
                }
                q0[r] = (int)a;
                off[r] = (int)nu;
                nu += b - a;
            }
            WarpPatch P{};
            P.tile = tile; P.X0 = X0; P.Y0 = Y0;
            P.wide = (!fits || nu > cap) ? 1 : 0;
            P.uoff = (int)units.size();
            P.units = P.wide ? 0 : (int)nu;
            if (!P.wide)
                for (int r = 0; r < nv; r++) {
                    const int row = std::min(vmin + r, ph - 1);
                    const int n = (r + 1 < nv ? off[r + 1] : (int)nu) - off[r];
                    for (int u = 0; u < n; u++) {
                        const int col = (int)((((4LL * (q0[r] + u)) % pw) + pw) % pw);
                        units.push_back(((uint32_t)row * (uint32_t)pw + (uint32_t)col) * 4u);
                    }
                }
            for (int Y = Y0; Y < Y1; Y++)
                for (int X = X0; X < X1; X++) {
                    const long long i = (long long)Y * g.w + X;
                    const uint32_t m = wxy[i];
                    const int x0 = (int)(m & 0xFFFFu), y0 = (int)(m >> 16);
                    if (P.wide) {  // k_warp_local's global form: index | x1 != x0 | y1 != y0
                        loc[i] = (uint32_t)(y0 * pw + x0) | (x0 < pw - 1 ? 1u << 31 : 0u) |
                                 (y0 < ph - 1 ? 1u << 30 : 0u);
                    } else {
                        const int r = y0 - vmin;
                        const long long xf = rx + wrap_du_h(x0 - rx, pw);  // unwrapped column
                        const uint32_t lt = (uint32_t)(4LL * (off[r] - q0[r]) + xf);
                        const uint32_t lb = (uint32_t)(4LL * (off[r + 1] - q0[r + 1]) + xf);
                        loc[i] = lt | lb << 16;
                    }
                }
            patches.push_back(P);
        }
}

// The RGB warp's texel taps (row f4 / a18): the GL camera ray of pixel centre (i, r)
// (SaveCubeMap, Main.cpp:246-269) -> the exact sphere texcoord (fs_perspective.txt:67-73) ->
// GL_LINEAR + GL_REPEAT corners and weights, in double with glibc atan2/sqrt/fmod as the oracle
// (pfo_warp_rgb) evaluates them; once per layout and panorama size.
void rgb_taps_host(const RgbCam& cam, int W, int H, int pw, int ph, RgbTap* taps)
{
    host_rows(H, [&](int ra, int rb) {
        for (int r = ra; r < rb; r++)
            for (int i = 0; i < W; i++) {
                const double xn = 2.0 * (i + 0.5) / W - 1.0, yn = 1.0 - 2.0 * (r + 0.5) / H;
                double d[3];
                for (int k = 0; k < 3; k++)
                    d[k] = cam.f[k] + cam.s[k] * (xn * cam.tx) + cam.u[k] * (yn * cam.ty);
                double az = fmod(atan2(d[1], d[0]), 2 * PF_MYPI);
                if (az < 0) az += 2 * PF_MYPI;
                const double zen = atan2(sqrt(d[0] * d[0] + d[1] * d[1]), d[2]);
                const float uu = (float)(az / (2 * PF_MYPI)), vv = (float)(zen / PF_MYPI);
                const float sx = uu * (float)pw - 0.5f, sy = vv * (float)ph - 0.5f;
                const int ix = (int)floorf(sx), iy = (int)floorf(sy);
                RgbTap t;
                t.ax = sx - (float)ix;
                t.ay = sy - (float)iy;
                const int ix0 = ((ix % pw) + pw) % pw, ix1 = (((ix + 1) % pw) + pw) % pw;
                const int iy0 = ((iy % ph) + ph) % ph, iy1 = (((iy + 1) % ph) + ph) % ph;
                t.x0y0 = (uint32_t)ix0 | ((uint32_t)iy0 << 16);
                t.x1y1 = (uint32_t)ix1 | ((uint32_t)iy1 << 16);
                taps[(long long)r * W + i] = t;
            }
    });
}

__device__ __forceinline__ int patch_pixel(const WarpPatch& P, const TileGeom& g, int t, int k,
                                           int& i)
{  // thread t, slot k -> tile pixel index i; returns 0 outside the tile.  A thread owns kPx
   // consecutive pixels of one patch row (one 16-B store per panorama), a wave 8 whole rows.
#if PF_WARP_ROWPX
    static_assert(kPx == 4 && kPatch == 32, "4 pixels per thread, 8 threads per patch row");
    const int X = P.X0 + 4 * (t & 7) + k, Y = P.Y0 + (t >> 3);
#else  // a block covers kWB/kPatch whole rows per slot
    const int X = P.X0 + (t & (kPatch - 1)), Y = P.Y0 + t / kPatch + k * (kWB / kPatch);
#endif
    i = Y * g.w + X;
    return X < g.w && Y < g.h;
}

__device__ __forceinline__ int wrap_du(int d, int pw)
{
    if (d > pw / 2) d -= pw;
    if (d < -(pw / 2)) d += pw;
    return d;
}

// Pass 2: per patch the azimuth-unwrapped footprint box of all its corners (+1 row/column).
__global__ void __launch_bounds__(kWB) k_patch_box(const TileGeom* __restrict__ geom,
                                                   WarpPatch* __restrict__ patches, int pw,
                                                   const uint32_t* __restrict__ wxy)
{
    __shared__ int red[4];
    WarpPatch P = patches[blockIdx.x];
    const TileGeom& g = geom[P.tile];
    const int t = threadIdx.x;
    const int ref = (int)(wxy[g.pix_off + P.Y0 * g.w + P.X0] & 0xFFFFu);
    if (t == 0) { red[0] = INT32_MAX; red[1] = INT32_MIN; red[2] = INT32_MAX; red[3] = INT32_MIN; }
    __syncthreads();
    int umin = INT32_MAX, umax = INT32_MIN, ymin = INT32_MAX, ymax = INT32_MIN;
#pragma unroll
    for (int k = 0; k < kPx; k++) {
        int i;
        if (!patch_pixel(P, g, t, k, i)) continue;
        const uint32_t m = wxy[g.pix_off + i];
        const int du = wrap_du((int)(m & 0xFFFFu) - ref, pw), y = (int)(m >> 16);
        umin = min(umin, du); umax = max(umax, du);
        ymin = min(ymin, y); ymax = max(ymax, y);
    }
    atomicMin(&red[0], umin); atomicMax(&red[1], umax);
    atomicMin(&red[2], ymin); atomicMax(&red[3], ymax);
    __syncthreads();
    if (t == 0) {
        int gx0 = ref + red[0];
        gx0 = gx0 < 0 ? gx0 + pw : (gx0 >= pw ? gx0 - pw : gx0);
        int bw = red[1] - red[0] + 2;
        if (PF_WARP_V4 && (pw & 3) == 0) {  // 16-B staging loads: origin and width in quads
            const int a = gx0 & 3;
            gx0 -= a;
            bw = (bw + a + 3) & ~3;
        }
        P.gx0 = gx0;
        P.gy0 = red[2];
        P.bw = bw;
        P.bh = red[3] - red[2] + 2;
        P.wide = (P.bw * P.bh > kCap || P.bw > pw / 2) ? 1 : 0;
        patches[blockIdx.x] = P;
    }
}

// Pass 3: per tile pixel the corner index inside its patch's box (or, for a wide patch, the
// global index | (x1 != x0) << 31 | (y1 != y0) << 30).  In place over wxy.
__global__ void __launch_bounds__(kWB) k_warp_local(const TileGeom* __restrict__ geom,
                                                    const WarpPatch* __restrict__ patches,
                                                    int pw, int ph, uint32_t* __restrict__ wxy)
{
    const WarpPatch P = patches[blockIdx.x];
    const TileGeom& g = geom[P.tile];
    const int t = threadIdx.x;
#pragma unroll
    for (int k = 0; k < kPx; k++) {
        int i;
        if (!patch_pixel(P, g, t, k, i)) continue;
        const uint32_t m = wxy[g.pix_off + i];
        const int x0 = (int)(m & 0xFFFFu), y0 = (int)(m >> 16);
        uint32_t o;
        if (P.wide) {
            o = (uint32_t)(y0 * pw + x0) | (x0 < pw - 1 ? 1u << 31 : 0u) |
                (y0 < ph - 1 ? 1u << 30 : 0u);
        } else {
            int d = x0 - P.gx0;
            if (d < 0) d += pw;
            o = (uint32_t)((y0 - P.gy0) * P.bw + d);
        }
        wxy[g.pix_off + i] = o;
    }
}

// Per-panorama response of one tile with its noise key mix32(seed), staged in LDS at block start
// (a scalar load per panorama inside the loop would expose its latency on lgkmcnt with the LDS
// reads).  The seed is unique per (panorama, layout-wide tile): pf_synth.responses folds the tile
// index in, so a shard's sub-layout draws the same noise as the whole layout.
struct RespK {
    float alpha, kappa, beta, sigma;
    uint32_t key, pad[3];
};

__device__ __forceinline__ RespK resp_key(const Resp* __restrict__ resp, int b, int ntiles,
                                          int tile)
{
    RespK k{};
    if (resp) {
        const Resp r = resp[(long long)b * ntiles + tile];
        k.alpha = r.alpha; k.kappa = r.kappa; k.beta = r.beta; k.sigma = r.sigma;
        k.key = mix32(r.seed);
    }
    return k;
}

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 pk_add_clamp01(f2 a, f2 b)
{  // v_pk_add_f32 with the output clamp: both lanes to [0, 1] as the reference-style
   // `if (t < 0) t = 0; else if (t > 1) t = 1` (t is finite and never -0: beta != 0)
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 clamp" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// The noise draw of pfo_hash32: hp = mix32(pixel) is per pixel (hoisted out of the panorama
// loop), key = mix32(seed) per panorama, and one full-rate 24x24-bit multiply mixes them.  Returns
// h >> 8 as a float; the caller forms nz = u*2 - 1 (u = (h >> 8) * 2^-24) as fma(., 2^-23, -1),
// exact because the product is a power-of-two scaling of an integer < 2^24.
__device__ __forceinline__ float noise_top24(uint32_t hp, uint32_t key)
{
    const uint32_t h = ((hp ^ key) & 0xFFFFFFu) * 0x9E3779u;
    return (float)(h >> 8);
}

__device__ __forceinline__ float add_f32(float a, float b)
{  // a scalar v_add_f32: keeps the SLP vectoriser from re-pairing lane sums into packed adds
   // (which costs a v_mov per operand to rebuild the register pairs)
    float r;
    asm("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// Bilinear sample in the reference's operand order, no contraction: P = (c00, c01) * (1-fx, fx)
// and Q = (c10, c11) * (1-fx, fx) are one packed multiply each, top/bot their lane sums,
// v = top*(1-fy) + bot*fy with the two products as one more packed multiply.
__device__ __forceinline__ float bilinear(f2 c0, f2 c1, f2 wx, f2 wy)
{
    const f2 p = c0 * wx, q = c1 * wx;
    const f2 tb = f2{add_f32(p.x, p.y), add_f32(q.x, q.y)} * wy;
    return add_f32(tb.x, tb.y);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes)
{  // raw buffer descriptor (wave-uniform inputs): 32-bit byte offsets, range-checked
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

static constexpr int kLPx = PF_WARP_WAVEBOX ? 4 : kPx;  // pixels per lane in the main kernel
struct WarpLanes {  // one thread's kLPx pixels, all panorama-invariant
    uint32_t la[kLPx];  // LDS float index of corner (x0, y0) in the parity-interleaved box (x2)
    uint32_t oo[kLPx];  // byte offset of the pixel inside one panorama's tile block; past the
                        // block (a dropped buffer store) for lanes outside the tile
    uint32_t hp[kLPx];  // mix32(pixel index): the per-pixel half of the noise hash
    f2 wx[kLPx], wy[kLPx];  // (1-fx, fx), (1-fy, fy)
    bool ok[kLPx];
    bool full;  // the kPx pixels are inside the tile and contiguous (one channel): 16-B store
    // XPOSE: oo[] are the byte offsets of the lane's 4 pixels AFTER the transpose (row
    // 2*wave + (l>>3 & 1) + 8*(l>>4), columns 4*(l&7)..+3 of the patch); full = all inside,
    // one channel, 16-B aligned
};

// LDS-staged interpolation of kNB panoramas for a box of at most NS*256 staging units (floats,
// or with V4 column quads: 16-B loads of a box whose origin and width are whole quads, which
// k_patch_box guarantees when pw % 4 == 0).  The box is double-buffered with the two parities
// interleaved (element e of parity PA at box[2e + PA]), so a pixel's c00/c01 (and c10/c11) are
// one ds_read2_b32 with immediate offsets in both parities.  Every staging load is issued
// unconditionally (slots past the box reload a valid unit, panoramas past the chunk reload the
// last one), so the loads for panorama q+2 go out before panorama q is interpolated and the wait
// for panorama q+1's loads -- an in-order vmcnt -- never covers them.  A thread's four pixels
// are consecutive in one tile row: one 16-B store per panorama when they are all inside.
#ifndef PF_WARP_MASKU
// 1: staging slots past a patch's footprint issue no load (exec-masked lanes) instead of
// reloading a valid unit.  Measured (round 5, two alternating rounds, serial C3 steps): the
// depth warp 0.510-0.516 ms against 0.501-0.502 unmasked; the RGB warp 0.668 ms against
// 0.594-0.610 (the masks push it to 15 spilled VGPRs).  Off.
#define PF_WARP_MASKU 0
#endif
#ifndef PF_RGB_MASKU
#define PF_RGB_MASKU 0  // the same in the RGB warp
#endif
typedef uint32_t u4v __attribute__((ext_vector_type(4)));
#if !PF_WARP_WAVEBOX  // the block form (default)
template <int NS, bool RESP, bool V4, bool RAG = false>
__device__ __forceinline__ void warp_staged(float* box, float* xbuf, const RespK* rk,
                                            const WarpPatch& P,
                                            int t, const WarpLanes& W,
                                            const float* __restrict__ pano, int pw, int ph,
                                            long long pstride, float* __restrict__ tiles,
                                            long long tstride, int bbeg, int nb,
                                            const uint32_t* __restrict__ unit_tbl = nullptr)
{
    static_assert(!RAG || (V4 && PF_WARP_SPLIT), "ragged footprints: 16-B units, split parities");
    constexpr int U = V4 ? 4 : 1;  // floats per staging unit
    const int bw2 = 2 * P.bw, bwu = RAG ? 1 : P.bw / U, units = RAG ? P.units : bwu * P.bh;
    uint32_t goff[NS];  // unit e = t + 256*s of the box -> panorama byte offset
    bool live[NS];      // PF_WARP_MASKU: slots past the box load nothing (exec-masked lanes)
#pragma unroll
    for (int s = 0; s < NS; s++) {
        int e = t + s * kWB;
        live[s] = e < units;
        e = e < units ? e : units - 1;
        if constexpr (RAG) {
            goff[s] = unit_tbl[P.uoff + e];
        } else {
            const int r = e / bwu, c = (e - r * bwu) * U;
            int row = P.gy0 + r;
            row = row < ph ? row : ph - 1;
            int col = P.gx0 + c;
            col = col < pw ? col : col - pw;
            goff[s] = (uint32_t)(row * pw + col) * 4u;
        }
    }
    constexpr int D = PF_WARP_PFD;  // prefetch depth: panorama j is staged in stg[j % D]
    float stg[D][NS][U];
    const uint32_t pbytes = (uint32_t)(pstride * 4);
    auto fetch = [&](float (*dst)[U], int q) {
        const auto pr = rsrc(pano + (long long)(bbeg + (q < nb ? q : nb - 1)) * pstride, pbytes);
#pragma unroll
        for (int s = 0; s < NS; s++) {
            if constexpr (PF_WARP_DIAG == 2) {
                for (int j = 0; j < U; j++) dst[s][j] = (float)(goff[s] & 1023u) * 1e-3f;
            } else if constexpr (V4) {
                if (!PF_WARP_MASKU || live[s]) {
                    const u4v v = __builtin_amdgcn_raw_buffer_load_b128(pr, (int)goff[s], 0, 0);
#pragma unroll
                    for (int j = 0; j < 4; j++) dst[s][j] = __uint_as_float(v[j]);
                }
            } else {
                dst[s][0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(pr, (int)goff[s], 0, 0));
            }
        }
    };
    auto put = [&](int pa, const float (*src)[U]) {
#pragma unroll
        for (int s = 0; s < NS; s++)
#pragma unroll
            for (int j = 0; j < U; j++) {
                if constexpr (PF_WARP_SPLIT) box[pa * kCap + (t + s * kWB) * U + j] = src[s][j];
                else box[2 * ((t + s * kWB) * U + j) + pa] = src[s][j];
            }
    };
    auto iter = [&](auto parity, auto slot, int q) {
        constexpr int PA = decltype(parity)::value, SL = decltype(slot)::value;  // q%2, q%D
        fetch(stg[SL], q + D);  // panorama q was put into parity PA last iteration: reuse stg[SL]
        const float* L = PF_WARP_SPLIT ? box + PA * kCap : box + PA;
        const int b = bbeg + q;
        const auto orr = rsrc(tiles + b * tstride, (uint32_t)(tstride * 4));
        f2 al{}, ka{}, be{}, si{};
        uint32_t key = 0;
        if (RESP) {
            const RespK r = rk[q];
            al = f2{r.alpha, r.alpha}; ka = f2{r.kappa, r.kappa};
            be = f2{r.beta, r.beta}; si = f2{r.sigma, r.sigma};
            key = r.key;
        }
        float out[kPx];
#pragma unroll
        for (int k = 0; k < kPx; k += 2) {
            f2 v;
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const float* c = L + (RAG ? (W.la[k + j] & 0xFFFFu) : W.la[k + j]);
                if constexpr (RAG) {  // the bottom pair sits on its own packed row
                    const float* c2 = L + (W.la[k + j] >> 16);
                    v[j] = bilinear(f2{c[0], c[1]}, f2{c2[0], c2[1]}, W.wx[k + j], W.wy[k + j]);
                } else if constexpr (PF_WARP_SPLIT)
                    v[j] = bilinear(f2{c[0], c[1]}, f2{c[P.bw], c[P.bw + 1]}, W.wx[k + j],
                                    W.wy[k + j]);
                else
                    v[j] = bilinear(f2{c[0], c[2]}, f2{c[bw2], c[bw2 + 2]}, W.wx[k + j],
                                    W.wy[k + j]);
            }
            if (RESP) {
                const f2 u = f2{noise_top24(W.hp[k], key), noise_top24(W.hp[k + 1], key)};
                const f2 nz = __builtin_elementwise_fma(u, f2{0x1p-23f, 0x1p-23f},
                                                        f2{-1.0f, -1.0f});
                f2 tt = al * v;
                tt = tt + (ka * v) * v;
                tt = tt + be;
                v = pk_add_clamp01(tt, si * nz);
            }
            out[k] = v[0];
            out[k + 1] = v[1];
        }
        if constexpr (PF_WARP_XPOSE) {  // wave-local transpose through LDS (in order per wave)
            float* xt = xbuf + (t >> 6) * (kPx * 64);
#pragma unroll
            for (int k = 0; k < kPx; k++) xt[k * 64 + (t & 63)] = out[k];
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            const float4 r = *reinterpret_cast<const float4*>(xt + 4 * (t & 63));
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            out[0] = r.x; out[1] = r.y; out[2] = r.z; out[3] = r.w;
        }
        if (PF_WARP_DIAG == 1 && out[0] != -12345.0f) {
        } else if (kPx >= 4 && W.full) {
            const u4v o = {__float_as_uint(out[0]), __float_as_uint(out[1]),
                           __float_as_uint(out[2 % kPx]), __float_as_uint(out[3 % kPx])};
            __builtin_amdgcn_raw_buffer_store_b128(o, orr, (int)W.oo[0], 0, PF_WARP_STPOL);
        } else {
#pragma unroll
            for (int k = 0; k < kPx; k++)
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(out[k]), orr, (int)W.oo[k],
                                                      0, PF_WARP_STPOL);
        }
        put(1 - PA, stg[(SL + 1) % D]);  // panorama q+1 (a duplicate past the chunk: unread)
        __syncthreads();
    };
#pragma unroll
    for (int j = 0; j < D; j++) fetch(stg[j], j);
    put(0, stg[0]);
    __syncthreads();
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2 % D>;
    if constexpr (D == 2) {
        for (int q = 0; q < nb; q += 2) {
            iter(I0{}, I0{}, q);
            if (q + 1 < nb) iter(I1{}, I1{}, q + 1);
        }
    } else {  // D == 3: parity x slot repeats every 6 panoramas
        static_assert(D == 3, "prefetch depth 2 or 3");
        for (int q = 0; q < nb; q += 6) {
            iter(I0{}, I0{}, q);
            if (q + 1 < nb) iter(I1{}, I1{}, q + 1);
            if (q + 2 < nb) iter(I0{}, I2{}, q + 2);
            if (q + 3 < nb) iter(I1{}, I0{}, q + 3);
            if (q + 4 < nb) iter(I0{}, I1{}, q + 4);
            if (q + 5 < nb) iter(I1{}, I2{}, q + 5);
        }
    }
}

#ifndef PF_WARP_DMA
// 1: ragged footprints of <= 2 units per thread are staged by LDS-DMA (global_load_lds_dwordx4:
// each 16-B unit lands in LDS with no VGPR round trip and no ds_write), in three LDS buffers with
// two panoramas in flight, counted vmcnt waits and raw barriers
#define PF_WARP_DMA 0
#endif
#if PF_WARP_DMA
typedef __attribute__((address_space(1))) const void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;
template <int NS, bool RESP>
__device__ __forceinline__ void warp_dma(float* box, const RespK* rk, const WarpPatch& P, int t,
                                         const WarpLanes& W, const float* __restrict__ pano,
                                         long long pstride, float* __restrict__ tiles,
                                         long long tstride, int bbeg, int nb,
                                         const uint32_t* __restrict__ unit_tbl)
{
    constexpr int BUF = NS * kWB * 4;  // floats per buffer: unit e at [4e, 4e + 4)
    static_assert(3 * BUF <= 2 * kCap, "three buffers fit the box");
    static_assert(!PF_WARP_ROWPX && !PF_WARP_XPOSE, "kPx tile stores per panorama");
    const int units = P.units;
    uint32_t gofl[NS];  // float offset (in one panorama) of unit t + s*kWB
#pragma unroll
    for (int s = 0; s < NS; s++) {
        const int e = t + s * kWB;
        gofl[s] = unit_tbl[P.uoff + (e < units ? e : units - 1)] >> 2;
    }
    const int wv = t >> 6;
    auto dma = [&](int buf, int q) {
        const float* pp = pano + (long long)(bbeg + (q < nb ? q : nb - 1)) * pstride;
#pragma unroll
        for (int s = 0; s < NS; s++)  // wave-uniform destination, lane l at +16 l bytes
            __builtin_amdgcn_global_load_lds((gptr_t)(pp + gofl[s]),
                                             (lptr_t)(box + buf * BUF + (s * kWB + wv * 64) * 4),
                                             16, 0, 0);
    };
    dma(0, 0);
    dma(1, 1);
    for (int q = 0; q < nb; q++) {
        // panorama q's units are in: every VMEM op issued after them is panorama q+1's NS loads
        // and panorama q-1's kPx tile stores (they retire in issue order)
        if (q == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NS) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NS + kPx) : "memory");
        __builtin_amdgcn_s_barrier();  // every wave's units of q landed; q-1's reads are done
        dma((q + 2) % 3, q + 2);       // into the buffer panorama q-1 was read from
        const float* L = box + (q % 3) * BUF;
        const int b = bbeg + q;
        const auto orr = rsrc(tiles + b * tstride, (uint32_t)(tstride * 4));
        f2 al{}, ka{}, be{}, si{};
        uint32_t key = 0;
        if (RESP) {
            const RespK r = rk[q];
            al = f2{r.alpha, r.alpha}; ka = f2{r.kappa, r.kappa};
            be = f2{r.beta, r.beta}; si = f2{r.sigma, r.sigma};
            key = r.key;
        }
        float out[kPx];
#pragma unroll
        for (int k = 0; k < kPx; k += 2) {
            f2 v;
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const float* c = L + (W.la[k + j] & 0xFFFFu);
                const float* c2 = L + (W.la[k + j] >> 16);
                v[j] = bilinear(f2{c[0], c[1]}, f2{c2[0], c2[1]}, W.wx[k + j], W.wy[k + j]);
            }
            if (RESP) {
                const f2 u = f2{noise_top24(W.hp[k], key), noise_top24(W.hp[k + 1], key)};
                const f2 nz = __builtin_elementwise_fma(u, f2{0x1p-23f, 0x1p-23f},
                                                        f2{-1.0f, -1.0f});
                f2 tt = al * v;
                tt = tt + (ka * v) * v;
                tt = tt + be;
                v = pk_add_clamp01(tt, si * nz);
            }
            out[k] = v[0];
            out[k + 1] = v[1];
        }
#pragma unroll
        for (int k = 0; k < kPx; k++)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(out[k]), orr, (int)W.oo[k], 0,
                                                  PF_WARP_STPOL);
    }
    // no LDS-DMA may land after the workgroup ends (the duplicate loads past the chunk)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
#endif

template <int NS, bool V4, bool RAG = false>
__device__ __forceinline__ void warp_staged_sel(bool resp, float* box, float* xbuf,
                                                const RespK* rk,
                                                const WarpPatch& P, int t, const WarpLanes& W,
                                                const float* pano, int pw, int ph,
                                                long long pstride, float* tiles,
                                                long long tstride, int bbeg, int nb,
                                                const uint32_t* unit_tbl = nullptr)
{
    if (resp) warp_staged<NS, true, V4, RAG>(box, xbuf, rk, P, t, W, pano, pw, ph, pstride, tiles,
                                             tstride, bbeg, nb, unit_tbl);
    else warp_staged<NS, false, V4, RAG>(box, xbuf, rk, P, t, W, pano, pw, ph, pstride, tiles,
                                         tstride, bbeg, nb, unit_tbl);
}

#ifndef PF_WARP_WPE
#define PF_WARP_WPE 1   // amdgpu_waves_per_eu minimum (occupancy target for the register budget)
#endif
__global__ void __launch_bounds__(kWB) __attribute__((amdgpu_waves_per_eu(PF_WARP_WPE)))
k_warp_depth(const TileGeom* __restrict__ geom,
                                                    int ntiles,
                                                    const WarpPatch* __restrict__ patches,
                                                    const uint32_t* __restrict__ unit_tbl,
                                                    int npatch, const uint32_t* __restrict__ wloc,
                                                    const float2* __restrict__ wfxy,
                                                    const float* __restrict__ pano, int pw,
                                                    int ph, long long pstride,
                                                    const Resp* __restrict__ resp,
                                                    float* __restrict__ tiles,
                                                    long long tstride, int batch)
{
    // one LDS object: the staging box, then the per-panorama response keys (a second __shared__
    // object beside an LDS-DMA target makes hipcc wait vmcnt(0) before every box read)
    __shared__ float box[2 * kCap + kNB * (int)(sizeof(RespK) / sizeof(float))];
    // XCD-contiguous runs of patches; the host sorts the patches by panorama footprint, so the
    // blocks resident on one XCD stage overlapping boxes and re-read each other's lines from L2
    const unsigned lb = xcd_remap(blockIdx.x, gridDim.x);
    const int pid = (int)(lb % (unsigned)npatch);
    const int chunk = (int)(lb / (unsigned)npatch);
    const WarpPatch P = patches[pid];
    const TileGeom& g = geom[P.tile];
    const int t = threadIdx.x;
    const int bbeg = chunk * kNB;
    const int nb = min(kNB, batch - bbeg);

    WarpLanes W;
#pragma unroll
    for (int k = 0; k < kPx; k++) {
        int i;
        W.ok[k] = patch_pixel(P, g, t, k, i);
        W.la[k] = 0; W.wx[k] = f2{1.0f, 0.0f}; W.wy[k] = f2{1.0f, 0.0f};
        W.hp[k] = mix32((uint32_t)i);
        W.oo[k] = W.ok[k] ? (uint32_t)(g.off + (long long)i * g.c) * 4u : 0xFFFFFFF0u;
        if (W.ok[k]) {
            W.la[k] = wloc[g.pix_off + i];
            const float2 f = wfxy[g.pix_off + i];
            W.wx[k] = f2{1.0f - f.x, f.x};
            W.wy[k] = f2{1.0f - f.y, f.y};
        }
    }

    if (P.wide) {  // footprint too large for LDS (near a pole): direct corner gathers
        for (int q = 0; q < nb; q++) {
            const int b = bbeg + q;
            const float* pp = pano + b * pstride;
            const RespK r = resp_key(resp, b, ntiles, P.tile);
            float* out = tiles + b * tstride;
#pragma unroll
            for (int k = 0; k < kPx; k++) {
                if (!W.ok[k]) continue;
                const uint32_t o00 = W.la[k] & 0x3FFFFFFFu, dx = W.la[k] >> 31;
                const uint32_t o10 = o00 + (((W.la[k] >> 30) & 1u) ? (uint32_t)pw : 0u);
                float v = bilinear(f2{pp[o00], pp[o00 + dx]}, f2{pp[o10], pp[o10 + dx]},
                                   W.wx[k], W.wy[k]);
                if (resp) {
                    const float nz = __builtin_fmaf(noise_top24(W.hp[k], r.key), 0x1p-23f, -1.0f);
                    float tt = r.alpha * v;
                    tt = tt + (r.kappa * v) * v;
                    tt = tt + r.beta;
                    tt = tt + r.sigma * nz;
                    v = tt < 0.0f ? 0.0f : (tt > 1.0f ? 1.0f : tt);
                }
                out[W.oo[k] >> 2] = v;
            }
        }
        return;
    }

    W.full = PF_WARP_ROWPX && W.ok[0] && W.ok[kPx - 1] && g.c == 1;
#if PF_WARP_XPOSE
    static_assert(kPx == 4 && kPatch == 32 && !PF_WARP_ROWPX, "transpose: 8 rows x 32 per wave");
    __shared__ float xbuf[kWB * kPx];
    {
        const int l = t & 63, rr = l >> 3;
        const int Y = P.Y0 + 2 * (t >> 6) + (rr & 1) + 8 * (rr >> 1), X = P.X0 + 4 * (l & 7);
        bool all = Y < g.h && g.c == 1;
#pragma unroll
        for (int j = 0; j < kPx; j++) {
            const bool in = Y < g.h && X + j < g.w;
            all = all && in;
            W.oo[j] = in ? (uint32_t)(g.off + ((long long)Y * g.w + X + j) * g.c) * 4u : 0xFFFFFFF0u;
        }
        W.full = all && (W.oo[0] & 15u) == 0;
    }
#else
    float* xbuf = nullptr;
#endif
#pragma unroll
    for (int k = 0; k < kPx; k++) W.la[k] *= PF_WARP_SPLIT ? 1 : 2;  // parity-interleaved box
    RespK* const rk = reinterpret_cast<RespK*>(box + 2 * kCap);  // published by the first barrier
    if (t < nb) rk[t] = resp_key(resp, bbeg + t, ntiles, P.tile);
    const bool rs = resp != nullptr;
    if (PF_WARP_V4 && PF_WARP_SPLIT && P.units > 0) {  // ragged footprint (warp_patches_host)
        const int nq = (P.units + kWB - 1) / kWB;  // uniform: 16-B loads per thread
#if PF_WARP_DMA
        if (nq <= 2) {
            if (nq <= 1) {
                if (rs) warp_dma<1, true>(box, rk, P, t, W, pano, pstride, tiles, tstride, bbeg, nb, unit_tbl);
                else warp_dma<1, false>(box, rk, P, t, W, pano, pstride, tiles, tstride, bbeg, nb, unit_tbl);
            } else {
                if (rs) warp_dma<2, true>(box, rk, P, t, W, pano, pstride, tiles, tstride, bbeg, nb, unit_tbl);
                else warp_dma<2, false>(box, rk, P, t, W, pano, pstride, tiles, tstride, bbeg, nb, unit_tbl);
            }
        } else
#endif
        if (nq <= 1) warp_staged_sel<1, true, true>(rs, box, xbuf, rk, P, t, W, pano, pw, ph, pstride,
                                                    tiles, tstride, bbeg, nb, unit_tbl);
        else if (nq <= 2) warp_staged_sel<2, true, true>(rs, box, xbuf, rk, P, t, W, pano, pw, ph,
                                                         pstride, tiles, tstride, bbeg, nb, unit_tbl);
        else warp_staged_sel<kSlots / 4, true, true>(rs, box, xbuf, rk, P, t, W, pano, pw, ph,
                                                     pstride, tiles, tstride, bbeg, nb, unit_tbl);
    } else if (PF_WARP_V4 && (pw & 3) == 0) {  // quad-aligned boxes (k_patch_box): 16-B staging loads
        const int nq = (P.bw * P.bh / 4 + kWB - 1) / kWB;  // uniform: loads per thread
        if (nq <= 1) warp_staged_sel<1, true>(rs, box, xbuf, rk, P, t, W, pano, pw, ph, pstride, tiles,
                                              tstride, bbeg, nb);
        else if (nq <= 2) warp_staged_sel<2, true>(rs, box, xbuf, rk, P, t, W, pano, pw, ph, pstride,
                                                   tiles, tstride, bbeg, nb);
        else warp_staged_sel<kSlots / 4, true>(rs, box, xbuf, rk, P, t, W, pano, pw, ph, pstride,
                                               tiles, tstride, bbeg, nb);
    } else {
        const int ns = (P.bw * P.bh + kWB - 1) / kWB;  // uniform: staging loads per thread
        // staging slots never exceed kSlots: slot s writes LDS unit t + s*kWB < kCap
        constexpr int N1 = kSlots < 4 ? kSlots : 4, N2 = kSlots < 8 ? kSlots : 8;
        if (ns <= N1) warp_staged_sel<N1, false>(rs, box, xbuf, rk, P, t, W, pano, pw, ph, pstride,
                                                 tiles, tstride, bbeg, nb);
        else if (ns <= N2) warp_staged_sel<N2, false>(rs, box, xbuf, rk, P, t, W, pano, pw, ph, pstride,
                                                      tiles, tstride, bbeg, nb);
        else warp_staged_sel<kSlots, false>(rs, box, xbuf, rk, P, t, W, pano, pw, ph, pstride, tiles,
                                            tstride, bbeg, nb);
    }
}

#endif  // !PF_WARP_WAVEBOX

#if PF_WARP_WAVEBOX
__device__ __forceinline__ void wave_sync()
{  // a wave's LDS operations complete in order; this only keeps the compiler from moving them
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One wave, one 32x8 patch: the warp_staged loop with the box in the wave's own LDS region
// (kCap floats per parity) and wave_sync() where the block form has __syncthreads().
template <int NS, bool RESP, bool V4>
__device__ __forceinline__ void warp_wave(float* box, const RespK* rk, const WarpPatch& P, int l,
                                          const WarpLanes& W, const float* __restrict__ pano,
                                          int pw, int ph, long long pstride,
                                          float* __restrict__ tiles, long long tstride, int bbeg,
                                          int nb)
{
    constexpr int U = V4 ? 4 : 1;
    static_assert(NS * 64 * U <= kCap, "staging slots stay inside the wave's box");
    const int bwu = P.bw / U, units = bwu * P.bh;
    uint32_t goff[NS];
#pragma unroll
    for (int s = 0; s < NS; s++) {
        int e = l + s * 64;
        e = e < units ? e : units - 1;
        const int r = e / bwu, c = (e - r * bwu) * U;
        int row = P.gy0 + r;
        row = row < ph ? row : ph - 1;
        int col = P.gx0 + c;
        col = col < pw ? col : col - pw;
        goff[s] = (uint32_t)(row * pw + col) * 4u;
    }
    float stg[2][NS][U];
    const uint32_t pbytes = (uint32_t)(pstride * 4);
    auto fetch = [&](float (*dst)[U], int q) {
        const auto pr = rsrc(pano + (long long)(bbeg + (q < nb ? q : nb - 1)) * pstride, pbytes);
#pragma unroll
        for (int s = 0; s < NS; s++) {
            if constexpr (V4) {
                const u4v v = __builtin_amdgcn_raw_buffer_load_b128(pr, (int)goff[s], 0, 0);
#pragma unroll
                for (int j = 0; j < 4; j++) dst[s][j] = __uint_as_float(v[j]);
            } else {
                dst[s][0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(pr, (int)goff[s], 0, 0));
            }
        }
    };
    auto put = [&](int pa, const float (*src)[U]) {
#pragma unroll
        for (int s = 0; s < NS; s++)
#pragma unroll
            for (int j = 0; j < U; j++) box[pa * kCap + (l + s * 64) * U + j] = src[s][j];
    };
    auto iter = [&](auto parity, int q) {
        constexpr int PA = decltype(parity)::value;
        fetch(stg[PA], q + 2);
        const float* L = box + PA * kCap;
        const int b = bbeg + q;
        const auto orr = rsrc(tiles + b * tstride, (uint32_t)(tstride * 4));
        f2 al{}, ka{}, be{}, si{};
        uint32_t key = 0;
        if (RESP) {
            const RespK r = rk[q];
            al = f2{r.alpha, r.alpha}; ka = f2{r.kappa, r.kappa};
            be = f2{r.beta, r.beta}; si = f2{r.sigma, r.sigma};
            key = r.key;
        }
        float out[kLPx];
#pragma unroll
        for (int k = 0; k < kLPx; k += 2) {
            f2 v;
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const float* c = L + W.la[k + j];
                v[j] = bilinear(f2{c[0], c[1]}, f2{c[P.bw], c[P.bw + 1]}, W.wx[k + j], W.wy[k + j]);
            }
            if (RESP) {
                const f2 u = f2{noise_top24(W.hp[k], key), noise_top24(W.hp[k + 1], key)};
                const f2 nz = __builtin_elementwise_fma(u, f2{0x1p-23f, 0x1p-23f},
                                                        f2{-1.0f, -1.0f});
                f2 tt = al * v;
                tt = tt + (ka * v) * v;
                tt = tt + be;
                v = pk_add_clamp01(tt, si * nz);
            }
            out[k] = v[0];
            out[k + 1] = v[1];
        }
#pragma unroll
        for (int k = 0; k < kLPx; k++)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(out[k]), orr, (int)W.oo[k], 0,
                                                  PF_WARP_STPOL);
        put(1 - PA, stg[1 - PA]);  // panorama q+1 (a duplicate past the chunk: unread)
        wave_sync();
    };
    fetch(stg[0], 0);
    fetch(stg[1], 1);
    put(0, stg[0]);
    wave_sync();
    for (int q = 0; q < nb; q += 2) {
        iter(std::integral_constant<int, 0>{}, q);
        if (q + 1 < nb) iter(std::integral_constant<int, 1>{}, q + 1);
    }
}

template <int NS, bool V4>
__device__ __forceinline__ void warp_wave_sel(bool resp, float* box, const RespK* rk,
                                              const WarpPatch& P, int l, const WarpLanes& W,
                                              const float* pano, int pw, int ph, long long pstride,
                                              float* tiles, long long tstride, int bbeg, int nb)
{
    if (resp) warp_wave<NS, true, V4>(box, rk, P, l, W, pano, pw, ph, pstride, tiles, tstride,
                                      bbeg, nb);
    else warp_wave<NS, false, V4>(box, rk, P, l, W, pano, pw, ph, pstride, tiles, tstride, bbeg,
                                  nb);
}

__global__ void __launch_bounds__(kWB) k_warp_wave(const TileGeom* __restrict__ geom, int ntiles,
                                                   const WarpPatch* __restrict__ patches,
                                                   int npatch, const uint32_t* __restrict__ wloc,
                                                   const float2* __restrict__ wfxy,
                                                   const float* __restrict__ pano, int pw, int ph,
                                                   long long pstride, const Resp* __restrict__ resp,
                                                   float* __restrict__ tiles, long long tstride,
                                                   int batch)
{
    __shared__ float boxes[4][2 * kCap];
    __shared__ RespK rks[4][kNB];
    const int npb = (npatch + 3) / 4;
    const unsigned lb = xcd_remap(blockIdx.x, gridDim.x);
    const int pb = (int)(lb % (unsigned)npb), chunk = (int)(lb / (unsigned)npb);
    const int w = (int)(threadIdx.x >> 6), l = (int)(threadIdx.x & 63);
    const int pid = pb * 4 + w;
    if (pid >= npatch) return;  // whole wave; nothing below synchronises across waves
    const WarpPatch P = patches[pid];
    const TileGeom& g = geom[P.tile];
    const int bbeg = chunk * kNB;
    const int nb = min(kNB, batch - bbeg);
    WarpLanes W;
#pragma unroll
    for (int k = 0; k < kLPx; k++) {  // lane l: column l & 31, rows (l >> 5) + 2k of the patch
        const int X = P.X0 + (l & 31), Y = P.Y0 + (l >> 5) + 2 * k;
        const int i = Y * g.w + X;
        W.ok[k] = X < g.w && Y < g.h;
        W.la[k] = 0; W.wx[k] = f2{1.0f, 0.0f}; W.wy[k] = f2{1.0f, 0.0f};
        W.hp[k] = mix32((uint32_t)i);
        W.oo[k] = W.ok[k] ? (uint32_t)(g.off + (long long)i * g.c) * 4u : 0xFFFFFFF0u;
        if (W.ok[k]) {
            W.la[k] = wloc[g.pix_off + i];
            const float2 f = wfxy[g.pix_off + i];
            W.wx[k] = f2{1.0f - f.x, f.x};
            W.wy[k] = f2{1.0f - f.y, f.y};
        }
    }
    if (P.wide) {  // footprint too large for the wave's box: direct corner gathers
        for (int q = 0; q < nb; q++) {
            const int b = bbeg + q;
            const float* pp = pano + b * pstride;
            const RespK r = resp_key(resp, b, ntiles, P.tile);
            float* out = tiles + b * tstride;
#pragma unroll
            for (int k = 0; k < kLPx; k++) {
                if (!W.ok[k]) continue;
                const uint32_t o00 = W.la[k] & 0x3FFFFFFFu, dx = W.la[k] >> 31;
                const uint32_t o10 = o00 + (((W.la[k] >> 30) & 1u) ? (uint32_t)pw : 0u);
                float v = bilinear(f2{pp[o00], pp[o00 + dx]}, f2{pp[o10], pp[o10 + dx]},
                                   W.wx[k], W.wy[k]);
                if (resp) {
                    const float nz = __builtin_fmaf(noise_top24(W.hp[k], r.key), 0x1p-23f, -1.0f);
                    float tt = r.alpha * v;
                    tt = tt + (r.kappa * v) * v;
                    tt = tt + r.beta;
                    tt = tt + r.sigma * nz;
                    v = tt < 0.0f ? 0.0f : (tt > 1.0f ? 1.0f : tt);
                }
                out[W.oo[k] >> 2] = v;
            }
        }
        return;
    }
    RespK* rk = rks[w];
    if (l < nb) rk[l] = resp_key(resp, bbeg + l, ntiles, P.tile);
    wave_sync();
    const bool rs = resp != nullptr;
    float* box = boxes[w];
    if (PF_WARP_V4 && (pw & 3) == 0) {
        const int nq = (P.bw * P.bh / 4 + 63) / 64;  // wave-uniform: 16-B loads per lane
        if (nq <= 1) warp_wave_sel<1, true>(rs, box, rk, P, l, W, pano, pw, ph, pstride, tiles,
                                            tstride, bbeg, nb);
        else if (nq <= 2) warp_wave_sel<2, true>(rs, box, rk, P, l, W, pano, pw, ph, pstride,
                                                 tiles, tstride, bbeg, nb);
        else warp_wave_sel<kCap / 256, true>(rs, box, rk, P, l, W, pano, pw, ph, pstride, tiles,
                                             tstride, bbeg, nb);
    } else {
        const int ns = (P.bw * P.bh + 63) / 64;
        if (ns <= 4) warp_wave_sel<4, false>(rs, box, rk, P, l, W, pano, pw, ph, pstride, tiles,
                                             tstride, bbeg, nb);
        else if (ns <= 8) warp_wave_sel<8, false>(rs, box, rk, P, l, W, pano, pw, ph, pstride,
                                                  tiles, tstride, bbeg, nb);
        else warp_wave_sel<kCap / 64, false>(rs, box, rk, P, l, W, pano, pw, ph, pstride, tiles,
                                             tstride, bbeg, nb);
    }
}
#endif

// ---------------------------------------------------------------------------------------------
void launch_warp_boxes(hipStream_t s, const TileGeom* geom, WarpPatch* patches, int npatch,
                       int pw, int ph, uint32_t* wloc)
{
    hipLaunchKernelGGL(k_patch_box, dim3(npatch), dim3(kWB), 0, s, geom, patches, pw,
                       (const uint32_t*)wloc);
    hipLaunchKernelGGL(k_warp_local, dim3(npatch), dim3(kWB), 0, s, geom,
                       (const WarpPatch*)patches, pw, ph, wloc);
}

int warp_patch_edge() { return kPatch; }
int warp_patch_height() { return kPatchH; }

void launch_warp_depth(hipStream_t s, const TileGeom* geom, int ntiles, const WarpPatch* patches,
                       const uint32_t* unit_tbl,
                       int npatch, const uint32_t* wloc, const float* wfxy, const float* pano,
                       int pw, int ph, long long pstride, const Resp* resp, float* tiles,
                       long long tstride, int batch)
{
#if PF_WARP_WAVEBOX
    const long long n = (long long)((npatch + 3) / 4) * ((batch + kNB - 1) / kNB);
    hipLaunchKernelGGL(k_warp_wave, dim3((unsigned)n), dim3(kWB), 0, s, geom, ntiles, patches,
                       npatch, wloc, (const float2*)wfxy, pano, pw, ph, pstride, resp, tiles,
                       tstride, batch);
#else
    const long long n = (long long)npatch * ((batch + kNB - 1) / kNB);
    hipLaunchKernelGGL(k_warp_depth, dim3((unsigned)n), dim3(kWB), 0, s, geom, ntiles, patches,
                       unit_tbl, npatch, wloc, (const float2*)wfxy, pano, pw, ph, pstride, resp,
                       tiles, tstride, batch);
#endif
}


// =============================================================================================
// E->P RGB warp (a18: SaveCubeMap, Main.cpp:242-326, the GL camera and GL_LINEAR + GL_REPEAT
// sampling of SphereMesh.cpp:74-77), LDS-staged like k_warp_depth.
//
// Per layout and panorama size the host cuts every tile into 64x16-pixel patches and, from the
// taps (rgb_taps_host), gives each patch the byte box of its corners' footprint: rows gy0.. and
// bytes bx0.. of the u8 RGB panorama, the origin rounded down to 16 B and the width up to 16 B,
// so the box is staged with whole 16-B loads (both wrap: GL_REPEAT in u and v).  One block =
// one patch x kNBR panoramas.  Per panorama each thread loads one 16-B unit of the box,
// converts its bytes to floats and writes them to LDS (double-buffered: the loads for panorama
// q+2 are in flight while q is blended); a thread then blends its 4 consecutive pixels of one
// tile row (per channel top = t00*(1-ax) + t01*ax, bottom likewise, v = top*(1-ay) + bot*ay:
// the oracle's fp32 operations in its order), rounds them to u8 and writes the 12 bytes with
// one 12-B store, so a wave writes four 192-B runs of tile rows.  Patches whose box exceeds
// the LDS slot (near the poles) blend from direct byte gathers of the taps.
// =============================================================================================
#ifndef PF_RGB_NB
// round 6 A/B (profiles/r06/ab/rgb_panoramas_per_block.txt): 8 slower, 32 the same
#define PF_RGB_NB 16
#endif
static constexpr int kNBR = PF_RGB_NB;  // panoramas per block

static inline int wrap_signed(int d, int n)
{
    if (d > n / 2) d -= n;
    if (d < -(n / 2)) d += n;
    return d;
}

// Footprint of a patch of nrow rows: per panorama row v (unwrapped from the patch's first
// corner) the x-range [xlo, xhi] of the corners that read it (pixels whose y0 is v or v-1, with
// their x0 and x0 + 1), rounded out to 16-B units of the u8 RGB row.  Returns the unit count.
static inline long long floor_div16(long long x) { return x >= 0 ? x / 16 : -((15 - x) / 16); }

struct RgbFoot {
    int vmin = 0, nv = 0;
    std::vector<int> xlo, xhi, u0, nu, off;  // per row: pixel range, first unit, units, LDS unit
    int units = 0;
};
static int rgb_footprint(const RgbTap* taps, int w, int X0, int X1, int Y0, int Y1, int pw,
                         int ph, int rx, int ry, RgbFoot& F)
{
    int vmin = INT32_MAX, vmax = INT32_MIN;
    for (int Y = Y0; Y < Y1; Y++)
        for (int X = X0; X < X1; X++) {
            const int dv = wrap_signed((int)(taps[(long long)Y * w + X].x0y0 >> 16) - ry, ph);
            vmin = std::min(vmin, dv);
            vmax = std::max(vmax, dv);
        }
    F.vmin = vmin;
    F.nv = vmax - vmin + 2;
    if (F.nv > ph / 2) return INT32_MAX;
    F.xlo.assign(F.nv, INT32_MAX);
    F.xhi.assign(F.nv, INT32_MIN);
    for (int Y = Y0; Y < Y1; Y++)
        for (int X = X0; X < X1; X++) {
            const RgbTap& t = taps[(long long)Y * w + X];
            const int du = wrap_signed((int)(t.x0y0 & 0xFFFFu) - rx, pw);
            const int dv = wrap_signed((int)(t.x0y0 >> 16) - ry, ph) - vmin;
            for (int r = dv; r <= dv + 1; r++) {
                F.xlo[r] = std::min(F.xlo[r], du);
                F.xhi[r] = std::max(F.xhi[r], du + 1);
            }
        }
    F.u0.resize(F.nv);
    F.nu.resize(F.nv);
    F.off.resize(F.nv);
    F.units = 0;
    for (int r = 0; r < F.nv; r++) {
        if (F.xhi[r] - F.xlo[r] + 1 > pw / 2) return INT32_MAX;
        const long long b0 = 3LL * (rx + F.xlo[r]), b1 = 3LL * (rx + F.xhi[r]) + 3;  // unwrapped
        const long long q0 = floor_div16(b0), q1 = floor_div16(b1 + 15);
        F.u0[r] = (int)q0;
        F.nu[r] = (int)(q1 - q0);
        F.off[r] = F.units;
        F.units += F.nu[r];
    }
    return F.units;
}

void rgb_patches_host(const TileGeom& g, int tile, const RgbTap* taps, int pw, int ph,
                      std::vector<RgbPatch>& patches, std::vector<uint32_t>& units,
                      uint32_t* loc, float* wts)
{
    const int rowu = 3 * pw / 16;  // units per panorama row
    for (int Y0 = 0; Y0 < g.h;) {
        // one band of patches of a common height: the tallest (16, 8, .., 1 rows) whose every
        // patch's footprint fits kRgbUnits units; rows that do not fit even alone go "wide"
        int hp = std::min(kRgbPH, g.h - Y0);
        std::vector<RgbFoot> feet;
        for (;; hp = std::max(1, hp / 2)) {
            feet.assign((g.w + kRgbPW - 1) / kRgbPW, RgbFoot{});
            bool fit = true;
            for (int X0 = 0, k = 0; X0 < g.w; X0 += kRgbPW, k++) {
                const RgbTap& t0 = taps[(long long)Y0 * g.w + X0];
                const int n = rgb_footprint(taps, g.w, X0, std::min(g.w, X0 + kRgbPW), Y0, Y0 + hp,
                                            pw, ph, (int)(t0.x0y0 & 0xFFFFu), (int)(t0.x0y0 >> 16),
                                            feet[k]);
                fit = fit && n <= kRgbUnits;
            }
            if (fit || hp == 1) break;
        }
        for (int X0 = 0, k = 0; X0 < g.w; X0 += kRgbPW, k++) {
            const RgbFoot& F = feet[k];
            RgbPatch P{};
            P.tile = tile; P.X0 = X0; P.Y0 = Y0; P.nrow = hp;
            P.wide = F.units > kRgbUnits ? 1 : 0;
            P.units = P.wide ? 1 : F.units;
            const RgbTap& t0 = taps[(long long)Y0 * g.w + X0];
            const int rx = (int)(t0.x0y0 & 0xFFFFu), ry = (int)(t0.x0y0 >> 16);
            const size_t base = units.size();
            units.resize(base + kRgbUnits, 0u);
            if (!P.wide)
                for (int r = 0; r < F.nv; r++) {
                    const int prow = ((ry + F.vmin + r) % ph + ph) % ph;
                    for (int u = 0; u < F.nu[r]; u++) {
                        const int cu = ((F.u0[r] + u) % rowu + rowu) % rowu;
                        units[base + F.off[r] + u] = (uint32_t)prow * (uint32_t)(3 * pw) +
                                                     (uint32_t)(16 * cu);
                    }
                }
            for (int Y = Y0; Y < Y0 + hp; Y++)
                for (int X = X0; X < std::min(g.w, X0 + kRgbPW); X++) {
                    const long long i = (long long)Y * g.w + X;
                    const RgbTap& t = taps[i];
                    uint32_t l = 0;
                    if (!P.wide) {
                        const int du = wrap_signed((int)(t.x0y0 & 0xFFFFu) - rx, pw);
                        const int dv = wrap_signed((int)(t.x0y0 >> 16) - ry, ph) - F.vmin;
                        const long long bx = 3LL * (rx + du);  // unwrapped byte of corner x0
                        const uint32_t lt = (uint32_t)(16 * (F.off[dv] - F.u0[dv]) + bx);
                        const uint32_t lb = (uint32_t)(16 * (F.off[dv + 1] - F.u0[dv + 1]) + bx);
                        l = lt | lb << 16;
                    }
                    loc[i] = l;
                    wts[2 * i] = t.ax;
                    wts[2 * i + 1] = t.ay;
                }
            patches.push_back(P);
        }
        Y0 += hp;
    }
}

__device__ __forceinline__ float lerp_ref(float a, float b, float w)
{  // a * (1 - w) + b * w with separate roundings (the oracle's / GL-restatement order)
    return a * (1.0f - w) + b * w;
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) k_warp_rgb_box(const TileGeom* __restrict__ geom,
                                                      const RgbPatch* __restrict__ patches,
                                                      int npatch,
                                                      const uint32_t* __restrict__ unit_tbl,
                                                      const uint32_t* __restrict__ loc,
                                                      const float2* __restrict__ wts,
                                                      const RgbTap* __restrict__ taps,
                                                      const long long* __restrict__ rgb_off,
                                                      const uint8_t* __restrict__ pano, int pw,
                                                      int ph, long long pstride,
                                                      uint8_t* __restrict__ tiles,
                                                      long long tstride, int batch)
{
    // two parities of kRgbCap bytes (+ one dword: a pixel's last 3-dword read may pass the end)
    __shared__ uint32_t boxw[2 * (kRgbCap / 4) + 4];
    const unsigned lb = xcd_remap(blockIdx.x, gridDim.x);
    const int pid = (int)(lb % (unsigned)npatch);
    const int chunk = (int)(lb / (unsigned)npatch);
    const RgbPatch P = patches[pid];
    const TileGeom& g = geom[P.tile];
    const int t = threadIdx.x;
    constexpr int kRL = kRgbPW / 4;  // lanes per patch row
    const int X = P.X0 + 4 * (t % kRL), Y = P.Y0 + t / kRL;
    const int bbeg = chunk * kNBR, nb = min(kNBR, batch - bbeg);
    const bool rowok = t / kRL < P.nrow && Y < g.h;
    bool ok[4];
    uint32_t la[4];
    float ax[4], ay[4];
    long long pix[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        ok[k] = rowok && X + k < g.w;
        pix[k] = (long long)Y * g.w + X + k;
        la[k] = 0; ax[k] = 0.0f; ay[k] = 0.0f;
        if (ok[k]) {
            la[k] = loc[g.pix_off + pix[k]];
            const float2 w = wts[g.pix_off + pix[k]];
            ax[k] = w.x;
            ay[k] = w.y;
        }
    }
    const long long toff = rgb_off[P.tile];
    // byte offset of the lane's first pixel inside one panorama's tile block (past the block for
    // lanes outside the tile: the buffer store is then dropped)
    const uint32_t ob = ok[0] ? (uint32_t)(toff + 3 * pix[0]) : 0xFFFFFFF0u;
    const uint32_t tbytes = (uint32_t)tstride;
    const uint32_t pbytes = (uint32_t)pstride;

    auto blend_store = [&](const auto& corner, uint8_t* tb) {
        // corner(k, c) -> the 12 floats c00 RGB, c01 RGB, c10 RGB, c11 RGB of pixel k
        typedef float f2 __attribute__((ext_vector_type(2)));
        float c00[12], c01[12], c10[12], c11[12];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            float c[12];
            corner(k, c);
#pragma unroll
            for (int ch = 0; ch < 3; ch++) {
                c00[3 * k + ch] = c[ch];
                c01[3 * k + ch] = c[3 + ch];
                c10[3 * k + ch] = c[6 + ch];
                c11[3 * k + ch] = c[9 + ch];
            }
        }
        // the 12 values (pixel k, channel ch) at 3k + ch, blended two at a time with packed fp32
        // (v_pk_mul / v_pk_add: per element the same IEEE operations as lerp_ref)
        float v[12];
#pragma unroll
        for (int i = 0; i < 6; i++) {
            const int e0 = 2 * i, e1 = 2 * i + 1;
            const f2 wx = {ax[e0 / 3], ax[e1 / 3]}, wy = {ay[e0 / 3], ay[e1 / 3]};
            const f2 one = {1.0f, 1.0f}, half = {0.5f, 0.5f};
            const f2 mx = one - wx, my = one - wy;
            const f2 top = f2{c00[e0], c00[e1]} * mx + f2{c01[e0], c01[e1]} * wx;
            const f2 bot = f2{c10[e0], c10[e1]} * mx + f2{c11[e0], c11[e1]} * wx;
            const f2 r = (top * my + bot * wy) + half;
            v[e0] = r.x;
            v[e1] = r.y;
        }
        // (int)floorf(v + 0.5f) clamped to [0, 255] (the oracle's u8 rounding), the 12 bytes packed into 3 dwords:
        // v + 0.5 >= 0.5 and, the blend being of values <= 255 with weights summing to 1 under
        // five fp32 roundings, below 255 * (1 + 2^-24)^5 + 0.5 < 256, so the truncating
        // conversion is the clamp and the floor; SDWA writes each result into its byte lane
        uint32_t o[3];
#pragma unroll
        for (int j = 0; j < 3; j++) {
            asm("v_cvt_u32_f32_sdwa %0, %1 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD"
                : "=v"(o[j]) : "v"(v[4 * j]));
            asm("v_cvt_u32_f32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE "
                "src0_sel:DWORD" : "+v"(o[j]) : "v"(v[4 * j + 1]));
            asm("v_cvt_u32_f32_sdwa %0, %1 dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE "
                "src0_sel:DWORD" : "+v"(o[j]) : "v"(v[4 * j + 2]));
            asm("v_cvt_u32_f32_sdwa %0, %1 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE "
                "src0_sel:DWORD" : "+v"(o[j]) : "v"(v[4 * j + 3]));
        }
        const auto orr = rsrc(tb, tbytes);
        if (ok[3]) {
            typedef uint32_t u3v __attribute__((ext_vector_type(3)));
            const u3v ov = {o[0], o[1], o[2]};
            __builtin_amdgcn_raw_buffer_store_b96(ov, orr, (int)ob, 0, 2);
        } else {
#pragma unroll
            for (int e = 0; e < 12; e++)
                if (ok[e / 3])
                    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(o[e / 4] >> (8 * (e % 4))), orr,
                                                         (int)(ob + e), 0, 2);
        }
    };

    if (P.wide) {  // even one row's footprint exceeds the LDS slot: direct byte gathers
        for (int q = 0; q < nb; q++) {
            const uint8_t* pp = pano + (long long)(bbeg + q) * pstride;
            blend_store([&](int k, float* c) {
                const RgbTap tp = ok[k] ? taps[g.pix_off + pix[k]] : RgbTap{0, 0, 0.0f, 0.0f};
                const long long x0 = tp.x0y0 & 0xFFFFu, y0 = tp.x0y0 >> 16;
                const long long x1 = tp.x1y1 & 0xFFFFu, y1 = tp.x1y1 >> 16;
                const long long a[4] = {(y0 * pw + x0) * 3, (y0 * pw + x1) * 3,
                                        (y1 * pw + x0) * 3, (y1 * pw + x1) * 3};
#pragma unroll
                for (int m = 0; m < 4; m++)
#pragma unroll
                    for (int ch = 0; ch < 3; ch++) c[3 * m + ch] = (float)pp[a[m] + ch];
            }, tiles + (long long)(bbeg + q) * tstride);
        }
        return;
    }

    // staging: thread t owns units t (and t + 256 when the footprint has more than 256 units: NU
    // = 2, a block-uniform choice) of the patch's footprint; units past it reload its first unit,
    // so every load is issued unconditionally.  LDS holds the u8 rows as they are (one 16-B
    // store per unit, consecutive lanes on consecutive 16 B: no bank conflicts); a pixel's
    // corner pair is the 6 bytes at its byte offset a, read as the 3 dwords from a & ~3 and
    // aligned with v_alignbyte (round 5: the fp32-widened box of the first version spent 70 % of
    // its LDS cycles in bank conflicts, SQ_LDS_BANK_CONFLICT, profiles/r05/rgb)
    // the 6 bytes R0 G0 B0 R1 G1 B1 at byte offset a of parity L, as floats into c[0..5]: the
    // three dwords from a & ~3 (the lanes of a tile row 3 dwords apart: an odd stride over the
    // banks), aligned with v_alignbyte (two 8-B reads from a & ~7 measured slower, 0.71 ms)
    auto pair6 = [&](const uint32_t* L, uint32_t a, float* c) {
        const uint32_t* w = L + (a >> 2);
        const uint32_t s0 = w[0], s1 = w[1], s2 = w[2], sh = a & 3u;
        const uint32_t lo = __builtin_amdgcn_alignbyte(s1, s0, sh);  // bytes a .. a+3
        const uint32_t hi = __builtin_amdgcn_alignbyte(s2, s1, sh);  // bytes a+4 .. a+7
        c[0] = (float)(lo & 0xFFu);
        c[1] = (float)((lo >> 8) & 0xFFu);
        c[2] = (float)((lo >> 16) & 0xFFu);
        c[3] = (float)(lo >> 24);
        c[4] = (float)(hi & 0xFFu);
        c[5] = (float)((hi >> 8) & 0xFFu);
    };
    auto staged = [&](auto nu) {
        constexpr int NU = decltype(nu)::value;
        uint32_t goff[NU];
#pragma unroll
        for (int u = 0; u < NU; u++) {
            const int e = t + 256 * u;
            goff[u] = unit_tbl[(long long)pid * kRgbUnits + (e < P.units ? e : 0)];
        }
        u4v stg[2][NU];
        bool live[NU];  // PF_RGB_MASKU: units past the footprint load nothing
#pragma unroll
        for (int u = 0; u < NU; u++) live[u] = t + 256 * u < P.units;
        auto fetch = [&](int sl, int q) {
            const auto pr = rsrc(pano + (long long)(bbeg + (q < nb ? q : nb - 1)) * pstride,
                                 pbytes);
#pragma unroll
            for (int u = 0; u < NU; u++)
                if (!PF_RGB_MASKU || live[u])
                    stg[sl][u] = __builtin_amdgcn_raw_buffer_load_b128(pr, (int)goff[u], 0, 0);
        };
        auto put = [&](int pa, const u4v* v) {
#pragma unroll
            for (int u = 0; u < NU; u++)
                *reinterpret_cast<u4v*>(boxw + pa * (kRgbCap / 4) + 4 * (t + 256 * u)) = v[u];
        };
        auto iter = [&](auto parity, int q) {
            constexpr int PA = decltype(parity)::value;
            fetch(PA, q + 2);  // stg[PA] held panorama q, put into parity PA last iteration
            const uint32_t* L = boxw + PA * (kRgbCap / 4);
            blend_store([&](int k, float* c) {
                pair6(L, la[k] & 0xFFFFu, c);
                pair6(L, la[k] >> 16, c + 6);
            }, tiles + (long long)(bbeg + q) * tstride);
            put(1 - PA, stg[1 - PA]);  // panorama q+1 (a duplicate past the chunk: unread)
            __syncthreads();
        };
        fetch(0, 0);
        fetch(1, 1);
        put(0, stg[0]);
        __syncthreads();
        using I0 = std::integral_constant<int, 0>;
        using I1 = std::integral_constant<int, 1>;
        for (int q = 0; q < nb; q += 2) {
            iter(I0{}, q);
            if (q + 1 < nb) iter(I1{}, q + 1);
        }
    };
    static_assert(kRgbUnits <= 512, "two units per thread at most");
    if (P.units <= 256) staged(std::integral_constant<int, 1>{});  // block-uniform
    else staged(std::integral_constant<int, 2>{});
}

void launch_warp_rgb_box(hipStream_t s, const TileGeom* geom, const RgbPatch* patches,
                         int npatch, const uint32_t* units, const uint32_t* loc, const float* wts,
                         const RgbTap* taps, const long long* rgb_off, const uint8_t* pano,
                         int pw, int ph, long long pstride, uint8_t* tiles, long long tstride,
                         int batch)
{
    const unsigned nblk = (unsigned)npatch * (unsigned)((batch + kNBR - 1) / kNBR);
    hipLaunchKernelGGL(k_warp_rgb_box, dim3(nblk), dim3(256), 0, s, geom, patches, npatch, units,
                       loc, (const float2*)wts, taps, rgb_off, pano, pw, ph, pstride, tiles,
                       tstride, batch);
}

}  // namespace pf
