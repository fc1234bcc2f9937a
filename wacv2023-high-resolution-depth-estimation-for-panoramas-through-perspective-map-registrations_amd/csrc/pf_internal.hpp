// pf_internal.hpp -- shared declarations of the panofuse HIP library (host + device).
//
// Numeric contract: every float expression that the reference evaluates
// in fp32 is evaluated here in fp32, in the reference's operand order, with separately rounded
// multiplies and adds (built with -ffp-contract=off and correctly rounded fp32 div/sqrt).
// Transcendentals of the fusion grid and registration grid are separable (a column term and a
// row term), so they are tabulated on the host with the same glibc sincosf the reference calls
// and uploaded once per layout/level; the device never evaluates sin/cos on the parity path.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <vector>

#include "../../include/panofuse.h"

#pragma clang fp contract(off)

#define PF_MYPI 3.14159265359  // Basic.h:11
#define PF_NAN_MARKER 0x7FBADBADu  // "un-windowed pixel" tag in the target array (sNaN payload)
#define PF_MAX_COVER 40            // normalised stencil weights are exactly {1,-0.25} up to here

namespace pf {

// Per-tile projection constants: PerspectiveMap's cached window (Depth.h:85-92) plus the
// loop-invariant pieces of SphericalTo2D (|hedge|, |vedge|, (middle-0).middle).
struct TileGeom {
    float middle[3], hedge[3], vedge[3], corner0[3];
    float mm, hl, vl, pad;
    int w, h, c;
    int pix_off;    // first pixel of the tile in layout-wide per-pixel tables (warp map)
    long long off;  // float offset of the tile inside one panorama's tile block
};

// Tile box at one fusion level (Depth.cpp:1497-1562) after the clamps.
struct TileBox {
    int x0, x1, y0, y1, xs, pad[3];
};

// Does the box (X from x0 stepping xs, stopping before x1; rows y0..y1) meet [X0,X1]x[Y0,Y1]?
// Host (per-patch tile masks of the targets gather) and device alike.
__host__ __device__ inline bool box_meets(const TileBox& bx, int X0, int X1, int Y0, int Y1)
{
    if (bx.y0 > bx.y1 || bx.y1 < Y0 || bx.y0 > Y1) return false;
    const int lo = bx.xs > 0 ? bx.x0 : bx.x1 + 1, hi = bx.xs > 0 ? bx.x1 - 1 : bx.x0;
    return lo <= hi && hi >= X0 && lo <= X1;
}

// Tap-index map extent of one tile at one level: its box plus a one-pixel ring, row-major,
// starting at element `off` of the level's map.
struct TapBox {
    int xmin, ymin, nx, ny;
    long long off;
};

// Tile box of SolveDepthBySmoothing (Depth.cpp:1795-1808): the fusion box without its clamps.
struct SmoothBox {
    int x0, x1, y0, y1, xs, pad[3];
};

struct GridCol { float az, ca, sa, pad; };   // column xx (index xx+1): az, cos az, sin az
struct GridRow { float zen, sz, cz, pad; };  // row yy (index yy+1): zen, sin zen, cos zen

// Registration grid of one tile (Depth.cpp:1298-1335).
struct RegGrid {
    int cols, rows, col_off, row_off;  // offsets into the shared GridCol / GridRow tables
    int soff;                          // first sample of this tile in the sample-index table
};

// GL camera of SaveCubeMap (Main.cpp:246-269) per tile, evaluated on the host in double.
struct RgbCam {
    double f[3], s[3], u[3];
    double tx, ty;
};

// One RGB warp tap (k_warp_rgb): GL_REPEAT corners (x | y << 16) and GL_LINEAR weights of a tile
// pixel, built on the host per layout and panorama size (rgb_taps_host).
struct RgbTap {
    uint32_t x0y0, x1y1;
    float ax, ay;
};

// One patch of an RGB tile for the LDS-staged RGB warp (k_warp_rgb_box): 64 pixels wide and
// nrow <= 16 rows (fewer where the footprint is large, near the poles).  Its corners' panorama
// footprint is staged as whole 16-B units of the u8 RGB rows it touches, each row only over the
// bytes its pixels use (a ragged footprint, not a bounding box); the host lists the units'
// byte offsets (rgb unit table, kRgbUnits per patch).
struct RgbPatch {
    int tile, X0, Y0, nrow;
    int units;  // staged 16-B units (<= kRgbUnits)
    int wide;   // even one row's footprint exceeds the LDS slot: direct corner gathers
    int pad[2];
};
#ifndef PF_RGB_PW
#define PF_RGB_PW 64
#endif
// RGB warp patch: 256 threads x 4 consecutive pixels of one row (kRgbPW / 4 lanes per row)
static constexpr int kRgbPW = PF_RGB_PW, kRgbPH = 1024 / kRgbPW;
static constexpr int kRgbUnits = 512;            // 16-B units per patch (two per thread)
static constexpr int kRgbCap = 16 * kRgbUnits;   // LDS bytes per parity: the u8 RGB rows as is

// Synthetic depth-net response (same layout as pf_response in panofuse.h).
struct Resp {
    float alpha, kappa, beta, sigma;
    uint32_t seed, pad;
};

// One square patch of a tile for the E->P depth warp (pf_warp.hip): its tile pixels and the
// azimuth-unwrapped panorama box their bilinear corners fall in (filled on the device).
struct WarpPatch {
    int tile, X0, Y0;
    int gx0, gy0, bw, bh;  // box origin (column mod pw, row) and size, +1 row/column
    int wide;              // box larger than the LDS staging capacity: direct gathers
    // ragged footprint (round 5, the default when pw % 4 == 0): the 16-B units of the panorama
    // rows the patch's corners read, each row only over its corners' columns, listed as byte
    // offsets at unit_tbl[uoff .. uoff + units) (warp_patches_host); 0 units = the box above
    int uoff, units;
};

struct LevelDims {
    int w, h, h0, h1, iters, nlevels;
};

// ------------------------------------------------------------------------------------------
// Imath Vec3<float> arithmetic in source order (ImathVec.h:1467-1486, 1631-1700).
__host__ __device__ inline float dot3(const float* a, const float* b)
{
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}

// SphericalTo2D (Depth.cpp:168-182) with dir = SphericalToWorld(az, zen) (Depth.cpp:2955-2958)
// given as the tabulated (sin zen, cos zen, cos az, sin az).  LinePlaneIntersection
// (Depth.cpp:34-42) with p = 0 and p0 = normal = middle: t = (middle.middle)/(dir.middle),
// pos = 0 + t*dir.
__host__ __device__ inline void sph_to_2d(const TileGeom& g, float sz, float cz, float ca,
                                          float sa, float& x, float& y)
{
    float d0 = sz * ca, d1 = sz * sa, d2 = cz;
    float den = d0 * g.middle[0] + d1 * g.middle[1] + d2 * g.middle[2];
    float t = g.mm / den;
    float p0 = 0.0f + t * d0, p1 = 0.0f + t * d1, p2 = 0.0f + t * d2;
    float e0 = p0 - g.corner0[0], e1 = p1 - g.corner0[1], e2 = p2 - g.corner0[2];
    float eh = e0 * g.hedge[0] + e1 * g.hedge[1] + e2 * g.hedge[2];
    float ev = e0 * g.vedge[0] + e1 * g.vedge[1] + e2 * g.vedge[2];
    x = (eh / g.hl) / g.hl;
    y = (ev / g.vl) / g.vl;
}

// PerspectiveMap::Value (Depth.cpp:111-118): truncating nearest lookup; returns the linear
// element index (Y*W+X)*C.
__host__ __device__ inline long long tile_index(const TileGeom& g, float x, float y)
{
    int X = (int)(x * (float)(g.w - 1));
    int Y = (int)(y * (float)(g.h - 1));
    return ((long long)Y * g.w + X) * g.c;
}

#ifndef PF_CUBIC_SEL
// 1: the clamps as selects.  Measured slower in the targets kernel (round 6, serial C3 trace:
// 0.488 against 0.450 ms; the selects' operands raise its scalar-register spills).  Off.
#define PF_CUBIC_SEL 0
#endif
// Depth2DepthTransform's per-pixel map (Depth.cpp:256-271).
__host__ __device__ inline float cubic_map(float X, float a, float b, float c, float d)
{
    // Depth2DepthTransform's clamps compare the float X against the double constants 1e-4 and
    // 1 - 1e-4 (Depth.cpp:245-274).  The float forms below decide identically for every one of
    // the 2^32 float bit patterns (NaN included; tests/test_cubic_thresholds.py runs the
    // exhaustive check): (double)X < 1e-4 iff X <= 0x38D1B717 (= (float)1e-4, the largest float
    // below 1e-4), and (double)X > 1 - 1e-4 iff X > 0x3F7FF972 (= (float)(1 - 1e-4), the largest
    // float below it).  No f64 conversion or compare per value.
    // (PF_CUBIC_SEL: selects instead of branches; the two forms are equal for every X and Y,
    // NaN included: the second test cannot hold after the first one did)
#if PF_CUBIC_SEL
    X = X <= 9.99999974737875e-05f ? (float)1e-4 : X;
    X = X > 0.99989998340606689f ? (float)(1 - 1e-4) : X;
    float Y = a * X * X * X + b * X * X + c * X + d;
    Y = Y < 0 ? 0.0f : Y;
    Y = Y > 1 ? 1.0f : Y;
#else  // round-5 form (A/B)
    if (X <= 9.99999974737875e-05f) X = (float)1e-4;
    else if (X > 0.99989998340606689f) X = (float)(1 - 1e-4);
    float Y = a * X * X * X + b * X * X + c * X + d;
    if (Y < 0) Y = 0;
    else if (Y > 1) Y = 1;
#endif
    return Y;
}

// XCD-aware block order.  The dispatcher deals workgroup b to XCD (b mod 8) (MI355X_MICROARCH.md,
// workgroup dispatch); this maps it to a logical block so that every XCD walks one contiguous
// range of logical blocks, and neighbouring blocks -- which re-read each other's edge lines --
// share that XCD's L2.  A bijection on [0, n).
__device__ __forceinline__ unsigned xcd_remap(unsigned b, unsigned n)
{
    const unsigned x = b & 7u, s = b >> 3, q = n >> 3, r = n & 7u;
    return x * q + (x < r ? x : r) + s;
}

// EquirectangularMap::ValueAtCoord (Depth.cpp:551-556): index math promoted to double by MYPI.
__host__ __device__ inline long long emap_index(float az, float zen, int w, int h, int c)
{
    int x = (int)((double)az / (PF_MYPI * 2) * (double)(float)(w - 1));
    int y = (int)((double)zen / PF_MYPI * (double)(float)(h - 1));
    return ((long long)y * w + x) * c;
}

// One temporally blocked Jacobi pass (pf_jacobi.hip).
struct JacobiPass {
    const float* src; long long sstride;    // SRC_BUF input
    const float* prev; long long pstride;   // SRC_UPSAMPLE input (previous level, w/2 x h/2)
    const float* emap; long long estride;   // SRC_SEED input
    int ew, eh, ec, src_mode;
    // SRC_SEED: ValueAtCoord's index split into its column and row terms (emap_index is
    // separable): x * ec per virtual column xx at ecol[xx + 1], y * ew * ec per row yy at
    // erow[yy + 1] (host-computed with the same fp64 expression, run_jacobi)
    const int* ecol; const int* erow;
    const GridCol* cols; const GridRow* rows;
    const float* lnorm; long long lstride;
    float* dst; long long dstride;
    uint16_t* out; long long ostride;
    int out_mode;
    int w, h, h0, h1;
    int V, Tp, nstrips, nchunks, rows_per_chunk;
    int row_lo, row_hi;  // rows stored by this pass: [row_lo, row_hi) within [h0, h1] (chunked)
    const float* hcol;  // packed form: per column 0.5 (covered) or 0 (un-windowed), w entries
};

// The resident level kernel (pf_jres.hip): all of a level's sweeps in one launch.
struct JresArgs {
    const float* src; long long sstride;    // src_mode 0: buffer
    const float* prev; long long pstride;   // src_mode 1: nearest upsample of the previous level
    const float* emap; long long estride;   // src_mode 2: level-0 seed through ecol / erow
    const int* ecol; const int* erow;
    const float* lnorm; long long lstride;
    const float* hcol;                      // separable-coverage certificate (packed form)
    float* dst; long long dstride;
    uint16_t* out; long long ostride;       // non-null: store the u16 quantisation instead
    int w, h, h0, h1, iters, batch, src_mode;
    int nb, core, K;       // row blocks per panorama, core rows per block, sweeps per round
    int half;              // 1: the half-height region (rows per wave halved; jres_region_rows)
    float* xbuf;           // hand-off rows [batch][nb][2 parity][2 edge][K][w]
    uint32_t* flags;       // [batch][nb] last round published (monotone across launches)
    uint32_t* ticket;      // workgroup ticket counter (monotone across launches)
    uint32_t* err;         // spin timeouts (pf_jres_errors)
    uint32_t* err_host;    // raised (system-scope store) on any timeout: coherent pinned memory
    uint32_t tbase, fbase; // this launch's first ticket / flag base
    int dbg;               // profiling only (wrong results): 1 no hand-offs, 4 no rows, 8 no
                           // barriers; 16 (pf_debug_jres_fault): row block 0 withholds its flag
    int spin_log2;         // a hand-off wait gives up (and counts into err) after 2^spin_log2 polls
};
int jres_region_rows(int w, bool half = false);  // 0: not supported
int jres_threads();
int jres_words_per_value();
int jres_flags_per_block(int K);  // 2: the hand-off rows travel as {value, tag} granules
int jres_blocks_per_cu(int w, bool half);
void launch_jres(hipStream_t s, const JresArgs& A);

// ------------------------------------------------------------------------------------------
// Kernel launchers (pf_kernels.hip, pf_jacobi.hip).  All are asynchronous on `stream`.
void launch_tapmap(hipStream_t s, const TileGeom* geom, const TapBox* tb, int ntiles,
                   long long max_points, const GridCol* cols, const GridRow* rows, int32_t* map);
void launch_targets_map(hipStream_t s, const TileGeom* geom, const TileBox* box,
                        const TapBox* tb, int ntiles, const int32_t* map, const float* tiles,
                        long long tstride, const float* coeffs, LevelDims L, float* lnorm,
                        long long lstride, int batch);
void launch_targets_patch(hipStream_t s, const TileGeom* geom, const TileBox* box,
                          const TapBox* tb, int ntiles, const int32_t* map, const float* tiles,
                          long long tstride, const float* coeffs, LevelDims L, float* lnorm,
                          long long lstride, int batch, const uint32_t* tmask = nullptr,
                          int nmw = 0);
// All levels' targets in one launch (pf_targets.hip): per level its tables and plane, and a host
// table of (level, patch) entries in gather order (fuse_range builds it once per level set).
struct TgtLevel {
    LevelDims L;
    const TileBox* box;
    const uint32_t* tmask;  // per patch, mask words of the tiles whose box meets it (tile order)
    int nmw;                // mask words per patch: ceil(ntiles / 32)
    const TapBox* tb;
    const int32_t* map;
    float* lnorm;
    long long lstride;
    int npx, npy;
};
struct TgtMulti {
    TgtLevel lv[4];
    int nlev, nentries;
};
int targets_patch_w();
int targets_patch_h();
int targets_batch();
void launch_targets_multi(hipStream_t s, const TileGeom* geom, int ntiles, const float* tiles,
                          long long tstride, const float* coeffs, const TgtMulti& M,
                          const int2* order, int batch);
bool jstream_supported_T(int T);
int jstream_waves_per_cu(int C, int T, bool fast);
bool jstream_supported_C(int C, bool fast);
void launch_jstream(hipStream_t s, const JacobiPass& P, int C, int T, int batch, bool fast);
bool jpipe_supported(int S, int TS);
int jpipe_waves_per_cu(int S, int TS);
void launch_jpipe(hipStream_t s, const JacobiPass& P, int S, int TS, int batch);
void launch_border(hipStream_t s, const float* prev, long long pstride, LevelDims L, float* a,
                   float* b, long long stride, uint16_t* out, long long ostride, int batch);
void launch_seed0(hipStream_t s, const float* emap, int ew, int eh, int ec, long long estride,
                  const GridCol* cols, const GridRow* rows, LevelDims L, float* buf,
                  long long bstride, int batch);
void launch_upsample(hipStream_t s, const float* prev, long long pstride, LevelDims L,
                     float* buf, long long bstride, int batch);
void launch_targets(hipStream_t s, const TileGeom* geom, const TileBox* box, int t0, int t1,
                    const GridCol* cols, const GridRow* rows, const float* tiles,
                    long long tstride, const float* coeffs, int ntiles_total, LevelDims L,
                    float* lnorm, long long lstride, int batch);
 // rows [r0,r1), -1: band
// the tile masks of the level's targets patches (LevelCache::tmask, targets_patch_w/h grid)
hipError_t launch_targets_partial(hipStream_t s, const TileGeom* geom, const TileBox* box,
                                const TapBox* tb, const uint32_t* tmask, int nmw, int t0, int t1,
                                const int32_t* map, const float* tiles, const float* coeffs,
                                LevelDims L, float* lsum, float* cnt, int r0, int r1);
void launch_coverage_rows(hipStream_t s, const TileBox* box, int ntiles, LevelDims L, float* cnt,
                          int r0, int r1);
void launch_rows_add(hipStream_t s, float* dst, const float* src, long long n);
// pf_rows_add_batch's kernel argument: up to kRowsAddBatch segments by value
static constexpr int kRowsAddBatch = 32;
struct RowsAddBatch {
    float* dst[kRowsAddBatch];
    const float* src[kRowsAddBatch];
    long long n[kRowsAddBatch];
};
void launch_rows_add_batch(hipStream_t s, const RowsAddBatch& B, int count, long long nmax);
void launch_normalize(hipStream_t s, const float* lsum, const float* cnt, LevelDims L,
                      float* lnorm, int r0 = -1, int r1 = -1);
void launch_multicover(hipStream_t s, const TileGeom* geom, const int2* pairs, int npairs,
                       int t0, int t1, const GridCol* cols, const GridRow* rows,
                       const float* tiles, const float* coeffs, LevelDims L, float* contrib);
void launch_multicover_patch(hipStream_t s, const int2* pairs, int npairs, const float* contrib,
                             float* lsum);
void launch_probe_taps(hipStream_t s, const TileGeom* geom, const TileBox* box, int ntiles,
                       const GridCol* cols, const GridRow* rows, LevelDims L, int32_t* out);
void launch_jacobi(hipStream_t s, float* buf_a, float* buf_b, const float* lnorm,
                   long long stride, LevelDims L, int iters, int batch, float** result);
void launch_quantize(hipStream_t s, const float* buf, long long bstride, int n, uint16_t* out,
                     long long ostride, int batch);
void launch_register(hipStream_t s, const TileGeom* geom, const RegGrid* grids,
                     const GridCol* rcols, const GridRow* rrows, int ntiles, const float* emap,
                     int ew, int eh, int ec, long long estride, const float* tiles,
                     long long tstride, int degree, int solver, float* coeffs, double* coeffs64,
                     int batch, double* sums = nullptr, const int* active = nullptr,
                     const int2* sidx = nullptr);
// the registration samples' tile-element and baseline indices (layout- and baseline-size-only),
// built once per (layout, zenith range, baseline size) so k_register only gathers
void launch_regidx(hipStream_t s, const TileGeom* geom, const RegGrid* grids,
                   const GridCol* rcols, const GridRow* rrows, int ntiles, int max_samples,
                   int ew, int eh, int ec, int2* sidx);
int register_sums_per_tile();
void launch_register_joint(hipStream_t s, const double* sums, const int* active, int ntiles,
                           int batch, int degree, int solver, float* coeffs, double* coeffs64);
void launch_apply_cubic(hipStream_t s, const TileGeom* geom, int ntiles, long long tile_elems,
                        float* tiles, long long tstride, const float* coeffs, int batch);
int warp_patch_edge();
int warp_patch_height();
// host tables (pf_warp.hip): wxy/wfxy of one tile's pixels; the RGB taps of one tile
void warp_coords_host(const TileGeom& g, int pw, int ph, uint32_t* wxy, float* wfxy);
void rgb_taps_host(const RgbCam& cam, int W, int H, int pw, int ph, RgbTap* taps);
// The depth warp's patches of one tile with ragged footprints (from its corner map wxy, as
// warp_coords_host writes it): appended to `patches`, their units' byte offsets to `units`, and
// per pixel loc = LDS float index of the top corner pair | of the bottom pair << 16 (for a "wide"
// patch the global corner index with the x1/y1 flags of k_warp_local).  Needs pw % 4 == 0.
void warp_patches_host(const TileGeom& g, int tile, const uint32_t* wxy, int pw, int ph,
                       std::vector<WarpPatch>& patches, std::vector<uint32_t>& units,
                       uint32_t* loc);
// The RGB warp's patches of one tile (its taps at `taps`), appended to `patches`; their staged
// units' byte offsets to `units` (kRgbUnits per patch); per pixel the LDS float indices of its
// top and bottom corner pairs (loc: top | bottom << 16) and the GL_LINEAR weights (wts: ax, ay).
// Needs (3 * pw) % 16 == 0, 3 * pw * ph < 2^32 and tile width % 4 == 0.
void rgb_patches_host(const TileGeom& g, int tile, const RgbTap* taps, int pw, int ph,
                      std::vector<RgbPatch>& patches, std::vector<uint32_t>& units,
                      uint32_t* loc, float* wts);
void launch_warp_rgb_box(hipStream_t s, const TileGeom* geom, const RgbPatch* patches,
                         int npatch, const uint32_t* units, const uint32_t* loc, const float* wts,
                         const RgbTap* taps,
                         const long long* rgb_off, const uint8_t* pano, int pw, int ph,
                         long long pstride, uint8_t* tiles, long long tstride, int batch);
// patch footprint boxes and in-box corner indices from the uploaded wxy (in place over wloc)
void launch_warp_boxes(hipStream_t s, const TileGeom* geom, WarpPatch* patches, int npatch,
                       int pw, int ph, uint32_t* wloc);
void launch_warp_depth(hipStream_t s, const TileGeom* geom, int ntiles, const WarpPatch* patches,
                       const uint32_t* unit_tbl,
                       int npatch, const uint32_t* wloc, const float* wfxy, const float* pano,
                       int pw, int ph, long long pstride, const Resp* resp, float* tiles,
                       long long tstride, int batch);
void launch_warp_rgb(hipStream_t s, const RgbTap* taps, const TileGeom* geom, int ntiles,
                     long long npix_max, const long long* rgb_off, const uint8_t* pano, int pw,
                     int ph, long long pstride, uint8_t* tiles, long long tstride, int batch);

// SolveDepthBySmoothing (pf_smooth.hip).
void launch_smooth_map(hipStream_t s, const TileGeom* geom, const SmoothBox* box, int ntiles,
                       const GridCol* cols, const GridRow* rows, int w, int h, int2* src,
                       uint8_t* mask);
void launch_smooth_seed(hipStream_t s, const TileGeom* geom, int ntiles, const int2* src,
                        const float* tiles, long long tstride, const float* coeffs, int w, int h,
                        float* buf, int batch);
void launch_smooth_list(hipStream_t s, const int* list, const int* off, int nk, int w, int h,
                        int smin, int smax, int iters, float* buf, int batch);
// the row-band form: tickets, per-block step flags (monotone across launches), timeouts
struct SmoothSync {
    uint32_t* ticket;
    uint32_t* flags;     // [batch][nb]
    uint32_t* err;
    uint32_t* err_host;  // coherent pinned flag (PF_ETIMEOUT), may be null
    uint32_t tbase, fbase;
    int spin_log2;       // a neighbour wait gives up (counted, flagged) after 2^spin_log2 polls
    int fault;           // pf_debug_smooth_fault: row block 0 never publishes its steps
};
void launch_smooth_band(hipStream_t s, const int* list, const int* off, int nk, int nb, int w,
                        int h, int smin, int smax, int iters, float* buf, int batch,
                        const SmoothSync& S);
void launch_smooth(hipStream_t s, const TileGeom* geom, int ntiles, const int2* src,
                   const uint8_t* mask, const float* tiles, long long tstride,
                   const float* coeffs, int w, int h, int h0, int h1, int iters, float* buf,
                   int batch);

// Accuracy metrics (pf_metrics.hip).
struct MetricsJob {
    const float* gt;
    int gw, gh, gc;
    const float* given;
    const uint16_t* given16;
    int w, h, gc_given, batch;
    int h0, h1;  // compared rows, inclusive, clipped to [0, h-1]
    int align_way, cap_depth;
    int sequential;  // the reference's summation order (PF_METRICS_SEQUENTIAL)
};
size_t metrics_workspace_bytes(const MetricsJob& j);
void launch_d2d_map(hipStream_t s, float* data, long long npx, int c, const float* abcd);
void launch_metrics(hipStream_t s, const MetricsJob& j, void* ws, pf_metrics* out);

}  // namespace pf
