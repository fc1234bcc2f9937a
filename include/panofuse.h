/*
 * panofuse.h -- C-ABI of the MI355X (gfx950) panorama-depth fusion library (libpanofuse.so).
 *
 * Drop-in for the reference's DepthNamespace hot path (Depth.h:286-307 and the OpenGL E->P
 * render of Main.cpp:242-326).  Plain pointers and sizes only; every data pointer is a DEVICE
 * pointer (hipMalloc'd memory or a torch tensor's data_ptr()) owned by the caller, and every
 * call is stream-ordered on the context's stream.  Calls return PF_OK (0) or a negative PF_E*
 * code; pf_last_error() gives the message.  A context is bound to one device and one stream and
 * is not thread-safe: use one context per host thread per device.
 *
 * Batched layout in HBM (row-major, row 0 = zenith 0):
 *   emap  [batch][eh][ew][ec]           fp32 baseline equirectangular depth in [0,1]
 *   tiles [batch][sum_i th_i*tw_i*tc]   fp32 perspective tiles, tile i at offset sum_{j<i}
 *   out   [batch][out_h][out_w]         u16 fused panorama
 *   coeffs[batch][ntiles][4]            fp32 {a,b,c,d} of y = a x^3 + b x^2 + c x + d
 */
#ifndef PANOFUSE_H
#define PANOFUSE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PF_OK 0
#define PF_EINVAL (-1)     /* bad argument, shape or layout */
#define PF_ENOMEM (-2)     /* device allocation failed */
#define PF_EHIP (-3)       /* HIP runtime error */
#define PF_ESTATE (-4)     /* call order (e.g. no tiles set) */
#define PF_EDEGENERATE (-5) /* a tile box with x0 == x1 (the reference loops forever there) */
#define PF_ETIMEOUT (-6)   /* a resident-kernel hand-off wait timed out: the output of that
                            * fusion (or row-band smoothing) is invalid (see pf_jres_errors);
                            * reported by pf_synchronize, and by the next pf_fuse / pf_merge /
                            * pf_solve_smoothing once the timed-out call has finished */

typedef struct pf_ctx pf_ctx;

/* {azimuth_left, azimuth_right, zenith_top, zenith_down} in radians.  As a viewing window
 * this is PerspectiveMap::SetWindow's argument list (Depth.cpp:120); as a valid range it is
 * PerspectiveMap::ranges (Depth.h:82). */
typedef struct pf_window {
    float az_left, az_right, zen_top, zen_down;
} pf_window;

/* Synthetic stand-in for the external depth net (not part of the reference): per tile,
 * d' = clamp01(alpha*d + (kappa*d)*d + beta + sigma*u), u uniform in [-1,1) hashed from
 * (seed, pixel) -- seed unique per (panorama, layout-wide tile) -- as the oracle's pfo_hash32.
 * Used only to manufacture benchmark tiles from a ground-truth pano. */
typedef struct pf_response {
    float alpha, kappa, beta, sigma;
    uint32_t seed, pad;
} pf_response;

int pf_create(int device, pf_ctx** out);
void pf_destroy(pf_ctx* ctx);
const char* pf_last_error(const pf_ctx* ctx);
/* hipStream_t to order all work on (NULL = the null stream). */
int pf_set_stream(pf_ctx* ctx, void* hip_stream);
/* Waits for the context stream.  Returns PF_ETIMEOUT (message in pf_last_error) when a fusion
 * enqueued since the last report had a resident-kernel wait time out, i.e. its u16 output is
 * invalid -- the reference's "return false" on a failed merge (Depth.cpp:767-778). */
int pf_synchronize(pf_ctx* ctx);
const char* pf_version(void);

/* Tile layout.  Replaces PerspectiveMap::SetWindow + ranges (Depth.cpp:780-786).
 * cap_ranges != 0 applies MergeDepthMaps' MIN2(range, D2R(359.9)) to ranges[0..1]
 * (Depth.cpp:783-784).  tile_c = channels per tile pixel (channel 0 is used, as Value() does). */
int pf_set_tiles(pf_ctx* ctx, const pf_window* fovs, const pf_window* ranges, int ntiles,
                 const int* tile_w, const int* tile_h, int tile_c, int cap_ranges);

/* Registration solver for degree 3 (the reference's cubic FunctorDepth2Depth3):
 *   PF_SOLVER_LM (default) -- the reference's Ceres 1.13 Levenberg-Marquardt (DENSE_SCHUR,
 *     default options, from (1,1,1,1); Depth.cpp:1270-1274, 1399-1404), run per tile from the
 *     fp64 moment sums of its samples;
 *   PF_SOLVER_NORMAL -- the exact least-squares minimiser (fp64 normal equations).
 * Lower degrees always take the normal equations (the reference has no lower-degree solve). */
#define PF_SOLVER_NORMAL 0
#define PF_SOLVER_LM 1
int pf_set_solver(pf_ctx* ctx, int solver);

/* SolveDepthToDepth (Depth.cpp:1261-1414) for every tile with only that tile active
 * (MergeDepthMaps' loop, Depth.cpp:794-805), fp64 least squares of degree `degree`
 * (3 = the reference's FunctorDepth2Depth3, with the context's solver; 1 = scale/shift);
 * coeffs may be NULL.  coeffs64 (optional, [batch][ntiles][4] doubles) receives the unrounded
 * solution.  apply != 0 then runs Depth2DepthTransform (Depth.cpp:245-274) on the tiles. */
int pf_register(pf_ctx* ctx, const float* emap, int ew, int eh, int ec, float* tiles,
                int batch, float zr0, float zr1, int degree, int apply, float* coeffs,
                double* coeffs64);

/* SolveDepthToDepth with several active maps (Depth.cpp:1261-1414: the sample grids of every
 * active tile in one least-squares problem): active is a HOST int[ntiles] mask; coeffs
 * ([batch][4] floats) / coeffs64 ([batch][4] doubles) are device pointers (either may be NULL). */
int pf_register_joint(pf_ctx* ctx, const float* emap, int ew, int eh, int ec, const float* tiles,
                      int batch, float zr0, float zr1, int degree, const int* active,
                      float* coeffs, double* coeffs64);

/* SolveDepthAll (Depth.cpp:1416-1771): multi-level Laplacian-target scatter + damped Jacobi,
 * u16 output.  coeffs (optional, from pf_register with apply = 0) fuses Depth2DepthTransform
 * into the tile gather instead of rewriting the tiles. */
int pf_fuse(pf_ctx* ctx, const float* emap, int ew, int eh, int ec, const float* tiles,
            const float* coeffs, int batch, int out_w, int out_h, float zr0, float zr1,
            uint16_t* out);

/* MergeDepthMaps core (Depth.cpp:789-913) without file I/O: pf_register (degree 3) then
 * pf_fuse with the transform fused.  Tiles are left untouched; coeffs (optional) receives the
 * per-tile abcd. */
int pf_merge(pf_ctx* ctx, const float* emap, int ew, int eh, int ec, const float* tiles,
             int batch, int out_w, float zr0, float zr1, float* coeffs, uint16_t* out);

/* E->P depth warp: tile pixel (X,Y) -> ToSphericalCoord(X/(W-1), Y/(H-1)) (Depth.cpp:157-166)
 * -> bilinear sample of pano [batch][ph][pw] at (az/2pi*(pw-1), zen/pi*(ph-1)).  resp
 * ([batch][ntiles], optional) applies the synthetic depth-net response. */
int pf_warp_depth(pf_ctx* ctx, const float* pano, int pw, int ph, int batch,
                  const pf_response* resp, float* tiles);

/* E->P RGB warp (Main.cpp:242-326 SaveCubeMap + SphereMesh.cpp:154-210 texture mapping):
 * u8 RGB pano [batch][ph][pw][3] -> tiles [batch][sum_i th_i*tw_i*3], GL camera conventions,
 * GL_LINEAR + GL_REPEAT, rows top-first. */
int pf_warp_rgb(pf_ctx* ctx, const uint8_t* pano, int pw, int ph, int batch, uint8_t* tiles);

/* SolveDepthBySmoothing (Depth.cpp:1773-1878; Depth.h:309), the reference's alternate solver
 * (not called by mode 0): every tile written into the out_w x out_h grid (a later tile
 * overwrites an earlier one), 500 in-place Gauss-Seidel smoothing iterations on the pixels within
 * 10 of a tile-box edge in rows [floor(h*zr0/MYPI), ceil(h*zr1/MYPI)], u16 quantisation.
 * tiles: [batch][tile_elems] float (channel 0 read); coeffs: NULL, or [batch][ntiles][4] applied
 * as Depth2DepthTransform on the fly; out: [batch][out_h][out_w] u16.  Bit-exact.  The
 * row-band form's hand-off waits are bounded: a timeout makes the output invalid and is reported
 * as PF_ETIMEOUT by pf_synchronize (or the next call), as for the fusions. */
int pf_solve_smoothing(pf_ctx* ctx, const float* tiles, const float* coeffs, int batch,
                       int out_w, int out_h, float zr0, float zr1, uint16_t* out);

/* ---- multi-GPU fusion of one panorama (tiles sharded over ranks) ----
 * pf_fuse_partial scatters the Laplacian targets of tiles [t0, t1) for level `level` into
 * lsum/cnt ([out levels h][w] fp32 and fp32 counts); the caller sums them over ranks
 * (RCCL reduce), then pf_fuse_finish_level runs normalisation + Jacobi on the summed grids. */
int pf_level_info(int out_w, int out_h, float zr0, float zr1, int level, int* w, int* h,
                  int* h0, int* h1, int* iters, int* nlevels);
int pf_fuse_partial(pf_ctx* ctx, const float* tiles, const float* coeffs, int t0, int t1,
                    int out_w, int out_h, float zr0, float zr1, int level, float* lsum,
                    float* cnt);
/* buf: the level's buffer (in: seed/upsampled values, out: after the sweeps).  When
 * level == nlevels-1, out (if not NULL) receives the u16 quantisation. */
int pf_fuse_seed(pf_ctx* ctx, const float* emap, int ew, int eh, int ec, const float* prev,
                 int out_w, int out_h, float zr0, float zr1, int level, float* buf);
int pf_fuse_finish_level(pf_ctx* ctx, const float* lsum, const float* cnt, int out_w,
                         int out_h, float zr0, float zr1, int level, float* buf,
                         uint16_t* out);
/* pf_fuse_seed + pf_fuse_finish_level in one: the level is seeded (level 0 from emap, else
 * the 2x upsample of prev, the previous level's plane) inside its first sweep pass, as
 * pf_merge does it, with no seeded plane and no full-plane copies.  buf receives the level
 * (every row), except on the last level with out != NULL, where only out is written.  cnt ==
 * NULL: lsum holds the normalised targets (pf_fuse_targets).  The replicated levels of the
 * row-sharded C5 flow (pf_dist.fuse_row_sharded).  Round 5. */
int pf_fuse_level(pf_ctx* ctx, const float* emap, int ew, int eh, int ec, const float* prev,
                  const float* lsum, const float* cnt, int out_w, int out_h, float zr0,
                  float zr1, int level, float* buf, uint16_t* out);
/* One level's normalised targets (every tile, one panorama; [h_l][w_l] fp32, the band rows
 * written) -- what pf_fuse_level takes as lsum with cnt == NULL, when no partial sums need to
 * travel (the one-rank row-sharded fusion).  Round 5. */
int pf_fuse_targets(pf_ctx* ctx, const float* tiles, const float* coeffs, int out_w, int out_h,
                    float zr0, float zr1, int level, float* lnorm);
/* Exactness of the summed grids.  Per pixel the reference adds the covering tiles' Laplacians
 * one at a time (Depth.cpp:1609-1617); summing per-rank partials reproduces that for pixels
 * covered by at most two tiles, not for the few covered by three or more (sector corners on
 * shared band rows: 7 pixels per level in the C5 layout).  pf_fuse_multicover lists their
 * (pixel, tile) pairs (count in *npairs; contrib == NULL: count only) and writes contrib[i] =
 * the contribution of pair i's tile if it lies in [t0, t1), else 0; summing contrib over ranks
 * (exact: one non-zero per pair) and pf_fuse_multicover_patch then rewrites those pixels of
 * the summed lsum in the reference's single-thread order (tiles ascending). */
int pf_fuse_multicover(pf_ctx* ctx, const float* tiles, const float* coeffs, int t0, int t1,
                       int out_w, int out_h, float zr0, float zr1, int level, float* contrib,
                       int* npairs);
int pf_fuse_multicover_patch(pf_ctx* ctx, int out_w, int out_h, float zr0, float zr1, int level,
                             const float* contrib, float* lsum);

/* ---- row-band sharding of one level's Jacobi over ranks (pf_dist.py) ----
 * Every rank holds full-size level buffers but owns the rows [row0, row1) of the band [h0, h1].
 * pf_fuse_normalize: the normalised targets of (summed) pf_fuse_partial grids.
 * pf_fuse_border: the rows outside [h0, h1] (0 at level 0, else the nearest upsample of prev)
 *   into both ping-pong buffers a and b, or into the u16 out on the last level (and then, if
 *   a / b are given, their rows h0-1 and h1+1, which the passes' halo lanes read).
 * pf_fuse_band_plan: the sweep depths T[0..n) of the level's passes (returns n), a function of
 *   (level, nbands) only, so every rank derives the same plan.
 * pf_fuse_band_pass: one pass of depth T over rows [row0, row1): reads rows row0-T-1 .. row1+T
 *   of src (src_mode 0), or of the upsample of prev (1) or the emap seed (2, level 0) for the
 *   first pass; writes rows [row0, row1) of dst, or of the u16 out (when out != NULL: the last
 *   pass of the last level).  Between passes the caller refreshes the T+1 halo rows on each side
 *   from the neighbouring bands. */
int pf_fuse_normalize(pf_ctx* ctx, const float* lsum, const float* cnt, int out_w, int out_h,
                      float zr0, float zr1, int level, float* lnorm);
int pf_fuse_border(pf_ctx* ctx, const float* prev, int out_w, int out_h, float zr0, float zr1,
                   int level, float* a, float* b, uint16_t* out);
int pf_fuse_band_plan(pf_ctx* ctx, int out_w, int out_h, float zr0, float zr1, int level,
                      int nbands, int* T, int cap);
int pf_fuse_band_pass(pf_ctx* ctx, const float* emap, int ew, int eh, int ec, const float* prev,
                      const float* lnorm, int src_mode, const float* src, float* dst,
                      uint16_t* out, int out_w, int out_h, float zr0, float zr1, int level, int T,
                      int row0, int row1);
/* Row-restricted pieces of the sharded fusion (round 5): a rank computes only the rows it sweeps
 * plus their halo, and the rows its own tiles contribute to its neighbours'.
 * pf_fuse_partial_rows: pf_fuse_partial's sums of tiles [t0, t1) on rows [row0, row1) of the
 *   level only (clipped to the band [h0, h1]; nothing is zeroed elsewhere).
 * pf_fuse_coverage_rows: the coverage count n of ALL tiles on rows [row0, row1) (layout-only:
 *   a rank counts its rows itself instead of receiving the other ranks' counts).
 * pf_fuse_normalize_rows: pf_fuse_normalize on rows [row0, row1) only.
 * pf_fuse_tile_rows: [*ymin, *ymax] = the rows where tiles [t0, t1) have non-zero partial sums at
 *   this level (*ymin > *ymax when none); host only, from the cached boxes.
 * pf_rows_add: dst[i] += src[i], i < n (a received partial-sum segment; exact where a pixel is
 *   covered by at most two tiles -- the rest is pf_fuse_multicover's).
 * pf_rows_add_batch: the same for `count` segments (dst[k], src[k], n[k]: host arrays of device
 *   pointers and sizes) in one launch; the segments must not overlap. */
int pf_fuse_partial_rows(pf_ctx* ctx, const float* tiles, const float* coeffs, int t0, int t1,
                         int out_w, int out_h, float zr0, float zr1, int level, int row0,
                         int row1, float* lsum, float* cnt);
int pf_fuse_coverage_rows(pf_ctx* ctx, int out_w, int out_h, float zr0, float zr1, int level,
                          int row0, int row1, float* cnt);
int pf_fuse_normalize_rows(pf_ctx* ctx, const float* lsum, const float* cnt, int out_w,
                           int out_h, float zr0, float zr1, int level, int row0, int row1,
                           float* lnorm);
int pf_fuse_tile_rows(pf_ctx* ctx, int out_w, int out_h, float zr0, float zr1, int level, int t0,
                      int t1, int* ymin, int* ymax);
int pf_rows_add(pf_ctx* ctx, float* dst, const float* src, long long n);
int pf_rows_add_batch(pf_ctx* ctx, float* const* dst, const float* const* src,
                      const long long* n, int count);

/* ---- stage timing (hipEvents on the context stream; replaces the reference's timeGetTime
 * brackets around registration and fusion, Depth.cpp:792-808, 907-916) ----
 * While enabled, every entry point records an event pair around each stage it launches.
 * pf_profile_read synchronises, then writes PF_NSTAGES entries of: elapsed ms, algorithmic
 * bytes (SURVEY.md section 8d accounting) and kernel launches; it resets the accumulators. */
#define PF_STAGE_WARP 0
#define PF_STAGE_REGISTER 1
#define PF_STAGE_SEED 2
#define PF_STAGE_TARGETS 3
#define PF_STAGE_JACOBI 4
#define PF_STAGE_QUANTIZE 5
#define PF_STAGE_METRICS 6
#define PF_NSTAGES 7
int pf_profile_enable(pf_ctx* ctx, int on);
int pf_profile_read(pf_ctx* ctx, double* ms, double* bytes, long long* launches);

/* ---- cross-stream ordering (no reference counterpart) ----
 * Makes `hip_stream` (another stream on the same device) wait until level `level` of the
 * context's most recently enqueued fusion (pf_fuse / pf_merge) has finished its sweeps, e.g. to
 * start memory-bound work beside the finer levels instead of beside the coarse one.  Returns
 * PF_EINVAL if no fusion with that many levels was enqueued on this context. */
int pf_stream_wait_level(pf_ctx* ctx, int level, void* hip_stream);

/* ---- Jacobi engine selection (no reference counterpart; every engine is bit-identical) ----
 * mode 1 (default; the environment variable PF_JRES=0 changes the default to 0): levels of
 * width 256 or 512 with the separable-coverage certificate run all their sweeps in one resident
 * launch, in row_blocks blocks per panorama (0: chosen by the cost model); mode 0: the
 * streaming temporally blocked passes everywhere. */
int pf_set_jacobi_engine(pf_ctx* ctx, int mode, int row_blocks);

/* ---- Jacobi pass planning for concurrent fusions (no reference counterpart) ----
 * The streaming passes cut each level's band into row chunks by a cost model of the chip's wave
 * slots (more chunks: more waves, but every chunk re-runs a T-row fill).  Contexts whose fusions
 * run concurrently on one GPU (several fusion lanes) each see only part
 * of the chip: `share` (0 < share <= 1, default 1) is the fraction this context's plans count
 * on, so they take fewer, longer chunks -- less total work.  Results are bit-identical for any
 * share (the chunking never changes a value).  PF_EINVAL for a share outside (0, 1]. */
int pf_set_jacobi_share(pf_ctx* ctx, double share);

/* ---- resident level kernel health (no reference counterpart) ----
 * The coarse fusion level runs all its sweeps in one launch whose row blocks trade halo rows
 * through device memory (pf_jres.hip).  Its waits are bounded: a wait that times out is counted
 * here instead of hanging the device (the level's result is then invalid).  Synchronises the
 * context stream; returns the count since the context was created (>= 0) or an error code. */
int pf_jres_errors(pf_ctx* ctx);
/* Test hook (no reference counterpart): in the context's NEXT resident launch, row block 0 of
 * every panorama withholds its hand-off flag and every wait gives up after 2^spin_log2 polls
 * (spin_log2 in [4, 24]), so the neighbouring blocks time out: the fusion must then report
 * PF_ETIMEOUT.  The launch after that runs normally. */
int pf_debug_jres_fault(pf_ctx* ctx, int spin_log2);
/* The same hook for the context's NEXT row-band smoothing launch (pf_solve_smoothing with more
 * than one row block per panorama): row block 0 never publishes its steps, its neighbour's wait
 * gives up after 2^spin_log2 polls (and stops waiting for the rest of the launch), and
 * pf_synchronize / the next call reports PF_ETIMEOUT. */
int pf_debug_smooth_fault(pf_ctx* ctx, int spin_log2);

/* ---- parity probes (bit-exact index maps) ----
 * For level `level` of out_w: per covered pixel and tap k (5 taps in std::map order), the
 * linear tile index (Y*W+X)*C of the tap for the first covering tile, -1 elsewhere.
 * tap_index: [out_h_level][w][5] int32 device buffer.  lsum/cnt as pf_fuse_partial. */
int pf_probe_taps(pf_ctx* ctx, int out_w, int out_h, float zr0, float zr1, int level,
                  int32_t* tap_index);
/* The E->P warps' coordinate maps, exactly as pf_warp_depth / pf_warp_rgb build and cache them
 * (host code, glibc transcendentals as the reference calls them; no context or GPU needed).
 * HOST buffers, one tile of tile_w x tile_h with viewing window *fov, panorama pw x ph:
 *   pf_probe_warp_coords: wxy[h*w] = x0 | y0 << 16, wfxy[h*w][2] = (fx, fy) -- the bilinear
 *     corner and weights of ToSphericalCoord (Depth.cpp:157-166) at ValueAtCoord's convention;
 *   pf_probe_rgb_taps: taps[h*w][4] = {ix0 | iy0 << 16, ix1 | iy1 << 16, ax bits, ay bits} --
 *     the GL_REPEAT corners and GL_LINEAR weights of SaveCubeMap's camera ray (Main.cpp:246-269,
 *     fs_perspective.txt:67-73). */
int pf_probe_warp_coords(const pf_window* fov, int tile_w, int tile_h, int pw, int ph,
                         uint32_t* wxy, float* wfxy);
int pf_probe_rgb_taps(const pf_window* fov, int tile_w, int tile_h, int pw, int ph,
                      uint32_t* taps);

/* ---- accuracy metrics ----
 * ErrorData (Depth.cpp:1980-2213) when given16 != NULL: the u16 result [batch][h][w];
 * ErrorEmap (Depth.cpp:2215-2458) when given != NULL: a float map [batch][h][w][given_c]
 * (channel 0).  gt: [batch][gh][gw][gc] float in 0..1 (channel 0).  Rows
 * [(int)(zr0/MYPI*h), (int)(zr1/MYPI*h)] are compared, gt < 1e-4 is skipped, cap_depth caps
 * both at 10 m; align_way 0 = none, 1 = median shift (exact medians), 2 = least squares.
 * out: DEVICE array of batch pf_metrics.  Replaces the reference's float outputs
 * (mse, mae, mre, mselog, delta1..3) and the optional median_shift_factor / least_square_shift. */
typedef struct pf_metrics {
    float mse, mae, mre, mselog, delta1, delta2, delta3;
    float median_shift;          /* gt_median / given_median (align_way 1), else 1 */
    float ls_s, ls_o;            /* least_square {s, o} (align_way 2), else 0 */
    float gt_median, given_median;
    int32_t n, nlog;             /* num_compares, num_log_compares */
    int32_t reserved[2];
} pf_metrics;
int pf_error_metrics(pf_ctx* ctx, const float* gt, int gw, int gh, int gc, const float* given,
                     const uint16_t* given16, int w, int h, int given_c, int batch, float zr0,
                     float zr1, int align_way, int cap_depth, pf_metrics* out);
/* Summation order of the means (mse, mae, mre, mselog) and of the least-squares sums:
 *   PF_METRICS_TREE (the C-ABI's default) -- fp64 partial sums in a fixed tree: deterministic,
 *     0.9 ms per 64 panoramas at C3, means within 1e-5 relative of exact fp64 sums (and within
 *     1e-2 of the reference's drifting float sums).
 *   PF_METRICS_SEQUENTIAL -- "bit-exact means": the reference's order, row-major float
 *     accumulators (mse and mselog through a double add, Depth.cpp:2119-2123, 2178-2186);
 *     bit-exact to it (mselog within 1e-5: device log10f).  The per-pixel terms are formed by
 *     producer waves beside verified fp32 chains: ~7.4 ms per 64-panorama call at C3.
 * The facade (include/pf_depth.h) and panofuse_main default to PF_METRICS_SEQUENTIAL, the order
 * the reference prints; PF_METRICS_ORDER=tree / --metrics-order tree select the tree. */
#define PF_METRICS_TREE 0
#define PF_METRICS_SEQUENTIAL 1
int pf_set_metrics_order(pf_ctx* ctx, int order);

/* Depth2DepthTransform of one map (Depth.cpp:245-274): channel 0 of npix pixels of a DEVICE
 * buffer with `channels` interleaved channels, X = clamp(v, 1e-4, 1-1e-4),
 * v' = clamp01(a X^3 + b X^2 + c X + d) in the reference's fp32 order; abcd is a HOST float[4]. */
int pf_depth_transform(pf_ctx* ctx, float* data, long long npix, int channels, const float* abcd);

#ifdef __cplusplus
}
#endif
#endif
