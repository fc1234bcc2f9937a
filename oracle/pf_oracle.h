/*
 * pf_oracle.h -- CPU restatement of the reference's panorama-depth fusion path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product library links, loads or calls this code;
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, as the checker.
 *
 * PARITY STATUS: "parity unpinned" against the reference's own outputs.  The reference path
 * (Depth.cpp) cannot be built in this image without stand-ins (it includes <windows.h>, links
 * OpenCV's Windows libraries and needs a CMake-built Ceres with a generated config.h), and the
 * reference ships no tests, fixtures or golden vectors for this path.
 * This file is a line-by-line restatement of the reference arithmetic (every function cites the
 * Depth.cpp / ImathVec.h lines it follows); it is pinned only by the structural facts the survey
 * measured on the compiled reference (level bands, seam widths, out-of-tile tap counts), which
 * tests/test_oracle.py checks.
 *
 * Numeric contract: fp32 for projection and fusion with no FMA
 * contraction (compile with -ffp-contract=off), fp64 where the reference promotes through the
 * double constant MYPI, glibc sincosf/tanf/atan2f for the transcendentals.
 */
#ifndef PF_ORACLE_H
#define PF_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PFO_MYPI 3.14159265359 /* Basic.h:11 -- deliberately not exact pi */

/* One perspective tile: PerspectiveMap (Depth.h:61-158) minus the triangulation members. */
typedef struct pfo_tile {
    int width, height, channels;
    long long offset;        /* offset (in floats) of this tile inside the packed tile buffer */
    float az_left, az_right, zen_top, zen_down; /* viewing window, radians (Depth.h:76-79) */
    float ranges[4];         /* valid {azi_left, azi_right, zen_up, zen_down} (Depth.h:82) */
    float middle[3], hedge[3], vedge[3];
    float corner0[3], corner1[3], corner2[3], corner3[3];
} pfo_tile;

/* Synthetic stand-in for the external depth net's response (per tile):
 * d' = clamp01(alpha*d + (kappa*d)*d + beta + sigma*u), u uniform in [-1,1) from
 * pfo_hash32(seed, pixel) >> 8; seed is unique per (panorama, layout-wide tile). */
typedef struct pfo_response {
    float alpha, kappa, beta, sigma;
    uint32_t seed;
    uint32_t pad;
} pfo_response;

/* ---------------- projection (Depth.cpp:34-42, 111-182, 551-556, 2955-2971) ---------------- */
void  pfo_sph_to_world(float az, float zen, float out[3]);
void  pfo_world_to_sph(const float p[3], float out[2]);
void  pfo_set_window(pfo_tile* t, float az_left, float az_right, float zen_top, float zen_down);
void  pfo_sph_to_2d(const pfo_tile* t, float az, float zen, float out[2]);
void  pfo_to_spherical_coord(const pfo_tile* t, float x, float y, float out[2]);
long long pfo_tile_index(const pfo_tile* t, float x, float y);  /* (Y*W+X)*C of Value() */
float pfo_tile_value(const pfo_tile* t, const float* tiles, float x, float y);
float pfo_emap_value_at_coord(const float* emap, int w, int h, int c, float az, float zen);

/* fusion-grid coordinate of pixel index xx (or yy) at a level (Depth.cpp:1456,1591) */
float pfo_grid_azimuth(int xx, int w);
float pfo_grid_zenith(int yy, int h);

/* ---------------- registration (Depth.cpp:1122-1138, 1261-1414, 245-274) ---------------- */
int  pfo_reg_grid(const pfo_tile* t, float zr0, float zr1, int* cols, int* rows,
                  float* zen_top, float* zen_down);
/* Writes the sample pairs (x = tile depth, y = baseline depth; both clamped, fp64) in the
 * reference's r-major, c-minor order.  Returns the sample count. */
int  pfo_reg_samples(const pfo_tile* t, const float* tiles, const float* emap, int ew, int eh,
                     int ec, float zr0, float zr1, double* xs, double* ys);
/* Least-squares fit of y ~ sum_k coef[k] x^(degree-k) (degree 3: a x^3 + b x^2 + c x + d),
 * normal equations accumulated in the fixed 256-lane order the HIP kernel uses, solved by
 * partially pivoted Gaussian elimination in fp64.  coef64 gets degree+1 doubles, abcd gets
 * the Vec4f rounding (Depth.cpp:1408) padded with leading zeros to 4 floats. */
int  pfo_register_tile(const pfo_tile* t, const float* tiles, const float* emap, int ew, int eh,
                       int ec, float zr0, float zr1, int degree, double* coef64, float* abcd);
/* Solver selection (degree 3 only; lower degrees always take the normal equations):
 * PFO_SOLVER_NORMAL = the fp64 normal equations above; PFO_SOLVER_LM = the reference's Ceres LM
 * run from the same moment sums (pfo_lm_moments, pf_oracle_lm.c) -- the HIP default. */
enum { PFO_SOLVER_NORMAL = 0, PFO_SOLVER_LM = 1 };
int  pfo_register_tile_solver(const pfo_tile* t, const float* tiles, const float* emap, int ew,
                              int eh, int ec, float zr0, float zr1, int degree, int solver,
                              double* coef64, float* abcd);
void pfo_depth_to_depth(const pfo_tile* t, float* tiles, const float abcd[4]);

/* The reference's registration solver itself: Ceres 1.13 trust-region Levenberg-Marquardt with
 * DENSE_SCHUR and default options from (1,1,1,1) (pf_oracle_lm.c cites each rule it restates). */
enum { PFO_LM_NO_CONVERGENCE = 0, PFO_LM_FUNCTION_TOL = 1, PFO_LM_PARAMETER_TOL = 2,
       PFO_LM_GRADIENT_TOL = 3, PFO_LM_MIN_RADIUS = 4, PFO_LM_FAILURE = 5 };
typedef struct pfo_lm_summary {
    int iterations, successful, unsuccessful, termination;
    double initial_cost, final_cost;
} pfo_lm_summary;
/* Fit of y ~ a x^3 + b x^2 + c x + d over the samples (FunctorDepth2Depth3 residuals),
 * sample-wise exactly as Ceres evaluates it. */
/* The LM strategy state of levenberg_marquardt_strategy.cc (radius schedule and the diagonal
 * regulariser), shared by both LM forms and exposed for the Ceres-unit-test pins. */
typedef struct pfo_lm_strategy {
    double radius, max_radius, decrease, min_diag, max_diag;
    int reuse_diag;
    double diag[4];
} pfo_lm_strategy;
void pfo_lms_init(pfo_lm_strategy* s, double initial_radius, double max_radius, double min_diag,
                  double max_diag);
void pfo_lms_accepted(pfo_lm_strategy* s, double step_quality);
void pfo_lms_rejected(pfo_lm_strategy* s, double step_quality);
void pfo_lms_regularizer(pfo_lm_strategy* s, const double* colsq, int n, double* D);
int  pfo_lm_fit(const double* xs, const double* ys, int n, double coef[4], pfo_lm_summary* s);
int  pfo_register_tile_lm(const pfo_tile* t, const float* tiles, const float* emap, int ew,
                          int eh, int ec, float zr0, float zr1, double* coef64, float* abcd,
                          pfo_lm_summary* s);
/* The same LM run from the 15 moment sums (J'J upper triangle, J'y, y'y): the HIP kernel's form. */
int  pfo_lm_moments(const double S[15], double coef[4], pfo_lm_summary* s);
/* MergeDepthMaps core with the sample-wise LM registration (tile_data transformed in place). */
int  pfo_merge_lm(const float* emap, int ew, int eh, int ec, const pfo_tile* tiles, int ntiles,
                  float* tile_data, int out_w, float zr0, float zr1, uint16_t* out,
                  float* abcd_out);

/* SolveDepthBySmoothing (Depth.cpp:1773-1878): tiles written into the width x height grid (a
 * later tile overwrites), 500 in-place Gauss-Seidel iterations on the pixels within 10 of a box
 * edge, u16.  Returns 0, -1 (x0 == x1), -2 (box or stencil leaves the buffer). */
int  pfo_solve_smoothing(const pfo_tile* tiles, int ntiles, const float* tile_data, int width,
                         int height, float zr0, float zr1, uint16_t* data);

/* ---------------- fusion (Depth.cpp:1416-1771) ---------------- */
typedef struct pfo_level {
    int w, h, h0, h1, iters, max_level;
} pfo_level;
int  pfo_level_dims(int out_w, int out_h, float zr0, float zr1, int level, pfo_level* L);
void pfo_seed_level0(const float* emap, int ew, int eh, int ec, const pfo_level* L, float* buf);
void pfo_upsample(const float* prev, const pfo_level* L, float* buf);
/* Per tile: box of the level (after clamps), xs step.  Returns 0, or -1 if x0 == x1 (the
 * reference loops forever there). */
int  pfo_tile_box(const pfo_tile* t, const pfo_level* L, int* x0, int* x1, int* y0, int* y1,
                  int* xs);
/* Target Laplacians: Lsum (sum over covering tiles, tile order), n (number of covering tiles).
 * oops = number of taps outside [0,1]^2 (Depth.cpp:1595); oob = taps whose linear index
 * left the tile buffer (reference reads out of bounds there; we clamp). */
int  pfo_targets(const pfo_tile* tiles, int ntiles, const float* tile_data,
                 const pfo_level* L, float* Lsum, int32_t* n, long long* oops, long long* oob);
/* Normalised target per pixel (Depth.cpp:1626-1647).  Uncovered -> NaN marker bits. */
void pfo_normalize(const float* Lsum, const int32_t* n, const pfo_level* L, float* Lnorm);
/* Damped Jacobi sweeps (Depth.cpp:1649-1718); Lnorm with the marker for un-windowed pixels. */
void pfo_jacobi(float* buf, float* tmp, const float* Lnorm, const pfo_level* L, int iters);
void pfo_quantize(const float* buf, int n, uint16_t* out);
/* SolveDepthAll (Depth.cpp:1416-1771).  Returns 0 or a negative error. */
int  pfo_solve_depth_all(const float* emap, int ew, int eh, int ec, const pfo_tile* tiles,
                         int ntiles, const float* tile_data, int out_w, int out_h, float zr0,
                         float zr1, uint16_t* out, long long* oops);
/* MergeDepthMaps core (Depth.cpp:789-913): per-tile registration + transform, then fusion.
 * tile_data is modified in place (as the reference's pmaps are). */
int  pfo_merge(const float* emap, int ew, int eh, int ec, const pfo_tile* tiles, int ntiles,
               float* tile_data, int out_w, float zr0, float zr1, int degree, int solver,
               uint16_t* out, float* abcd_out);

/* ---------------- E->P depth warp (a5 mapping, Depth.cpp:157-166 + 2960-2971) ------------ */
void pfo_warp_depth(const float* pano, int pw, int ph, const pfo_tile* tiles, int ntiles,
                    const pfo_response* resp, float* tile_data);
uint32_t pfo_hash32(uint32_t seed, uint32_t idx);
/* its coordinate map for one tile: wxy = x0 | y0 << 16, wfxy = (fx, fy) per pixel */
void pfo_warp_coords(const pfo_tile* t, int pw, int ph, uint32_t* wxy, float* wfxy);

/* ---------------- E->P RGB warp (a18: Main.cpp:242-326, fs_perspective.txt:67-73) --------- */
void pfo_warp_rgb(const uint8_t* pano, int pw, int ph, const pfo_tile* tiles, int ntiles,
                  uint8_t* out);
/* its tap map: 4 words per tile pixel {ix0 | iy0 << 16, ix1 | iy1 << 16, ax bits, ay bits} */
void pfo_rgb_taps(int pw, int ph, const pfo_tile* tiles, int ntiles, uint32_t* taps);

int  pfo_probe_taps(const pfo_tile* tiles, int ntiles, const pfo_level* L, int32_t* out);
void pfo_set_threads(int n);
uint32_t pfo_nan_marker(void);

/* ErrorData (Depth.cpp:1980-2213; given16 != NULL) / ErrorEmap (Depth.cpp:2215-2458; given
 * != NULL): sequential fp32 accumulation exactly as written, medians by sorting (the element at
 * index size/2).  out[0..6] = mse, mae, mre, mselog, delta1, delta2, delta3; out[7] = median
 * shift; out[8..9] = least-squares {s, o}; out[10..11] = gt / given medians; cnt[0..1] = n, nlog. */
void pfo_error_metrics(const float* gt, int gw, int gh, int gc, const float* given,
                       const uint16_t* given16, int w, int h, int given_c, float zr0, float zr1,
                       int align_way, int cap_depth, float* out, int* cnt);

#ifdef __cplusplus
}
#endif
#endif
