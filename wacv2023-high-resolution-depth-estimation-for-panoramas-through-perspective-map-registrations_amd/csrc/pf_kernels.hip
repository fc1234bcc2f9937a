// pf_kernels.hip -- gfx950 kernels of the panorama-depth fusion path.
//
// Every kernel is HBM/L2-bandwidth or VALU bound; there is no dense contraction, so no MFMA.
// Layout: batch-major planes, row-major pixels; one workgroup-grid dimension walks pixels
// (coalesced 64-lane rows), grid.y walks the batch (or the tile for per-tile work).
#include "pf_internal.hpp"

#include <cfloat>

namespace pf {

static constexpr int kBlock = 256;

__device__ __forceinline__ float bits_f(uint32_t u) { return __uint_as_float(u); }
__device__ __forceinline__ uint32_t f_bits(float f) { return __float_as_uint(f); }

// ---------------------------------------------------------------------------------------------
// Level-0 seed (Depth.cpp:1442-1465): rows [h0,h1] take ValueAtCoord of the pixel's spherical
// coordinate, other rows 0.
__global__ void __launch_bounds__(kBlock) k_seed0(const float* __restrict__ emap, int ew, int eh,
                                                  int ec, long long estride,
                                                  const GridCol* __restrict__ cols,
                                                  const GridRow* __restrict__ rows,
                                                  LevelDims L, float* __restrict__ buf,
                                                  long long bstride)
{
    long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
    long long n = (long long)L.w * L.h;
    if (i >= n) return;
    int b = blockIdx.y;
    int y = (int)(i / L.w), x = (int)(i - (long long)y * L.w);
    float v = 0.0f;
    if (y >= L.h0 && y <= L.h1) {
        long long e = emap_index(cols[x + 1].az, rows[y + 1].zen, ew, eh, ec);
        v = emap[b * estride + e];
    }
    buf[b * bstride + i] = v;
}

// Nearest 2x upsample of the previous level (Depth.cpp:1467-1485).
__global__ void __launch_bounds__(kBlock) k_upsample(const float* __restrict__ prev,
                                                     long long pstride, LevelDims L,
                                                     float* __restrict__ buf, long long bstride)
{
    long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
    long long n = (long long)L.w * L.h;
    if (i >= n) return;
    int b = blockIdx.y;
    int y = (int)(i / L.w), x = (int)(i - (long long)y * L.w);
    int wp = L.w / 2;
    buf[b * bstride + i] = prev[b * pstride + (long long)(y / 2) * wp + x / 2];
}

// ---------------------------------------------------------------------------------------------
// Laplacian target of tile p at pixel (X, Y): the 5-point mask in std::map key order
// (X-1,Y), (X,Y-1), (X,Y), (X,Y+1), (X+1,Y) with weights -1/4,-1/4,1,-1/4,-1/4, each tap
// projected through SphericalTo2D and read with Value() (Depth.cpp:1570-1606).  A tap whose
// linear index leaves the tile is clamped (the reference reads out of bounds there).
__device__ __forceinline__ float tap_value(const TileGeom& g, const float* __restrict__ tile,
                                           const GridCol& c, const GridRow& r, bool xform,
                                           float4 abcd)
{
    float x, y;
    sph_to_2d(g, r.sz, r.cz, c.ca, c.sa, x, y);
    long long idx = tile_index(g, x, y);
    long long lim = (long long)g.w * g.h * g.c;
    if (idx < 0) idx = 0;
    if (idx >= lim) idx = lim - g.c;
    float v = tile[idx];
    if (xform) v = cubic_map(v, abcd.x, abcd.y, abcd.z, abcd.w);
    return v;
}

__device__ __forceinline__ float target_one(const TileGeom& g, const float* __restrict__ tile,
                                            const GridCol* __restrict__ cols,
                                            const GridRow* __restrict__ rows, int X, int Y,
                                            bool xform, float4 abcd)
{
    float Lp = 0;
    Lp += tap_value(g, tile, cols[X], rows[Y + 1], xform, abcd) * -0.25f;      // (X-1, Y)
    Lp += tap_value(g, tile, cols[X + 1], rows[Y], xform, abcd) * -0.25f;      // (X, Y-1)
    Lp += tap_value(g, tile, cols[X + 1], rows[Y + 1], xform, abcd) * 1.0f;    // (X, Y)
    Lp += tap_value(g, tile, cols[X + 1], rows[Y + 2], xform, abcd) * -0.25f;  // (X, Y+1)
    Lp += tap_value(g, tile, cols[X + 2], rows[Y + 1], xform, abcd) * -0.25f;  // (X+1, Y)
    return Lp;
}

// X iterates x0, x0+xs, ... and stops before x1 (Depth.cpp:1565-1623).
__device__ __forceinline__ bool in_box(const TileBox& bx, int X, int Y)
{
    if (Y < bx.y0 || Y > bx.y1) return false;
    return bx.xs > 0 ? (X >= bx.x0 && X < bx.x1) : (X <= bx.x0 && X > bx.x1);
}

// Targets + normalisation for the band rows [h0, h1] (Depth.cpp:1487-1647).  Gather form of
// the reference's scatter: each pixel visits the tiles in index order, which is the reference's
// single-thread accumulation order (and bit-identical to any order for coverage <= 2).
// Output: normalised target, or PF_NAN_MARKER for an un-windowed pixel.
__global__ void __launch_bounds__(kBlock) k_targets(const TileGeom* __restrict__ geom,
                                                    const TileBox* __restrict__ box, int t0,
                                                    int t1, const GridCol* __restrict__ cols,
                                                    const GridRow* __restrict__ rows,
                                                    const float* __restrict__ tiles,
                                                    long long tstride,
                                                    const float* __restrict__ coeffs,
                                                    int ntiles_total, LevelDims L,
                                                    float* __restrict__ lnorm,
                                                    long long lstride)
{
    long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
    long long nband = (long long)L.w * (L.h1 - L.h0 + 1);
    if (i >= nband) return;
    int b = blockIdx.y;
    int Y = (int)(i / L.w) + L.h0, X = (int)(i - (long long)(Y - L.h0) * L.w);
    const float* tb = tiles + b * tstride;
    float acc = 0.0f;
    int n = 0;
    if (Y > L.h0 && Y < L.h1) {
        for (int p = t0; p < t1; p++) {
            TileBox bx = box[p];
            if (!in_box(bx, X, Y)) continue;
            const TileGeom& g = geom[p];
            float4 abcd = make_float4(0, 0, 0, 0);
            bool xf = coeffs != nullptr;
            if (xf) abcd = *reinterpret_cast<const float4*>(coeffs + ((long long)b * ntiles_total + p) * 4);
            acc += target_one(g, tb + g.off, cols, rows, X, Y, xf, abcd);
            n++;
        }
    }
    float out;
    if (n == 0) out = bits_f(PF_NAN_MARKER);
    else if (n == 1) out = acc;
    else {
        float center = 0.0f;
        for (int k = 0; k < n; k++) center += 1.0f;
        out = acc * (1.0f / center);
    }
    lnorm[b * lstride + (long long)Y * L.w + X] = out;
}

__global__ void __launch_bounds__(kBlock) k_normalize(const float* __restrict__ lsum,
                                                      const float* __restrict__ cnt,
                                                      LevelDims L, float* __restrict__ lnorm,
                                                      int r0, int r1)
{  // rows [r0, r1) of the band
    long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
    long long nband = (long long)L.w * (r1 - r0);
    if (i >= nband) return;
    long long o = (long long)r0 * L.w + i;
    int Y = (int)(o / L.w);
    float n = cnt[o];
    float out;
    if (Y <= L.h0 || Y >= L.h1 || n == 0.0f) out = bits_f(PF_NAN_MARKER);
    else if (n == 1.0f) out = lsum[o];
    else out = lsum[o] * (1.0f / n);
    lnorm[o] = out;
}

// Coverage count of rows [r0, r1) of the band by ALL tiles (the n of pf_fuse_partial over every
// tile, from the boxes alone): layout-only, so a rank of the sharded fusion counts its own rows
// instead of receiving the other ranks' counts.
__global__ void __launch_bounds__(kBlock) k_coverage_rows(const TileBox* __restrict__ box,
                                                          int ntiles, LevelDims L,
                                                          float* __restrict__ cnt, int r0, int r1)
{
    long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
    long long n = (long long)L.w * (r1 - r0);
    if (i >= n) return;
    const int Y = (int)(i / L.w) + r0, X = (int)(i - (long long)(Y - r0) * L.w);
    float c = 0.0f;
    if (Y > L.h0 && Y < L.h1)
        for (int p = 0; p < ntiles; p++) c += in_box(box[p], X, Y) ? 1.0f : 0.0f;
    cnt[(long long)Y * L.w + X] = c;
}

// dst[i] += src[i]: a received partial-target segment added into this rank's sums.  Exact for
// pixels covered by at most two tiles (one of the addends is zero, or the pair is the whole sum);
// the three-or-more pixels are re-added in tile order by pf_fuse_multicover_patch.
__global__ void __launch_bounds__(kBlock) k_rows_add(float* __restrict__ dst,
                                                     const float* __restrict__ src, long long n)
{
    const long long i = ((long long)blockIdx.x * kBlock + threadIdx.x) * 4;
    if (i + 3 < n) {
        float4 a = *reinterpret_cast<const float4*>(dst + i);
        const float4 b = *reinterpret_cast<const float4*>(src + i);
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
        *reinterpret_cast<float4*>(dst + i) = a;
    } else {
        for (long long j = i; j < n; j++) dst[j] += src[j];
    }
}

// Several segments in one launch (pf_rows_add_batch): blockIdx.y = segment.
__global__ void __launch_bounds__(kBlock) k_rows_add_batch(RowsAddBatch B)
{
    const int k = blockIdx.y;
    float* __restrict__ dst = B.dst[k];
    const float* __restrict__ src = B.src[k];
    const long long n = B.n[k];
    for (long long i = ((long long)blockIdx.x * kBlock + threadIdx.x) * 4; i < n;
         i += (long long)gridDim.x * kBlock * 4) {
        if (i + 3 < n && ((reinterpret_cast<uintptr_t>(dst + i) | reinterpret_cast<uintptr_t>(src + i)) & 15) == 0) {
            float4 a = *reinterpret_cast<const float4*>(dst + i);
            const float4 b = *reinterpret_cast<const float4*>(src + i);
            a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
            *reinterpret_cast<float4*>(dst + i) = a;
        } else {
            for (long long j = i; j < n && j < i + 4; j++) dst[j] += src[j];
        }
    }
}

// Parity probe: linear tile index of each tap of the first covering tile.
__global__ void __launch_bounds__(kBlock) k_probe_taps(const TileGeom* __restrict__ geom,
                                                       const TileBox* __restrict__ box,
                                                       int ntiles,
                                                       const GridCol* __restrict__ cols,
                                                       const GridRow* __restrict__ rows,
                                                       LevelDims L, int32_t* __restrict__ out)
{
    long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
    long long n = (long long)L.w * L.h;
    if (i >= n) return;
    int Y = (int)(i / L.w), X = (int)(i - (long long)Y * L.w);
    int32_t r[5] = {-1, -1, -1, -1, -1};
    if (Y > L.h0 && Y < L.h1) {
        for (int p = 0; p < ntiles; p++) {
            if (!in_box(box[p], X, Y)) continue;
            const TileGeom& g = geom[p];
            const int dc[5] = {0, 1, 1, 1, 2}, dr[5] = {1, 0, 1, 2, 1};
            for (int k = 0; k < 5; k++) {
                float x, y;
                const GridCol& c = cols[X + dc[k]];
                const GridRow& rr = rows[Y + dr[k]];
                sph_to_2d(g, rr.sz, rr.cz, c.ca, c.sa, x, y);
                r[k] = (int32_t)tile_index(g, x, y);
            }
            break;
        }
    }
    for (int k = 0; k < 5; k++) out[i * 5 + k] = r[k];
}

// ---------------------------------------------------------------------------------------------
// One damped Jacobi sweep over the band rows (Depth.cpp:1680-1717).  Taps are read by linear
// index so the east tap of column w-1 is pixel (0, Y+1), exactly like buffer[yy*width+xx].
__global__ void __launch_bounds__(kBlock) k_jacobi(const float* __restrict__ src,
                                                   float* __restrict__ dst,
                                                   const float* __restrict__ lnorm,
                                                   long long stride, LevelDims L)
{
    long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
    long long nband = (long long)L.w * (L.h1 - L.h0 + 1);
    if (i >= nband) return;
    long long base = (long long)blockIdx.y * stride;
    long long o = (long long)L.h0 * L.w + i;
    const float* s = src + base;
    float Lt = lnorm[base + o];
    float b = s[o];
    float cur = 0.0f, tgt = 0.0f;
    if (f_bits(Lt) != PF_NAN_MARKER) {
        tgt = Lt;
        cur += s[o - 1] * -0.25f;
        cur += s[o - L.w] * -0.25f;
        cur += b * 1.0f;
        cur += s[o + L.w] * -0.25f;
        cur += s[o + 1] * -0.25f;
    }
    const float reg = (float)1e-4;
    const float reg_ = 1 - reg;
    float target_val = b + (tgt - cur) * 0.5f;
    float v = target_val * reg_ + b * reg;
    if (v < 0) v = 0;
    else if (v > 1) v = 1;
    dst[base + o] = v;
}

__global__ void __launch_bounds__(kBlock) k_quantize(const float* __restrict__ buf,
                                                     long long bstride, int n,
                                                     uint16_t* __restrict__ out,
                                                     long long ostride)
{
    long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    int b = blockIdx.y;
    float v = buf[b * bstride + i];
    if (v < 0) v = 0;
    if (v > 1) v = 1;
    out[b * ostride + i] = (uint16_t)(v * 65535.0f);
}

// ---------------------------------------------------------------------------------------------
// Registration: one workgroup per (tile, panorama).  Lane l accumulates the 15 fp64 sums of
// J^T J / J^T y / y^T y over samples l, l+256, ... (J = (x^3, x^2, x, 1) of FunctorDepth2Depth3,
// Depth.cpp:1122-1138), then a fixed pairwise tree; lane 0 solves.  The order is fixed, so the
// result is reproducible and identical to the oracle's restatement.
static constexpr int kRegLanes = 256;
static constexpr int kRegSums = 15;

__device__ __forceinline__ double clamp_depth(double v)
{
    if (v < 1e-4) v = 1e-4;
    else if (v > (1 - 1e-4)) v = 1 - 1e-4;
    return v;
}

__device__ int solve_normal(const double* S, int degree, double* coef)
{
    const int idx[4][4] = {{0, 1, 2, 3}, {1, 4, 5, 6}, {2, 5, 7, 8}, {3, 6, 8, 9}};
    int n = degree + 1, off = 3 - degree;
    double A[4][5];
    for (int i = 0; i < n; i++) {
        for (int j = 0; j < n; j++) A[i][j] = S[idx[i + off][j + off]];
        A[i][n] = S[10 + i + off];
    }
    for (int k = 0; k < n; k++) {
        int piv = k;
        double best = fabs(A[k][k]);
        for (int i = k + 1; i < n; i++)
            if (fabs(A[i][k]) > best) { best = fabs(A[i][k]); piv = i; }
        if (!(best > 0.0)) return -1;
        if (piv != k)
            for (int j = 0; j <= n; j++) { double t = A[k][j]; A[k][j] = A[piv][j]; A[piv][j] = t; }
        for (int i = k + 1; i < n; i++) {
            double f = A[i][k] / A[k][k];
            for (int j = k; j <= n; j++) A[i][j] = A[i][j] - f * A[k][j];
        }
    }
    for (int i = n - 1; i >= 0; i--) {
        double s = A[i][n];
        for (int j = i + 1; j < n; j++) s = s - A[i][j] * coef[j];
        coef[i] = s / A[i][i];
    }
    return 0;
}


// ---------------------------------------------------------------------------------------------
// The reference's registration solver: Ceres 1.13 trust-region Levenberg-Marquardt, DENSE_SCHUR,
// default options, from (1,1,1,1) (Depth.cpp:1270-1274, 1399-1404), evaluated from the 15 moment
// sums -- the residuals are linear in (a,b,c,d), so cost, gradient and J'J are exact functions of
// them.  Every rule (Jacobi column scaling, LM diagonal and radius updates, step validity and
// quality, the parameter/function/gradient tolerances, returning the best accepted point) is
// cited in oracle/pf_oracle_lm.c, whose pfo_lm_moments is this function operation for operation
// (fp64 +, -, *, /, sqrt only, no contraction), so the two agree bit for bit.
namespace {
constexpr int kLmMaxIter = 50;
constexpr double kLmInitRadius = 1e4, kLmMaxRadius = 1e16, kLmMinRadius = 1e-32;
constexpr double kLmMinRelDecrease = 1e-3, kLmMinDiag = 1e-6, kLmMaxDiag = 1e32;
constexpr int kLmMaxInvalid = 5;
constexpr double kLmFuncTol = 1e-6, kLmGradTol = 1e-10, kLmParamTol = 1e-8;

struct Mom {
    double M[4][4], Jy[4], yy;
};

__device__ double mom_cost(const Mom& m, const double p[4])
{
    double pMp = 0.0, pJy = 0.0;
    for (int i = 0; i < 4; i++) {
        double q = 0.0;
        for (int j = 0; j < 4; j++) q = q + m.M[i][j] * p[j];
        pMp = pMp + p[i] * q;
        pJy = pJy + p[i] * m.Jy[i];
    }
    return 0.5 * ((m.yy - 2.0 * pJy) + pMp);
}

__device__ void mom_gradient(const Mom& m, const double p[4], double g[4])
{
    for (int i = 0; i < 4; i++) {
        double q = 0.0;
        for (int j = 0; j < 4; j++) q = q + m.M[i][j] * p[j];
        g[i] = q - m.Jy[i];
    }
}

__device__ double inv_psd1(double v)
{  // Eigen LLT of a 1x1 block solved against 1 (InvertPSDMatrix, full rank)
    const double l = sqrt(v);
    return (1.0 / l) / l;
}

__device__ bool llt3_solve(double S[3][3], const double rhs[3], double z[3])
{  // Eigen LLT<Upper> of the 3x3 reduced Schur system (schur_complement_solver.cc:197-213)
    double L[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    for (int k = 0; k < 3; k++) {
        double x = S[k][k];
        if (k > 0) {
            double sq = 0.0;
            for (int i = 0; i < k; i++) sq = sq + L[k][i] * L[k][i];
            x = x - sq;
        }
        if (!(x > 0.0)) return false;
        L[k][k] = x = sqrt(x);
        for (int j = k + 1; j < 3; j++) {
            double a = S[k][j];
            for (int i = 0; i < k; i++) a = a - L[j][i] * L[k][i];
            L[j][k] = a / x;
        }
    }
    double y[3] = {rhs[0], rhs[1], rhs[2]};
    for (int k = 0; k < 3; k++) {
        y[k] = y[k] / L[k][k];
        for (int j = k + 1; j < 3; j++) y[j] = y[j] - L[j][k] * y[k];
    }
    for (int k = 2; k >= 0; k--) {
        y[k] = y[k] / L[k][k];
        for (int j = 0; j < k; j++) y[j] = y[j] - L[k][j] * y[k];
    }
    z[0] = y[0]; z[1] = y[1]; z[2] = y[2];
    return true;
}

__device__ double norm4(const double v[4])
{
    return sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3]);
}
}  // namespace

__device__ void lm_moments(const double* S, double coef[4])
{
    Mom m;
    const int idx[4][4] = {{0, 1, 2, 3}, {1, 4, 5, 6}, {2, 5, 7, 8}, {3, 6, 8, 9}};
    for (int i = 0; i < 4; i++) {
        for (int j = 0; j < 4; j++) m.M[i][j] = S[idx[i][j]];
        m.Jy[i] = S[10 + i];
    }
    m.yy = S[14];
    double x[4] = {1.0, 1.0, 1.0, 1.0}, best[4] = {1.0, 1.0, 1.0, 1.0};
    double sc[4], Ms[4][4], g[4], gs[4], diag[4] = {0, 0, 0, 0}, D[4], step[4], cand[4];
    for (int k = 0; k < 4; k++) sc[k] = 1.0 / (1.0 + sqrt(m.M[k][k]));
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) Ms[i][j] = (m.M[i][j] * sc[i]) * sc[j];
    double radius = kLmInitRadius, decrease = 2.0, x_norm = -1.0;
    bool reuse_diag = false, successful = true;
    int invalid_run = 0, iteration = 0;
    double x_cost = mom_cost(m, x);
    mom_gradient(m, x, g);
    double min_cost = DBL_MAX;
    for (;;) {
        if (successful && x_cost < min_cost) {
            min_cost = x_cost;
            for (int k = 0; k < 4; k++) best[k] = x[k];
        }
        if (iteration >= kLmMaxIter) break;
        if (successful) {
            double gmax = 0.0;
            for (int k = 0; k < 4; k++) {
                const double d = fabs(x[k] - (x[k] + -g[k]));
                if (d > gmax) gmax = d;
            }
            if (gmax <= kLmGradTol) break;
        }
        if (radius <= kLmMinRadius) break;
        iteration++;
        if (!reuse_diag)
            for (int k = 0; k < 4; k++) {
                const double d = Ms[k][k] > kLmMinDiag ? Ms[k][k] : kLmMinDiag;
                diag[k] = d < kLmMaxDiag ? d : kLmMaxDiag;
            }
        for (int k = 0; k < 4; k++) D[k] = sqrt(diag[k] / radius);
        for (int k = 0; k < 4; k++) gs[k] = sc[k] * g[k];
        const double ete = D[0] * D[0] + Ms[0][0];
        double R[3][3], rhs[3], z[3];
        for (int a = 0; a < 3; a++)
            for (int b = a; b < 3; b++)
                R[a][b] = Ms[1 + a][1 + b] + (a == b ? D[1 + a] * D[1 + a] : 0.0);
        const double inv = inv_psd1(ete);
        const double inv_g = inv * gs[0];
        for (int a = 0; a < 3; a++) rhs[a] = gs[1 + a] - Ms[0][1 + a] * inv_g;
        for (int a = 0; a < 3; a++) {
            const double bt = Ms[0][1 + a] * inv;
            for (int b = a; b < 3; b++) R[a][b] = R[a][b] - bt * Ms[0][1 + b];
        }
        bool ok = llt3_solve(R, rhs, z);
        if (ok) {
            double ya = gs[0];
            for (int a = 0; a < 3; a++) ya = ya - Ms[0][1 + a] * z[a];
            step[0] = inv * ya;
            step[1] = z[0]; step[2] = z[1]; step[3] = z[2];
            for (int k = 0; ok && k < 4; k++) ok = isfinite(step[k]);
        }
        reuse_diag = true;
        double mcc = 0.0;
        bool valid = false;
        if (ok) {
            for (int k = 0; k < 4; k++) step[k] = step[k] * -1.0;
            double sJr = 0.0, sMs = 0.0;
            for (int i = 0; i < 4; i++) {
                double q = 0.0;
                for (int j = 0; j < 4; j++) q = q + Ms[i][j] * step[j];
                sMs = sMs + step[i] * q;
                sJr = sJr + step[i] * gs[i];
            }
            mcc = -(sJr + sMs / 2.0);
            valid = mcc > 0.0;
        }
        if (!valid) {
            if (++invalid_run >= kLmMaxInvalid) break;
            radius = radius / decrease;
            decrease *= 2.0;
            successful = false;
            continue;
        }
        invalid_run = 0;
        for (int k = 0; k < 4; k++) cand[k] = x[k] + step[k] * sc[k];
        double cand_cost = mom_cost(m, cand);
        if (!isfinite(cand_cost)) cand_cost = DBL_MAX;
        double dx[4];
        for (int k = 0; k < 4; k++) dx[k] = x[k] - cand[k];
        if (norm4(dx) <= kLmParamTol * (x_norm + kLmParamTol)) break;
        if (fabs(x_cost - cand_cost) <= kLmFuncTol * x_cost) break;
        const double rel = (x_cost - cand_cost) / mcc;
        if (rel > kLmMinRelDecrease) {
            for (int k = 0; k < 4; k++) x[k] = cand[k];
            x_norm = norm4(x);
            x_cost = mom_cost(m, x);
            mom_gradient(m, x, g);
            const double q = 2.0 * rel - 1.0;
            const double f = 1.0 - q * q * q;
            radius = radius / (f > 1.0 / 3.0 ? f : 1.0 / 3.0);
            radius = radius < kLmMaxRadius ? radius : kLmMaxRadius;
            decrease = 2.0;
            reuse_diag = false;
            successful = true;
        } else {
            radius = radius / decrease;
            decrease *= 2.0;
            successful = false;
        }
    }
    for (int k = 0; k < 4; k++) coef[k] = best[k];
}

// Degree-d least squares from the normal-equation sums (falling back to lower degrees when the
// system is singular), stored as {a, b, c, d} with the unused high-order terms 0.
__device__ void solve_store(const double* S, int degree, int solver, float* coeffs,
                            double* coeffs64, long long o)
{
    if (solver == PF_SOLVER_LM && degree == 3) {
        double c[4];
        lm_moments(S, c);
        for (int i = 0; i < 4; i++) {
            if (coeffs) coeffs[o + i] = (float)c[i];  // Vec4f(vars), Depth.cpp:1408
            if (coeffs64) coeffs64[o + i] = c[i];
        }
        return;
    }
    double coef[4] = {0, 0, 0, 0};
    int d = degree, rc = -1;
    while (d >= 0 && (rc = solve_normal(S, d, coef)) != 0) d--;
    if (rc != 0) { coef[0] = 0.0; d = 0; }
    double full[4] = {0, 0, 0, 0};
    for (int i = 0; i <= d; i++) full[3 - d + i] = coef[i];
    for (int i = 0; i < 4; i++) {
        if (coeffs) coeffs[o + i] = (float)full[i];
        if (coeffs64) coeffs64[o + i] = full[i];
    }
}

__global__ void __launch_bounds__(kRegLanes) k_register(
    const TileGeom* __restrict__ geom, const RegGrid* __restrict__ grids,
    const GridCol* __restrict__ rcols, const GridRow* __restrict__ rrows, int ntiles,
    const float* __restrict__ emap, int ew, int eh, int ec, long long estride,
    const float* __restrict__ tiles, long long tstride, int degree, int solver,
    float* __restrict__ coeffs, double* __restrict__ coeffs64, double* __restrict__ sums,
    const int* __restrict__ active, const int2* __restrict__ sidx)
{
    __shared__ double part[kRegSums][kRegLanes];
    // one linear grid, XCD-contiguous: the tiles of one panorama run on one XCD, so its emap is
    // fetched into one L2 (the samples of neighbouring tiles overlap in the emap)
    const unsigned lb = xcd_remap(blockIdx.x, gridDim.x);
    const int p = (int)(lb % (unsigned)ntiles), b = (int)(lb / (unsigned)ntiles), l = threadIdx.x;
    if (active && !active[p]) return;  // joint solve: an inactive tile is neither read nor solved
    const TileGeom g = geom[p];
    const RegGrid rg = grids[p];
    const float* tile = tiles + b * tstride + g.off;
    const float* em = emap + b * estride;
    const int ncol = rg.cols + 1;
    const int ns = ncol * (rg.rows + 1);
    double acc[kRegSums];
#pragma unroll
    for (int k = 0; k < kRegSums; k++) acc[k] = 0.0;
    // The lane's samples l, l + 256, ... in groups of kRegU: the gathers of a group are issued
    // together (they are independent), then added in sample order -- the same per-lane order as
    // one sample per iteration, so the sums are unchanged bit for bit.
    constexpr int kRegU = 4;
    for (int s0 = l; s0 < ns; s0 += kRegU * kRegLanes) {
        float tv[kRegU], ev[kRegU];
#pragma unroll
        for (int u = 0; u < kRegU; u++) {
            const int s = s0 + u * kRegLanes;
            tv[u] = 0.0f;
            ev[u] = 0.0f;
            if (s >= ns) continue;
            if (sidx) {  // the cached indices (k_regidx: the same arithmetic as below)
                const int2 ix = sidx[rg.soff + s];
                tv[u] = tile[ix.x];
                ev[u] = em[ix.y];
                continue;
            }
            int r = s / ncol, c = s - r * ncol;
            const GridCol cc = rcols[rg.col_off + c];
            const GridRow rr = rrows[rg.row_off + r];
            float x, y;
            sph_to_2d(g, rr.sz, rr.cz, cc.ca, cc.sa, x, y);
            if (x < 0) x = 0;
            if (x > 1) x = 1;
            if (y < 0) y = 0;
            if (y > 1) y = 1;
            tv[u] = tile[tile_index(g, x, y)];
            ev[u] = em[emap_index(cc.az, rr.zen, ew, eh, ec)];
        }
#pragma unroll
        for (int u = 0; u < kRegU; u++) {
            if (s0 + u * kRegLanes >= ns) break;
            double X = clamp_depth((double)tv[u]);
            double Yv = clamp_depth((double)ev[u]);
            double X2 = X * X, X3 = X * X * X;
            acc[0] = acc[0] + X3 * X3; acc[1] = acc[1] + X3 * X2; acc[2] = acc[2] + X3 * X;
            acc[3] = acc[3] + X3;      acc[4] = acc[4] + X2 * X2; acc[5] = acc[5] + X2 * X;
            acc[6] = acc[6] + X2;      acc[7] = acc[7] + X * X;   acc[8] = acc[8] + X;
            acc[9] = acc[9] + 1.0;
            acc[10] = acc[10] + X3 * Yv; acc[11] = acc[11] + X2 * Yv; acc[12] = acc[12] + X * Yv;
            acc[13] = acc[13] + Yv;
            acc[14] = acc[14] + Yv * Yv;
        }
    }
#pragma unroll
    for (int k = 0; k < kRegSums; k++) part[k][l] = acc[k];
    __syncthreads();
    for (int stride = kRegLanes / 2; stride >= 1; stride >>= 1) {
        if (l < stride)
            for (int k = 0; k < kRegSums; k++) part[k][l] = part[k][l] + part[k][l + stride];
        __syncthreads();
    }
    if (l == 0) {
        double S[kRegSums];
        for (int k = 0; k < kRegSums; k++) S[k] = part[k][0];
        if (sums) {  // joint solve: hand the tile's normal-equation sums to k_register_joint
            for (int k = 0; k < kRegSums; k++) sums[((long long)b * ntiles + p) * kRegSums + k] = S[k];
            return;
        }
        solve_store(S, degree, solver, coeffs, coeffs64, ((long long)b * ntiles + p) * 4);
    }
}

// SolveDepthToDepth with several active maps (Depth.cpp:1274-1376: every active map's sample
// grid feeds one problem): the active tiles' sums added in tile order, one solve per panorama.
__global__ void k_register_joint(const double* __restrict__ sums, const int* __restrict__ active,
                                 int ntiles, int batch, int degree, int solver,
                                 float* __restrict__ coeffs, double* __restrict__ coeffs64)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch) return;
    double S[kRegSums];
    for (int k = 0; k < kRegSums; k++) S[k] = 0.0;
    for (int p = 0; p < ntiles; p++)
        if (active[p])
            for (int k = 0; k < kRegSums; k++)
                S[k] = S[k] + sums[((long long)b * ntiles + p) * kRegSums + k];
    solve_store(S, degree, solver, coeffs, coeffs64, (long long)b * 4);
}

// Pixels covered by three or more tiles (pf_fuse_multicover, sharded fusion): the contribution
// of tile p to pixel o for every listed (o, p) pair with p in [t0, t1), 0 for the others.
__global__ void __launch_bounds__(kBlock) k_multicover_contrib(
    const TileGeom* __restrict__ geom, const int2* __restrict__ pairs, int npairs, int t0, int t1,
    const GridCol* __restrict__ cols, const GridRow* __restrict__ rows,
    const float* __restrict__ tiles, const float* __restrict__ coeffs, LevelDims L,
    float* __restrict__ contrib)
{
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= npairs) return;
    const int o = pairs[i].x, p = pairs[i].y;
    float v = 0.0f;
    if (p >= t0 && p < t1) {
        const int Y = o / L.w, X = o - Y * L.w;
        const TileGeom& g = geom[p];
        float4 abcd = make_float4(0, 0, 0, 0);
        const bool xf = coeffs != nullptr;
        if (xf) abcd = *reinterpret_cast<const float4*>(coeffs + (long long)p * 4);
        v = target_one(g, tiles + g.off, cols, rows, X, Y, xf, abcd);
    }
    contrib[i] = v;
}

// The window sums of those pixels in the reference's single-thread order (tiles ascending, from
// 0, one rounding per tile), overwriting the rank-summed values; pairs are sorted by pixel, then
// tile.  One thread: a handful of pixels per level.
__global__ void k_multicover_patch(const int2* __restrict__ pairs, int npairs,
                                   const float* __restrict__ contrib, float* __restrict__ lsum)
{
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    int i = 0;
    while (i < npairs) {
        const int o = pairs[i].x;
        float acc = 0.0f;
        for (; i < npairs && pairs[i].x == o; i++) acc += contrib[i];
        lsum[o] = acc;
    }
}

// Depth2DepthTransform on all tiles (channel 0), in place.
__global__ void __launch_bounds__(kBlock) k_apply_cubic(const TileGeom* __restrict__ geom,
                                                        int ntiles, float* __restrict__ tiles,
                                                        long long tstride,
                                                        const float* __restrict__ coeffs)
{
    const int p = blockIdx.y, b = blockIdx.z;
    const TileGeom g = geom[p];
    long long npx = (long long)g.w * g.h;
    const float4 abcd = *reinterpret_cast<const float4*>(coeffs + ((long long)b * ntiles + p) * 4);
    float* t = tiles + b * tstride + g.off;
    for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < npx;
         i += (long long)gridDim.x * kBlock)
        t[i * g.c] = cubic_map(t[i * g.c], abcd.x, abcd.y, abcd.z, abcd.w);
}

// Depth2DepthTransform of one map (PerspectiveMap::Depth2DepthTransform, Depth.cpp:245-274),
// channel 0 of every pixel, in place.
__global__ void __launch_bounds__(kBlock) k_d2d_map(float* __restrict__ data, long long npx,
                                                    int c, float a, float b, float cc, float d)
{
    for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < npx;
         i += (long long)gridDim.x * kBlock)
        data[i * c] = cubic_map(data[i * c], a, b, cc, d);
}

// E->P RGB warp with the GL camera (a18): the taps (corners, weights) come from the host table
// (rgb_taps_host, glibc double atan2 as the oracle); per channel the GL_LINEAR blend in fp32 and
// the round-to-nearest u8 store.
__global__ void __launch_bounds__(kBlock) k_warp_rgb(const RgbTap* __restrict__ taps,
                                                     const TileGeom* __restrict__ geom,
                                                     const long long* __restrict__ rgb_off,
                                                     const uint8_t* __restrict__ pano, int pw,
                                                     int ph, long long pstride,
                                                     uint8_t* __restrict__ tiles,
                                                     long long tstride, int batch)
{
    const int p = blockIdx.y;
    const int W = geom[p].w, H = geom[p].h;
    long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
    if (i >= (long long)W * H) return;
    const RgbTap t = taps[geom[p].pix_off + i];
    const float ax = t.ax, ay = t.ay;
    const long long ix0 = t.x0y0 & 0xFFFFu, iy0 = t.x0y0 >> 16;
    const long long ix1 = t.x1y1 & 0xFFFFu, iy1 = t.x1y1 >> 16;
    long long a00 = (iy0 * pw + ix0) * 3, a01 = (iy0 * pw + ix1) * 3;
    long long a10 = (iy1 * pw + ix0) * 3, a11 = (iy1 * pw + ix1) * 3;
    for (int b = 0; b < batch; b++) {
        const uint8_t* pp = pano + b * pstride;
        uint8_t* out = tiles + b * tstride + rgb_off[p] + i * 3;
        for (int ch = 0; ch < 3; ch++) {
            float t00 = pp[a00 + ch], t01 = pp[a01 + ch], t10 = pp[a10 + ch], t11 = pp[a11 + ch];
            float top = t00 * (1.0f - ax) + t01 * ax;
            float bot = t10 * (1.0f - ax) + t11 * ax;
            float v = top * (1.0f - ay) + bot * ay;
            int q = (int)floorf(v + 0.5f);
            q = q < 0 ? 0 : (q > 255 ? 255 : q);
            out[ch] = (uint8_t)q;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Launchers.
static inline unsigned nblocks(long long n) { return (unsigned)((n + kBlock - 1) / kBlock); }

void launch_seed0(hipStream_t s, const float* emap, int ew, int eh, int ec, long long estride,
                  const GridCol* cols, const GridRow* rows, LevelDims L, float* buf,
                  long long bstride, int batch)
{
    dim3 grid(nblocks((long long)L.w * L.h), batch);
    hipLaunchKernelGGL(k_seed0, grid, dim3(kBlock), 0, s, emap, ew, eh, ec, estride, cols, rows,
                       L, buf, bstride);
}

void launch_upsample(hipStream_t s, const float* prev, long long pstride, LevelDims L,
                     float* buf, long long bstride, int batch)
{
    dim3 grid(nblocks((long long)L.w * L.h), batch);
    hipLaunchKernelGGL(k_upsample, grid, dim3(kBlock), 0, s, prev, pstride, L, buf, bstride);
}

void launch_targets(hipStream_t s, const TileGeom* geom, const TileBox* box, int t0, int t1,
                    const GridCol* cols, const GridRow* rows, const float* tiles,
                    long long tstride, const float* coeffs, int ntiles_total, LevelDims L,
                    float* lnorm, long long lstride, int batch)
{
    dim3 grid(nblocks((long long)L.w * (L.h1 - L.h0 + 1)), batch);
    hipLaunchKernelGGL(k_targets, grid, dim3(kBlock), 0, s, geom, box, t0, t1, cols, rows, tiles,
                       tstride, coeffs, ntiles_total, L, lnorm, lstride);
}

void launch_coverage_rows(hipStream_t s, const TileBox* box, int ntiles, LevelDims L, float* cnt,
                          int r0, int r1)
{
    if (r1 <= r0) return;
    hipLaunchKernelGGL(k_coverage_rows, dim3(nblocks((long long)L.w * (r1 - r0))), dim3(kBlock),
                       0, s, box, ntiles, L, cnt, r0, r1);
}

void launch_rows_add(hipStream_t s, float* dst, const float* src, long long n)
{
    if (n <= 0) return;
    hipLaunchKernelGGL(k_rows_add, dim3(nblocks((n + 3) / 4)), dim3(kBlock), 0, s, dst, src, n);
}

void launch_rows_add_batch(hipStream_t s, const RowsAddBatch& B, int count, long long nmax)
{
    if (count <= 0 || nmax <= 0) return;
    long long nb = (nmax + 4LL * kBlock - 1) / (4LL * kBlock);
    if (nb > 1024) nb = 1024;
    hipLaunchKernelGGL(k_rows_add_batch, dim3((unsigned)nb, (unsigned)count), dim3(kBlock), 0, s, B);
}

void launch_multicover(hipStream_t s, const TileGeom* geom, const int2* pairs, int npairs,
                       int t0, int t1, const GridCol* cols, const GridRow* rows,
                       const float* tiles, const float* coeffs, LevelDims L, float* contrib)
{
    if (npairs <= 0) return;
    hipLaunchKernelGGL(k_multicover_contrib, dim3(nblocks(npairs)), dim3(kBlock), 0, s, geom, pairs,
                       npairs, t0, t1, cols, rows, tiles, coeffs, L, contrib);
}

void launch_multicover_patch(hipStream_t s, const int2* pairs, int npairs, const float* contrib,
                             float* lsum)
{
    if (npairs <= 0) return;
    hipLaunchKernelGGL(k_multicover_patch, dim3(1), dim3(64), 0, s, pairs, npairs, contrib, lsum);
}

void launch_normalize(hipStream_t s, const float* lsum, const float* cnt, LevelDims L,
                      float* lnorm, int r0, int r1)
{
    if (r0 < 0) { r0 = L.h0; r1 = L.h1 + 1; }
    if (r1 <= r0) return;
    dim3 grid(nblocks((long long)L.w * (r1 - r0)));
    hipLaunchKernelGGL(k_normalize, grid, dim3(kBlock), 0, s, lsum, cnt, L, lnorm, r0, r1);
}

void launch_probe_taps(hipStream_t s, const TileGeom* geom, const TileBox* box, int ntiles,
                       const GridCol* cols, const GridRow* rows, LevelDims L, int32_t* out)
{
    dim3 grid(nblocks((long long)L.w * L.h));
    hipLaunchKernelGGL(k_probe_taps, grid, dim3(kBlock), 0, s, geom, box, ntiles, cols, rows, L,
                       out);
}

void launch_jacobi(hipStream_t s, float* buf_a, float* buf_b, const float* lnorm,
                   long long stride, LevelDims L, int iters, int batch, float** result)
{
    dim3 grid(nblocks((long long)L.w * (L.h1 - L.h0 + 1)), batch);
    float* src = buf_a;
    float* dst = buf_b;
    for (int it = 0; it < iters; it++) {
        hipLaunchKernelGGL(k_jacobi, grid, dim3(kBlock), 0, s, src, dst, lnorm, stride, L);
        float* t = src;
        src = dst;
        dst = t;
    }
    *result = src;
}

void launch_quantize(hipStream_t s, const float* buf, long long bstride, int n, uint16_t* out,
                     long long ostride, int batch)
{
    dim3 grid(nblocks(n), batch);
    hipLaunchKernelGGL(k_quantize, grid, dim3(kBlock), 0, s, buf, bstride, n, out, ostride);
}

void launch_register(hipStream_t s, const TileGeom* geom, const RegGrid* grids,
                     const GridCol* rcols, const GridRow* rrows, int ntiles, const float* emap,
                     int ew, int eh, int ec, long long estride, const float* tiles,
                     long long tstride, int degree, int solver, float* coeffs, double* coeffs64,
                     int batch, double* sums, const int* active, const int2* sidx)
{
    dim3 grid((unsigned)(ntiles * batch));
    hipLaunchKernelGGL(k_register, grid, dim3(kRegLanes), 0, s, geom, grids, rcols, rrows,
                       ntiles, emap, ew, eh, ec, estride, tiles, tstride, degree, solver, coeffs,
                       coeffs64, sums, active, sidx);
}

// One thread per registration sample: the tile element (SphericalTo2D, clamp, Value's index) and
// the baseline element (ValueAtCoord's index) of sample s of tile p, exactly as k_register's
// direct path computes them (Depth.cpp:1328-1387).
__global__ void __launch_bounds__(256) k_regidx(const TileGeom* __restrict__ geom,
                                                const RegGrid* __restrict__ grids,
                                                const GridCol* __restrict__ rcols,
                                                const GridRow* __restrict__ rrows, int ew, int eh,
                                                int ec, int2* __restrict__ sidx)
{
    const int p = blockIdx.y;
    const TileGeom g = geom[p];
    const RegGrid rg = grids[p];
    const int ncol = rg.cols + 1;
    const int ns = ncol * (rg.rows + 1);
    for (int s = blockIdx.x * 256 + threadIdx.x; s < ns; s += gridDim.x * 256) {
        const int r = s / ncol, c = s - r * ncol;
        const GridCol cc = rcols[rg.col_off + c];
        const GridRow rr = rrows[rg.row_off + r];
        float x, y;
        sph_to_2d(g, rr.sz, rr.cz, cc.ca, cc.sa, x, y);
        if (x < 0) x = 0;
        if (x > 1) x = 1;
        if (y < 0) y = 0;
        if (y > 1) y = 1;
        sidx[rg.soff + s] = make_int2((int)tile_index(g, x, y),
                                      (int)emap_index(cc.az, rr.zen, ew, eh, ec));
    }
}

void launch_regidx(hipStream_t s, const TileGeom* geom, const RegGrid* grids,
                   const GridCol* rcols, const GridRow* rrows, int ntiles, int max_samples,
                   int ew, int eh, int ec, int2* sidx)
{
    unsigned gx = (unsigned)((max_samples + 255) / 256);
    if (gx < 1) gx = 1;
    if (gx > 1024) gx = 1024;
    hipLaunchKernelGGL(k_regidx, dim3(gx, (unsigned)ntiles), dim3(256), 0, s, geom, grids, rcols,
                       rrows, ew, eh, ec, sidx);
}

int register_sums_per_tile() { return kRegSums; }

void launch_register_joint(hipStream_t s, const double* sums, const int* active, int ntiles,
                           int batch, int degree, int solver, float* coeffs, double* coeffs64)
{
    hipLaunchKernelGGL(k_register_joint, dim3((batch + 63) / 64), dim3(64), 0, s, sums, active,
                       ntiles, batch, degree, solver, coeffs, coeffs64);
}

void launch_apply_cubic(hipStream_t s, const TileGeom* geom, int ntiles, long long tile_elems,
                        float* tiles, long long tstride, const float* coeffs, int batch)
{
    long long per = tile_elems / (ntiles > 0 ? ntiles : 1);
    unsigned gx = nblocks(per);
    if (gx > 1024) gx = 1024;
    if (gx == 0) gx = 1;
    dim3 grid(gx, ntiles, batch);
    hipLaunchKernelGGL(k_apply_cubic, grid, dim3(kBlock), 0, s, geom, ntiles, tiles, tstride,
                       coeffs);
}

void launch_d2d_map(hipStream_t s, float* data, long long npx, int c, const float* abcd)
{
    unsigned gx = nblocks(npx);
    if (gx > 4096) gx = 4096;
    if (gx == 0) gx = 1;
    hipLaunchKernelGGL(k_d2d_map, dim3(gx), dim3(kBlock), 0, s, data, npx, c, abcd[0], abcd[1],
                       abcd[2], abcd[3]);
}

void launch_warp_rgb(hipStream_t s, const RgbTap* taps, const TileGeom* geom, int ntiles,
                     long long npix_max, const long long* rgb_off, const uint8_t* pano, int pw,
                     int ph, long long pstride, uint8_t* tiles, long long tstride, int batch)
{
    dim3 grid(nblocks(npix_max), ntiles);
    hipLaunchKernelGGL(k_warp_rgb, grid, dim3(kBlock), 0, s, taps, geom, rgb_off, pano, pw, ph,
                       pstride, tiles, tstride, batch);
}

}  // namespace pf
