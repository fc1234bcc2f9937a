// pf_targets.hip -- Laplacian-target scatter (Depth.cpp:1487-1647) as a two-stage gather.
//
// The projection of a fusion-grid point into a tile (SphericalTo2D + Value's truncation,
// Depth.cpp:111-118,168-182) depends only on the layout and the level, never on the panorama,
// and every grid point is a tap of up to five stencils.  So:
//
//  1. k_tapmap (once per layout and level, cached in the context): for every tile p and every
//     grid point of its box plus a one-pixel ring, the tile element index the reference's
//     Value() reads -- five correctly rounded divisions per point, done once instead of five
//     times per pixel and once per panorama.
//  2. k_targets_map (per call): for each band pixel, the covering tiles (index order, as the
//     reference's single-thread accumulation), five index loads from the map, and for
//     kTgtBatch panoramas at a time the five tile gathers (+ the fused Depth2DepthTransform),
//     the weighted sum in std::map key order and the normalisation of Depth.cpp:1626-1647.
#include "pf_internal.hpp"

namespace pf {

static constexpr int kTgtBatch = 8;

__global__ void __launch_bounds__(256) k_tapmap(const TileGeom* __restrict__ geom,
                                                const TapBox* __restrict__ tb, int ntiles,
                                                const GridCol* __restrict__ cols,
                                                const GridRow* __restrict__ rows,
                                                int32_t* __restrict__ map)
{
    const int p = blockIdx.y;
    const TapBox B = tb[p];
    const long long n = (long long)B.nx * B.ny;
    const TileGeom g = geom[p];
    const long long lim = (long long)g.w * g.h * g.c;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
         i += (long long)gridDim.x * 256) {
        int yy = B.ymin + (int)(i / B.nx), xx = B.xmin + (int)(i % B.nx);
        const GridCol c = cols[xx + 1];
        const GridRow r = rows[yy + 1];
        float x, y;
        sph_to_2d(g, r.sz, r.cz, c.ca, c.sa, x, y);
        long long idx = tile_index(g, x, y);
        if (idx < 0) idx = 0;  // out-of-tile tap: the reference reads out of bounds; clamp
        if (idx >= lim) idx = lim - g.c;
        map[B.off + i] = (int32_t)idx;
    }
}

__device__ __forceinline__ bool in_box2(const TileBox& bx, int X, int Y)
{  // X runs x0, x0+xs, ... and stops before x1 (Depth.cpp:1565-1623)
    if (Y < bx.y0 || Y > bx.y1) return false;
    return bx.xs > 0 ? (X >= bx.x0 && X < bx.x1) : (X <= bx.x0 && X > bx.x1);
}

template <bool XFORM>
__global__ void __launch_bounds__(256) k_targets_map(const TileGeom* __restrict__ geom,
                                                     const TileBox* __restrict__ box,
                                                     const TapBox* __restrict__ tb, int ntiles,
                                                     const int32_t* __restrict__ map,
                                                     const float* __restrict__ tiles,
                                                     long long tstride,
                                                     const float* __restrict__ coeffs,
                                                     LevelDims L, float* __restrict__ lnorm,
                                                     long long lstride, int batch)
{
    // XCD-contiguous runs of band rows: the N/C/S taps of neighbouring rows read the same tile
    // lines, and so do horizontally adjacent blocks.
    const unsigned lb = xcd_remap(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y);
    const unsigned bx = lb % gridDim.x, by = lb / gridDim.x;
    const long long i = (long long)bx * 256 + threadIdx.x;
    const long long nband = (long long)L.w * (L.h1 - L.h0 + 1);
    if (i >= nband) return;
    const int Y = (int)(i / L.w) + L.h0, X = (int)(i - (long long)(Y - L.h0) * L.w);
    const long long o = (long long)Y * L.w + X;
    const int bbeg = by * kTgtBatch;
    float acc[kTgtBatch];
#pragma unroll
    for (int q = 0; q < kTgtBatch; q++) acc[q] = 0.0f;
    int n = 0;
    if (Y > L.h0 && Y < L.h1) {
        for (int p = 0; p < ntiles; p++) {
            if (!in_box2(box[p], X, Y)) continue;
            const TapBox B = tb[p];
            const long long base = B.off + (long long)(Y - B.ymin) * B.nx + (X - B.xmin);
            // taps in std::map key order: (X-1,Y), (X,Y-1), (X,Y), (X,Y+1), (X+1,Y)
            const int32_t iw = map[base - 1], in = map[base - B.nx], ic = map[base],
                          is = map[base + B.nx], ie = map[base + 1];
            const long long toff = geom[p].off;
            float v[kTgtBatch][5];
#pragma unroll
            for (int q = 0; q < kTgtBatch; q++) {
                const int b = bbeg + q < batch ? bbeg + q : batch - 1;
                const float* t = tiles + b * tstride + toff;
                v[q][0] = t[iw]; v[q][1] = t[in]; v[q][2] = t[ic]; v[q][3] = t[is]; v[q][4] = t[ie];
            }
#pragma unroll
            for (int q = 0; q < kTgtBatch; q++) {
                if constexpr (XFORM) {
                    const int b = bbeg + q < batch ? bbeg + q : batch - 1;
                    const float4 k = *reinterpret_cast<const float4*>(coeffs + ((long long)b * ntiles + p) * 4);
#pragma unroll
                    for (int m = 0; m < 5; m++) v[q][m] = cubic_map(v[q][m], k.x, k.y, k.z, k.w);
                }
                float Lp = 0;
                Lp += v[q][0] * -0.25f;
                Lp += v[q][1] * -0.25f;
                Lp += v[q][2] * 1.0f;
                Lp += v[q][3] * -0.25f;
                Lp += v[q][4] * -0.25f;
                acc[q] += Lp;
            }
            n++;
        }
    }
    float scale = 1.0f;
    if (n > 1) {
        float center = 0.0f;
        for (int k = 0; k < n; k++) center += 1.0f;
        scale = 1.0f / center;
    }
#pragma unroll
    for (int q = 0; q < kTgtBatch; q++) {
        const int b = bbeg + q;
        if (b >= batch) break;
        float out;
        if (n == 0) out = __uint_as_float(PF_NAN_MARKER);
        else if (n == 1) out = acc[q];
        else out = acc[q] * scale;
        lnorm[b * lstride + o] = out;
    }
}

// ---------------------------------------------------------------------------------------------
// Patch-staged form (the default).  Every fusion-grid point is a tap of up to five stencils, so
// gathering per pixel reads each tile value five times.  Here a block owns a kTPW x kTPH patch of
// band pixels and kTNB panoramas; for every tile whose box meets the patch (index order), the tap
// values of the patch plus a one-pixel ring are gathered once per grid point, transformed once
// (Depth2DepthTransform), staged in LDS, and the five-point stencils read LDS.  The per-pixel
// arithmetic and the tile-order accumulation are exactly those of k_targets_map.
// patch height: 8 rows (2 pixels per thread) stages 1.29 grid points per pixel instead of 1.55
// at 4 rows; measured at C3 (profiles/r02 logs; recipe: tools/gpu_round.sh ab): 4 rows 0.687 ms, 8 rows 0.635, 16 rows 0.670
#ifndef PF_TGT_PH
#define PF_TGT_PH 8
#endif
static constexpr int kTPW = 64, kTPH = PF_TGT_PH;                // patch of kTPW x kTPH pixels
static constexpr int kTPP = kTPW * kTPH / 256;                   // pixels per thread
static constexpr int kTGW = kTPW + 2, kTGH = kTPH + 2, kTG = kTGW * kTGH;  // grid points + ring
#ifndef PF_TGT_NB
#define PF_TGT_NB 8
#endif
static constexpr int kTNB = PF_TGT_NB;                           // panoramas per block
#ifndef PF_TGT_DIAG
#define PF_TGT_DIAG 0  // probes only (wrong output, timing): bit 0 = no tile gathers, bit 1 = no stores
#endif
#ifndef PF_TGT_NT
// nt stores of the target planes keep the tiles' lines in L2 for the neighbouring patches: the
// stage went 0.629-0.633 -> 0.618-0.623 ms per C3 step (profiles/r03/tgt and profiles/r03/jnt; recipe: tools/gpu_round.sh ab, profiles/r03/tgt/);
// 4 / 16 panoramas per block measured 0.639-0.651 / 0.730
#define PF_TGT_NT 1
#endif

// One block's work: patch `pid` of level L for panoramas [bgrp*NB, +NB).
template <bool XFORM, int NB>
__device__ __forceinline__ void targets_patch(const TileGeom* __restrict__ geom,
                                              const TileBox* __restrict__ box,
                                              const TapBox* __restrict__ tb, int ntiles,
                                              const int32_t* __restrict__ map,
                                              const float* __restrict__ tiles, long long tstride,
                                              const float* __restrict__ coeffs, const LevelDims& L,
                                              int npx, int pid, int bgrp,
                                              float* __restrict__ lnorm, long long lstride,
                                              int batch, float (*sv0)[kTG],
                                              const uint32_t* __restrict__ tmask = nullptr,
                                              int nmw = 0, float (*sv1)[kTG] = nullptr)
{
    const int X0 = (pid % npx) * kTPW, Y0 = L.h0 + (pid / npx) * kTPH;
    const int t = threadIdx.x;
    const int X = X0 + (t & (kTPW - 1));
    const int bbeg = bgrp * NB;
    float acc[kTPP][NB];
    int n[kTPP];
#pragma unroll
    for (int j = 0; j < kTPP; j++) {
        n[j] = 0;
#pragma unroll
        for (int q = 0; q < NB; q++) acc[j][q] = 0.0f;
    }
    const int X1 = min(X0 + kTPW - 1, L.w - 1), Y1 = min(Y0 + kTPH - 1, L.h1);
    // one tile's contribution to the patch (tiles come in index order: the reference's
    // accumulation order); `last`: no staging follows, so no barrier after the stencils
    // sv1 (PF_TGT_DBUF): tiles alternate between two staging buffers, so a tile's staging never
    // overwrites what the previous tile's stencils read and one barrier per tile suffices
    int nt = 0;
    auto tile = [&](const int p, const bool last) {
        float (*sv)[kTG] = (sv1 && (nt & 1)) ? sv1 : sv0;
        nt++;
        const TileBox bx = box[p];
        const TapBox B = tb[p];
        const long long toff = geom[p].off;
        float4 k[NB];
        if constexpr (XFORM) {
#pragma unroll
            for (int q = 0; q < NB; q++) {
                const int b = bbeg + q < batch ? bbeg + q : batch - 1;
                k[q] = *reinterpret_cast<const float4*>(coeffs + ((long long)b * ntiles + p) * 4);
            }
        }
        // stage the tap values of the patch + ring that lie in this tile's tap-index map
        for (int g = t; g < kTG; g += 256) {
            const int gx = X0 - 1 + g % kTGW - B.xmin, gy = Y0 - 1 + g / kTGW - B.ymin;
            if (gx < 0 || gx >= B.nx || gy < 0 || gy >= B.ny) continue;
            const int32_t m = map[B.off + (long long)gy * B.nx + gx];
            float v[NB];
#pragma unroll
            for (int q = 0; q < NB; q++) {
                const int b = bbeg + q < batch ? bbeg + q : batch - 1;
                if constexpr ((PF_TGT_DIAG & 1) != 0) v[q] = (float)(m & 1023) * 1e-3f + (float)b;
                else v[q] = tiles[b * tstride + toff + m];
            }
#pragma unroll
            for (int q = 0; q < NB; q++) {
                float x = v[q];
                if constexpr (XFORM) x = cubic_map(x, k[q].x, k[q].y, k[q].z, k[q].w);
                sv[q][g] = x;
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kTPP; j++) {
            const int r = t / kTPW + j * (256 / kTPW);  // row inside the patch
            const int Y = Y0 + r;
            if (X < L.w && Y <= L.h1 && Y > L.h0 && Y < L.h1 && in_box2(bx, X, Y)) {
                const int c = (r + 1) * kTGW + (t & (kTPW - 1)) + 1;  // (X, Y) in the grid
#pragma unroll
                for (int q = 0; q < NB; q++) {
                    // taps in std::map key order: (X-1,Y), (X,Y-1), (X,Y), (X,Y+1), (X+1,Y)
                    float Lp = 0;
                    Lp += sv[q][c - 1] * -0.25f;
                    Lp += sv[q][c - kTGW] * -0.25f;
                    Lp += sv[q][c] * 1.0f;
                    Lp += sv[q][c + kTGW] * -0.25f;
                    Lp += sv[q][c + 1] * -0.25f;
                    acc[j][q] += Lp;
                }
                n[j]++;
            }
        }
        if (!last && !sv1) __syncthreads();  // the next tile's staging overwrites sv
    };
    if (tmask) {  // the host's list of the tiles whose box meets this patch, as mask words
        int left = 0;  // tiles still to come (block-uniform)
        for (int w = 0; w < nmw; w++) left += __builtin_popcount(tmask[(long long)pid * nmw + w]);
        for (int w = 0; w < nmw; w++) {
            uint32_t m = tmask[(long long)pid * nmw + w];  // block-uniform
            while (m) {
                tile(w * 32 + __builtin_ctz(m), --left == 0);
                m &= m - 1;
            }
        }
    } else {
        for (int p = 0; p < ntiles; p++)
            if (box_meets(box[p], X0, X1, Y0, Y1)) tile(p, false);  // block-uniform
    }
#pragma unroll
    for (int j = 0; j < kTPP; j++) {
        const int Y = Y0 + t / kTPW + j * (256 / kTPW);
        if (!(X < L.w && Y <= L.h1)) continue;
        float scale = 1.0f;
        if (n[j] > 1) {
            float center = 0.0f;
            for (int i = 0; i < n[j]; i++) center += 1.0f;
            scale = 1.0f / center;
        }
        const long long o = (long long)Y * L.w + X;
#pragma unroll
        for (int q = 0; q < NB; q++) {
            const int b = bbeg + q;
            if (b >= batch) break;
            float out;
            if (n[j] == 0) out = __uint_as_float(PF_NAN_MARKER);
            else if (n[j] == 1) out = acc[j][q];
            else out = acc[j][q] * scale;
            if constexpr ((PF_TGT_DIAG & 2) != 0) {
                if (out == -12345.0f) lnorm[b * lstride + o] = out;  // probe: no stores
            } else if constexpr (PF_TGT_NT) {
                __builtin_nontemporal_store(out, &lnorm[b * lstride + o]);
            } else {
                lnorm[b * lstride + o] = out;
            }
        }
    }
}

template <bool XFORM, int NB>
__global__ void __launch_bounds__(256) k_targets_patch(const TileGeom* __restrict__ geom,
                                                       const TileBox* __restrict__ box,
                                                       const TapBox* __restrict__ tb, int ntiles,
                                                       const int32_t* __restrict__ map,
                                                       const float* __restrict__ tiles,
                                                       long long tstride,
                                                       const float* __restrict__ coeffs,
                                                       LevelDims L, int npx, int npatch,
                                                       float* __restrict__ lnorm,
                                                       long long lstride, int batch,
                                                       const uint32_t* __restrict__ tmask,
                                                       int nmw)
{
    __shared__ float sv[NB][kTG];
    // XCD-contiguous runs of patches (neighbouring patches read the same tile lines)
    const unsigned lb = xcd_remap(blockIdx.x, gridDim.x);
    const int pid = (int)(lb % (unsigned)npatch), bgrp = (int)(lb / (unsigned)npatch);
    targets_patch<XFORM, NB>(geom, box, tb, ntiles, map, tiles, tstride, coeffs, L, npx, pid, bgrp,
                             lnorm, lstride, batch, sv, tmask, nmw);
}

// Every level's targets in ONE launch (round 4).  The per-level launches each streamed the
// tiles' lines from HBM: the coarse levels sample the same tile areas as the finest one, so the
// stage moved ~2x the tile bytes the finest level needs.  Here the blocks of all levels are
// ordered so that one region of the sphere is gathered at every level within a short window:
// per panorama group, the coarsest level's patch rows define zenith bands, and band by band the
// finest level's patches come first, then each coarser level's patches of the same band (a host
// table of (level, patch) entries).  The XCD-contiguous mapping gives every XCD a contiguous run
// of the table, so a band's lines are re-read from its L2 / the MALL instead of HBM.
#ifndef PF_TGT_DBUF
#define PF_TGT_DBUF 0  // two staging buffers, one barrier per covering tile (A/B)
#endif
template <bool XFORM, int NB>
__global__ void __launch_bounds__(256) k_targets_multi(const TileGeom* __restrict__ geom,
                                                       int ntiles, const float* __restrict__ tiles,
                                                       long long tstride,
                                                       const float* __restrict__ coeffs,
                                                       TgtMulti M, const int2* __restrict__ order,
                                                       int batch)
{
    __shared__ float sv[PF_TGT_DBUF ? 2 * NB : NB][kTG];
    const unsigned lb = xcd_remap(blockIdx.x, gridDim.x);
    const int e = (int)(lb % (unsigned)M.nentries), bgrp = (int)(lb / (unsigned)M.nentries);
    const int2 ent = order[e];  // (level, patch)
    const TgtLevel& T = M.lv[ent.x];
    targets_patch<XFORM, NB>(geom, T.box, T.tb, ntiles, T.map, tiles, tstride, coeffs, T.L, T.npx,
                         ent.y, bgrp, T.lnorm, T.lstride, batch, sv, T.tmask, T.nmw,
                         PF_TGT_DBUF ? sv + NB : nullptr);
}

int targets_patch_w() { return kTPW; }
int targets_patch_h() { return kTPH; }
int targets_batch() { return kTNB; }

void launch_targets_multi(hipStream_t s, const TileGeom* geom, int ntiles, const float* tiles,
                          long long tstride, const float* coeffs, const TgtMulti& M,
                          const int2* order, int batch)
{
    // one panorama (pf_merge, C2 / C5): blocks of one panorama, not kTNB copies of it
    const int nb = batch == 1 ? 1 : kTNB;
    const dim3 g((unsigned)((long long)M.nentries * ((batch + nb - 1) / nb)));
    if (nb == 1 && coeffs)
        hipLaunchKernelGGL((k_targets_multi<true, 1>), g, dim3(256), 0, s, geom, ntiles, tiles,
                           tstride, coeffs, M, order, batch);
    else if (nb == 1)
        hipLaunchKernelGGL((k_targets_multi<false, 1>), g, dim3(256), 0, s, geom, ntiles, tiles,
                           tstride, coeffs, M, order, batch);
    else if (coeffs)
        hipLaunchKernelGGL((k_targets_multi<true, kTNB>), g, dim3(256), 0, s, geom, ntiles, tiles,
                           tstride, coeffs, M, order, batch);
    else
        hipLaunchKernelGGL((k_targets_multi<false, kTNB>), g, dim3(256), 0, s, geom, ntiles,
                           tiles, tstride, coeffs, M, order, batch);
}

void launch_targets_patch(hipStream_t s, const TileGeom* geom, const TileBox* box,
                          const TapBox* tb, int ntiles, const int32_t* map, const float* tiles,
                          long long tstride, const float* coeffs, LevelDims L, float* lnorm,
                          long long lstride, int batch, const uint32_t* tmask, int nmw)
{
    const int npx = (L.w + kTPW - 1) / kTPW;
    const int npy = (L.h1 - L.h0 + 1 + kTPH - 1) / kTPH;
    const int npatch = npx * npy;
    const int nb = batch == 1 ? 1 : kTNB;
    const dim3 g((unsigned)((long long)npatch * ((batch + nb - 1) / nb)));
    if (nb == 1 && coeffs)
        hipLaunchKernelGGL((k_targets_patch<true, 1>), g, dim3(256), 0, s, geom, box, tb, ntiles,
                           map, tiles, tstride, coeffs, L, npx, npatch, lnorm, lstride, batch,
                           tmask, nmw);
    else if (nb == 1)
        hipLaunchKernelGGL((k_targets_patch<false, 1>), g, dim3(256), 0, s, geom, box, tb, ntiles,
                           map, tiles, tstride, coeffs, L, npx, npatch, lnorm, lstride, batch,
                           tmask, nmw);
    else if (coeffs)
        hipLaunchKernelGGL((k_targets_patch<true, kTNB>), g, dim3(256), 0, s, geom, box, tb,
                           ntiles, map, tiles, tstride, coeffs, L, npx, npatch, lnorm, lstride,
                           batch, tmask, nmw);
    else
        hipLaunchKernelGGL((k_targets_patch<false, kTNB>), g, dim3(256), 0, s, geom, box, tb,
                           ntiles, map, tiles, tstride, coeffs, L, npx, npatch, lnorm, lstride,
                           batch, tmask, nmw);
}

void launch_tapmap(hipStream_t s, const TileGeom* geom, const TapBox* tb, int ntiles,
                   long long max_points, const GridCol* cols, const GridRow* rows, int32_t* map)
{
    long long nb = (max_points + 255) / 256;
    if (nb > 4096) nb = 4096;
    if (nb < 1) nb = 1;
    dim3 grid((unsigned)nb, ntiles);
    hipLaunchKernelGGL(k_tapmap, grid, dim3(256), 0, s, geom, tb, ntiles, cols, rows, map);
}

// Partial sums of tiles [t0, t1) for one panorama on rows [r0, r1) of the band (pf_fuse_partial,
// pf_fuse_partial_rows: the sharded fusion): lsum = the tiles' Laplacians added in tile order,
// cnt = how many, with k_targets_map's per-pixel arithmetic.  Staged like targets_patch, for one
// panorama: a block owns one patch of the level's targets grid (kTPW x kTPH from row h0, the
// grid of the host's per-patch tile masks) and, for every tile of the range whose box meets the
// patch (the mask words ANDed with the range, index order), gathers the tap values of the patch
// plus a one-pixel ring once from the tap-index map, transforms them once
// (Depth2DepthTransform), stages them in LDS and reads the five-point stencils from LDS.  The
// launch covers the grid's patch rows that meet [r0, r1).  The per-pixel gather form re-read
// every tile value five times and tested all t1-t0 boxes per pixel: C5 at world 1 spent 1.17 ms
// per panorama in it, against 0.55 ms for the one-call path's k_targets_multi.
template <bool XFORM>
__global__ void __launch_bounds__(256) k_targets_patch_partial(const TileGeom* __restrict__ geom,
                                                               const TileBox* __restrict__ box,
                                                               const TapBox* __restrict__ tb,
                                                               const uint32_t* __restrict__ tmask,
                                                               int nmw, int t0, int t1,
                                                               const int32_t* __restrict__ map,
                                                               const float* __restrict__ tiles,
                                                               const float* __restrict__ coeffs,
                                                               LevelDims L, float* __restrict__ lsum,
                                                               float* __restrict__ cnt, int r0,
                                                               int r1, int npx, int py0)
{
    __shared__ float sv[kTG];
    const unsigned lb = xcd_remap(blockIdx.x, gridDim.x);
    const int px = (int)(lb % (unsigned)npx), py = py0 + (int)(lb / (unsigned)npx);
    const int pid = py * npx + px;
    const int X0 = px * kTPW, Y0 = L.h0 + py * kTPH;
    const int t = threadIdx.x;
    const int X = X0 + (t & (kTPW - 1));
    const int X1 = min(X0 + kTPW - 1, L.w - 1);
    // rows of the patch in [r0, r1) where Depth.cpp has targets (h0 < Y < h1)
    const int ya = max(max(Y0, r0), L.h0 + 1), yb = min(min(Y0 + kTPH - 1, r1 - 1), L.h1 - 1);
    float acc[kTPP], n[kTPP];
#pragma unroll
    for (int j = 0; j < kTPP; j++) acc[j] = n[j] = 0.0f;
    auto tile = [&](const int p) {
        const TileBox bx = box[p];
        const TapBox B = tb[p];
        const float* tv = tiles + geom[p].off;
        float4 k = make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (XFORM) k = *reinterpret_cast<const float4*>(coeffs + (long long)p * 4);
        for (int g = t; g < kTG; g += 256) {
            const int gx = X0 - 1 + g % kTGW - B.xmin, gy = Y0 - 1 + g / kTGW - B.ymin;
            if (gx < 0 || gx >= B.nx || gy < 0 || gy >= B.ny) continue;
            float x = tv[map[B.off + (long long)gy * B.nx + gx]];
            if constexpr (XFORM) x = cubic_map(x, k.x, k.y, k.z, k.w);
            sv[g] = x;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kTPP; j++) {
            const int r = t / kTPW + j * (256 / kTPW);
            const int Y = Y0 + r;
            if (X <= X1 && Y >= ya && Y <= yb && in_box2(bx, X, Y)) {
                const int c = (r + 1) * kTGW + (t & (kTPW - 1)) + 1;
                // taps in std::map key order: (X-1,Y), (X,Y-1), (X,Y), (X,Y+1), (X+1,Y)
                float Lp = 0;
                Lp += sv[c - 1] * -0.25f;
                Lp += sv[c - kTGW] * -0.25f;
                Lp += sv[c] * 1.0f;
                Lp += sv[c + kTGW] * -0.25f;
                Lp += sv[c + 1] * -0.25f;
                acc[j] += Lp;
                n[j] += 1.0f;
            }
        }
        __syncthreads();
    };
    if (ya <= yb && t0 < t1) {
        for (int w = t0 >> 5; w <= (t1 - 1) >> 5; w++) {
            const int lo = max(t0 - 32 * w, 0), hi = min(t1 - 32 * w, 32);
            const uint32_t range = (hi >= 32 ? 0xFFFFFFFFu : ((1u << hi) - 1u)) & ~((1u << lo) - 1u);
            uint32_t m = tmask[(long long)pid * nmw + w] & range;  // block-uniform
            while (m) {
                tile(w * 32 + __builtin_ctz(m));
                m &= m - 1;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < kTPP; j++) {
        const int Y = Y0 + t / kTPW + j * (256 / kTPW);
        if (X > X1 || Y < r0 || Y >= r1 || Y > L.h1) continue;
        const long long o = (long long)Y * L.w + X;
        lsum[o] = acc[j];
        cnt[o] = n[j];
    }
}

hipError_t launch_targets_partial(hipStream_t s, const TileGeom* geom, const TileBox* box,
                                const TapBox* tb, const uint32_t* tmask, int nmw, int t0, int t1,
                                const int32_t* map, const float* tiles, const float* coeffs,
                                LevelDims L, float* lsum, float* cnt, int r0, int r1)
{
    if (r1 <= r0 || L.w <= 0) return hipSuccess;
    // rows of [r0, r1) outside the band [h0, h1]: no targets (zero sums and counts)
    const size_t rowb = sizeof(float) * (size_t)L.w;
    const int za = r0, zb = min(r1, L.h0);
    hipError_t e = hipSuccess;
    if (zb > za) {
        if (e == hipSuccess) e = hipMemsetAsync(lsum + (size_t)za * L.w, 0, rowb * (zb - za), s);
        if (e == hipSuccess) e = hipMemsetAsync(cnt + (size_t)za * L.w, 0, rowb * (zb - za), s);
    }
    const int wa = max(r0, L.h1 + 1), wb = r1;
    if (wb > wa) {
        if (e == hipSuccess) e = hipMemsetAsync(lsum + (size_t)wa * L.w, 0, rowb * (wb - wa), s);
        if (e == hipSuccess) e = hipMemsetAsync(cnt + (size_t)wa * L.w, 0, rowb * (wb - wa), s);
    }
    const int ba = max(r0, L.h0), bb = min(r1, L.h1 + 1);  // band rows of the range
    if (e != hipSuccess || bb <= ba) return e;
    const int npx = (L.w + kTPW - 1) / kTPW;
    const int py0 = (ba - L.h0) / kTPH, py1 = (bb - 1 - L.h0) / kTPH;
    const unsigned g = (unsigned)npx * (unsigned)(py1 - py0 + 1);
    if (coeffs)
        hipLaunchKernelGGL(k_targets_patch_partial<true>, dim3(g), dim3(256), 0, s, geom, box, tb,
                           tmask, nmw, t0, t1, map, tiles, coeffs, L, lsum, cnt, r0, r1, npx, py0);
    else
        hipLaunchKernelGGL(k_targets_patch_partial<false>, dim3(g), dim3(256), 0, s, geom, box, tb,
                           tmask, nmw, t0, t1, map, tiles, coeffs, L, lsum, cnt, r0, r1, npx, py0);
    return hipGetLastError();
}

void launch_targets_map(hipStream_t s, const TileGeom* geom, const TileBox* box,
                        const TapBox* tb, int ntiles, const int32_t* map, const float* tiles,
                        long long tstride, const float* coeffs, LevelDims L, float* lnorm,
                        long long lstride, int batch)
{
    long long nband = (long long)L.w * (L.h1 - L.h0 + 1);
    dim3 grid((unsigned)((nband + 255) / 256), (batch + kTgtBatch - 1) / kTgtBatch);
    if (coeffs)
        hipLaunchKernelGGL(k_targets_map<true>, grid, dim3(256), 0, s, geom, box, tb, ntiles, map,
                           tiles, tstride, coeffs, L, lnorm, lstride, batch);
    else
        hipLaunchKernelGGL(k_targets_map<false>, grid, dim3(256), 0, s, geom, box, tb, ntiles, map,
                           tiles, tstride, coeffs, L, lnorm, lstride, batch);
}

}  // namespace pf
