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

void launch_tapmap(hipStream_t s, const TileGeom* geom, const TapBox* tb, int ntiles,
                   long long max_points, const GridCol* cols, const GridRow* rows, int32_t* map)
{
    long long nb = (max_points + 255) / 256;
    if (nb > 4096) nb = 4096;
    if (nb < 1) nb = 1;
    dim3 grid((unsigned)nb, ntiles);
    hipLaunchKernelGGL(k_tapmap, grid, dim3(256), 0, s, geom, tb, ntiles, cols, rows, map);
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
