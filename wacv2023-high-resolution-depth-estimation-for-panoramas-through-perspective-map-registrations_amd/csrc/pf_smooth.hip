// pf_smooth.hip -- SolveDepthBySmoothing (Depth.cpp:1773-1878), the reference's alternate
// solver (dead code in mode 0, kept as an ablation), bit-exact on gfx950.
//
// The reference writes every tile into one full-resolution buffer (a later tile overwrites an
// earlier one, Depth.cpp:1790-1835), marks the pixels within 10 of a tile-box edge, runs 500
// in-place Gauss-Seidel iterations over the marked pixels of rows [height0, height1] in
// row-major order (:1838-1856), and quantises (:1859-1872).
//
//  * k_smooth_map (layout-only): per pixel the last covering tile and its Value() index (the
//    projection of the fusion grid, SphericalTo2D + Value truncation, from the same host sincos
//    tables), and the to-smooth flag.
//  * k_smooth_seed: per panorama the buffer (0 where no tile covers), with the optional
//    Depth2DepthTransform applied on the fly as the fusion does.
//  * k_smooth_iter_list (default) / k_smooth_iter: the Gauss-Seidel sweeps.  Pixel (X, Y) of iteration i reads (X-1, Y) and
//    (X, Y-1) of iteration i and (X+1, Y), (X, Y+1) of iteration i-1, so the lexicographic order
//    is reproduced exactly by the wavefront schedule s = X + Y + 2i: every read comes from step
//    s-1 and is overwritten only at step s+1, and the pixels of one step (X + Y = s - 2i, one
//    parity) never neighbour each other.  One 1024-thread workgroup per panorama walks the
//    ~w + h + 2*iters steps with a barrier between them; a thread owns the columns X = t + 1024k.
//  * the u16 quantisation of every pixel (launch_quantize).
// Update arithmetic as the reference compiles it: avg = (((v0 + v1) + v2) + v3) / 4 in float,
// v' = (float)(v + 0.5 * (double)(avg - v)) -- the 0.5 is a double literal.
#include "pf_internal.hpp"

namespace pf {

__device__ __forceinline__ bool smooth_in_box(const SmoothBox& b, int X, int Y)
{  // X runs x0, x0+xs, ... and stops before x1; Y runs y0..y1 (Depth.cpp:1810-1834)
    if (Y < b.y0 || Y > b.y1) return false;
    return b.xs > 0 ? (X >= b.x0 && X < b.x1) : (X <= b.x0 && X > b.x1);
}

__global__ void __launch_bounds__(256) k_smooth_map(const TileGeom* __restrict__ geom,
                                                    const SmoothBox* __restrict__ box, int ntiles,
                                                    const GridCol* __restrict__ cols,
                                                    const GridRow* __restrict__ rows, int w, int h,
                                                    int2* __restrict__ src,
                                                    uint8_t* __restrict__ mask)
{
    const int i = (int)blockIdx.x * 256 + (int)threadIdx.x;
    if (i >= w * h) return;
    const int Y = i / w, X = i - Y * w;
    int last = -1;
    uint8_t m = 0;
    for (int p = 0; p < ntiles; p++) {  // tile order: the last covering tile's value stays
        const SmoothBox b = box[p];
        if (!smooth_in_box(b, X, Y)) continue;
        last = p;
        if (abs(X - b.x0) <= 10 || abs(X - b.x1) <= 10 || abs(Y - b.y0) <= 10 ||
            abs(Y - b.y1) <= 10)  // to_smooth_range (:1787, :1825)
            m = 1;
    }
    int2 s = make_int2(-1, 0);
    if (last >= 0) {
        const TileGeom g = geom[last];
        const GridCol c = cols[X + 1];
        const GridRow r = rows[Y + 1];
        float x, y;
        sph_to_2d(g, r.sz, r.cz, c.ca, c.sa, x, y);
        long long idx = tile_index(g, x, y);
        const long long lim = (long long)g.w * g.h * g.c;
        if (idx < 0) idx = 0;  // out-of-tile tap: the reference reads out of bounds; clamp
        if (idx >= lim) idx = lim - g.c;
        s = make_int2(last, (int)idx);
    }
    src[i] = s;
    mask[i] = m;
}

__global__ void __launch_bounds__(256) k_smooth_seed(const TileGeom* __restrict__ geom,
                                                     int ntiles, const int2* __restrict__ src,
                                                     int npx, const float* __restrict__ tiles,
                                                     long long tstride,
                                                     const float* __restrict__ coeffs,
                                                     float* __restrict__ buf)
{
    const int i = (int)blockIdx.x * 256 + (int)threadIdx.x;
    if (i >= npx) return;
    const int b = blockIdx.y;
    const int2 s = src[i];
    float v = 0.0f;  // memset(buffer, 0) (:1777)
    if (s.x >= 0) {
        v = tiles[b * tstride + geom[s.x].off + s.y];
        if (coeffs) {
            const float4 k = *reinterpret_cast<const float4*>(coeffs + ((long long)b * ntiles + s.x) * 4);
            v = cubic_map(v, k.x, k.y, k.z, k.w);
        }
    }
    buf[(long long)b * npx + i] = v;
}

__global__ void __launch_bounds__(1024) k_smooth_iter(float* __restrict__ buf,
                                                      const uint8_t* __restrict__ mask, int w,
                                                      int h, int h0, int h1, int iters)
{
    float* B = buf + (long long)blockIdx.x * w * h;
    const int t = threadIdx.x;
    const int smin = 1 + h0, smax = (w - 2) + h1 + 2 * (iters - 1);
    for (int s = smin; s <= smax; s++) {
        for (int X = 1 + t; X <= w - 2; X += 1024) {
            const int top = s - X;  // Y + 2i == top, i in [0, iters)
            int ylo = max(h0, top - 2 * (iters - 1));
            const int yhi = min(h1, top);
            ylo += (top - ylo) & 1;  // Y has the parity of top
            for (int Y = ylo; Y <= yhi; Y += 2) {
                const int o = Y * w + X;
                if (!mask[o]) continue;
                const float val = B[o];
                const float v0 = B[o - 1], v1 = B[o + 1], v2 = B[o - w], v3 = B[o + w];
                const float avg = (((v0 + v1) + v2) + v3) / 4.0f;
                B[o] = (float)((double)val + 0.5 * (double)(avg - val));
            }
        }
        __syncthreads();  // step s's writes are visible to step s+1 (one workgroup, one CU)
    }
}

// The same schedule over a compacted pixel list (the default): the masked pixels of the band,
// split by the parity of d = X + Y and sorted by d, with off[p*nk + k] the first index of
// d = 2k + p (nk + 1 entries per parity).  Step s updates exactly the pixels with
// d in [s - 2(iters-1), s] and d = s (mod 2) -- one contiguous index range -- instead of testing
// every (X, Y) of the diagonal band against the mask (most of which are not smoothed).
// Measured on MI355X (C3 layout, 2048x1024): 426 -> 180 ms at batch 1, 642 -> 256 ms at batch
// 64; 4 or 8 pixels per thread in flight measured the same or slower (tools/smooth_probe.py): the
// one workgroup per panorama is bound by its CU's vector-memory issue, ~2.1k wave-updates of 7
// scattered accesses per step.
__global__ void __launch_bounds__(1024) k_smooth_iter_list(float* __restrict__ buf,
                                                           const int* __restrict__ list,
                                                           const int* __restrict__ off, int nk,
                                                           int w, long long npx, int smin,
                                                           int smax, int iters)
{
    float* B = buf + (long long)blockIdx.x * npx;
    const int t = threadIdx.x;
    for (int s = smin; s <= smax; s++) {
        const int p = s & 1;
        const int dlo = s - 2 * (iters - 1);
        const int kl = dlo > p ? (dlo - p) >> 1 : 0, kh = min(nk - 1, (s - p) >> 1);
        if (kl <= kh) {
            const int* o2 = off + p * (nk + 1);
            const int lo = o2[kl], hi = o2[kh + 1];
            for (int j = lo + t; j < hi; j += 1024) {
                const int o = list[j];
                const float val = B[o];
                const float v0 = B[o - 1], v1 = B[o + 1], v2 = B[o - w], v3 = B[o + w];
                const float avg = (((v0 + v1) + v2) + v3) / 4.0f;
                B[o] = (float)((double)val + 0.5 * (double)(avg - val));
            }
        }
        __syncthreads();  // step s's writes are visible to step s+1 (one workgroup, one CU)
    }
}

void launch_smooth_list(hipStream_t s, const int* list, const int* off, int nk, int w, int h,
                        int smin, int smax, int iters, float* buf, int batch)
{
    hipLaunchKernelGGL(k_smooth_iter_list, dim3(batch), dim3(1024), 0, s, buf, list, off, nk, w,
                       (long long)w * h, smin, smax, iters);
}

void launch_smooth_map(hipStream_t s, const TileGeom* geom, const SmoothBox* box, int ntiles,
                       const GridCol* cols, const GridRow* rows, int w, int h, int2* src,
                       uint8_t* mask)
{
    const int n = w * h;
    hipLaunchKernelGGL(k_smooth_map, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, geom,
                       box, ntiles, cols, rows, w, h, src, mask);
}

void launch_smooth_seed(hipStream_t s, const TileGeom* geom, int ntiles, const int2* src,
                        const float* tiles, long long tstride, const float* coeffs, int w, int h,
                        float* buf, int batch)
{
    const int n = w * h;
    hipLaunchKernelGGL(k_smooth_seed, dim3((unsigned)((n + 255) / 256), batch), dim3(256), 0, s,
                       geom, ntiles, src, n, tiles, tstride, coeffs, buf);
}

void launch_smooth(hipStream_t s, const TileGeom* geom, int ntiles, const int2* src,
                   const uint8_t* mask, const float* tiles, long long tstride,
                   const float* coeffs, int w, int h, int h0, int h1, int iters, float* buf,
                   int batch)
{
    launch_smooth_seed(s, geom, ntiles, src, tiles, tstride, coeffs, w, h, buf, batch);
    hipLaunchKernelGGL(k_smooth_iter, dim3(batch), dim3(1024), 0, s, buf, mask, w, h, h0, h1,
                       iters);
}

}  // namespace pf
