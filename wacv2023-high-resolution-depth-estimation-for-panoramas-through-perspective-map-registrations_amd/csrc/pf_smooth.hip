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

// Row-band form (round 4, the default): the band's rows are cut into `nb` row blocks of about
// equal masked-pixel counts, and one 256-thread workgroup per (panorama, block) runs the same
// wavefront schedule over its block's pixels, so a panorama's steps spread over nb CUs.  A
// pixel's vertical neighbours may sit in the next block, so before step s a workgroup waits until
// both neighbouring blocks have finished step s-1 -- which orders every cross-block read after
// the write it needs (step s-1) and every write after the neighbour's last read of the old value
// (its step s-1).  The hand-off is MI355X_MICROARCH.md's write-through form: every access to the
// level is sc1 (L1-bypassing, write-through), every storing wave drains (vmcnt(0)), a barrier,
// one agent-scope flag store; one lane polls the two neighbours' flags, a barrier.  Workgroups
// take (panorama, block) from a ticket counter when they start, so a panorama's blocks are held
// by running workgroups and groups fill in ticket order (no co-residency assumption beyond nb
// workgroups).  Waits are bounded: a timeout is counted (and raised to the host's flag) instead
// of hanging the device.  Lists: per block, the masked pixels split by the parity of d = X + Y and
// sorted by d; off[(blk*2 + p)*(nk+1) + k] = first index of d = 2k + p in the block's list.
constexpr int kSB = 256;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t smooth_rsrc(const void* base, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float ld_sc1(__amdgpu_buffer_rsrc_t r, int o)
{
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, 4 * o, 0, 16));
}

__global__ void __launch_bounds__(kSB) k_smooth_band(float* __restrict__ buf,
                                                     const int* __restrict__ list,
                                                     const int* __restrict__ off, int nk, int nb,
                                                     int w, long long npx, int smin, int smax,
                                                     int iters, SmoothSync S)
{
    __shared__ uint32_t lds_ticket;
    __shared__ int lds_gave_up;
    const int tid = threadIdx.x;
    if (tid == 0) lds_gave_up = 0;
    if (tid == 0) lds_ticket = __hip_atomic_fetch_add(S.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const uint32_t tk = __builtin_amdgcn_readfirstlane(lds_ticket - S.tbase);
    const int pano = (int)(tk / (uint32_t)nb), blk = (int)(tk % (uint32_t)nb);
    const auto B = smooth_rsrc(buf + (long long)pano * npx, (uint32_t)(npx * 4));
    uint32_t* const flags = S.flags + (long long)pano * nb;
    const int* const offb = off + (long long)blk * 2 * (nk + 1);
    // after one timed-out wait this workgroup stops waiting: the call's output is already invalid
    // (reported as PF_ETIMEOUT), and every later step would otherwise wait out its own limit
    bool gave_up = false;
    for (int s = smin; s <= smax; s++) {
        if (s > smin && !gave_up) {  // both neighbouring blocks finished step s-1
            if (tid == 0) {
                const uint32_t want = S.fbase + (uint32_t)(s - smin);  // step s-1 done
                for (int nbj = blk - 1; nbj <= blk + 1; nbj += 2) {
                    if (nbj < 0 || nbj >= nb) continue;
                    int spins = 0;
                    while ((int)(__hip_atomic_load(&flags[nbj], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - want) < 0) {
                        __builtin_amdgcn_s_sleep(1);
                        if (++spins > (1 << S.spin_log2)) {
                            __hip_atomic_fetch_add(S.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            if (S.err_host) __hip_atomic_store(S.err_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                            lds_gave_up = 1;
                            break;
                        }
                    }
                }
            }
            __syncthreads();
            gave_up = lds_gave_up != 0;  // uniform: read after the barrier
        }
        const int p = s & 1;
        const int dlo = s - 2 * (iters - 1);
        const int kl = dlo > p ? (dlo - p) >> 1 : 0, kh = min(nk - 1, (s - p) >> 1);
        if (kl <= kh) {
            const int* o2 = offb + p * (nk + 1);
            const int lo = o2[kl], hi = o2[kh + 1];
            for (int j = lo + tid; j < hi; j += kSB) {
                const int o = list[j];
                const float val = ld_sc1(B, o);
                const float v0 = ld_sc1(B, o - 1), v1 = ld_sc1(B, o + 1), v2 = ld_sc1(B, o - w),
                            v3 = ld_sc1(B, o + w);
                const float avg = (((v0 + v1) + v2) + v3) / 4.0f;
                const float nv = (float)((double)val + 0.5 * (double)(avg - val));
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(nv), B, 4 * o, 0, 16);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0 && !(S.fault && blk == 0)) {  // fault hook: block 0 withholds its flag
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(&flags[blk], S.fbase + (uint32_t)(s - smin) + 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

void launch_smooth_band(hipStream_t s, const int* list, const int* off, int nk, int nb, int w,
                        int h, int smin, int smax, int iters, float* buf, int batch,
                        const SmoothSync& S)
{
    hipLaunchKernelGGL(k_smooth_band, dim3((unsigned)(nb * batch)), dim3(kSB), 0, s, buf, list, off,
                       nk, nb, w, (long long)w * h, smin, smax, iters, S);
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
