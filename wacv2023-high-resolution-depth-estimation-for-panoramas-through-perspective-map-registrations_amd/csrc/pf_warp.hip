// pf_warp.hip -- E->P depth warp as a region-staged gather for gfx950.
//
// For every tile pixel (X, Y) the reference mapping is ToSphericalCoord (Depth.cpp:157-166):
// corner0 + hedge*x + vedge*y -> WorldToSpherical (Depth.cpp:2960-2971) -> a bilinear sample of
// the panorama at ValueAtCoord's pixel convention (az/2pi*(pw-1), zen/pi*(ph-1)).  That mapping
// depends only on the layout and the panorama size, so it is evaluated once and cached by the
// context, and the per-call kernel does no trigonometry:
//
//  1. k_warp_coords:  per tile pixel the bilinear corner (x0, y0) and weights (fx, fy).
//  2. the host cuts every tile row into aligned strips of kWarpStrip pixels and groups the
//     strips of all tiles by where their corners fall in the panorama: sorted by band of
//     kWarpBand rows, then column, and cut into regions of at most kWarpRegionPx pixels whose
//     joint corner footprint fits one LDS box (pf_api.hip build_warp_regions).
//  3. k_warp_entries: per region its pixels' 16-B entries, strip by strip.
//
// k_warp_depth: one block per (region, chunk of kNB panoramas).  Per panorama the block stages
// the region's box from HBM into LDS with coalesced 16-B row loads, then every pixel reads its
// four corners from LDS.  Input-driven: the strips of overlapping tiles that look at the same
// part of the panorama share one staged box, so each panorama line is fetched about once per
// launch (plus the boxes' overlap, ~7-15 %), where the round-2 patch-per-tile boxes fetched each
// line ~1.8x; and a wave's two strips are two whole 128-B lines of output.  The chunks of one
// region are adjacent in the grid, so a region's entries come from HBM once and from L2 for
// the other chunks.  Strips whose own footprint is too wide for a box (near the poles) form
// "wide" regions served by direct corner gathers.
//
// Edge rule: the reference clamps x1 = min(x0+1, pw-1), y1 = min(y0+1, ph-1).  x0 == pw-1 only
// when px == pw-1 exactly (az < 2*MYPI), i.e. fx == 0, and likewise y0 == ph-1 means fy == 0; the
// neighbour's weight is then exactly zero, so the box may hold any finite value there (the next
// row's first pixel, or 0 past the panorama through the buffer range check).  Inputs are depth
// maps, finite by contract.
#include "pf_internal.hpp"

#include <cfloat>
#include <cstdlib>
#include <type_traits>

namespace pf {

static constexpr int kWB = 256;                          // threads per block
static constexpr int kPx = kWarpRegionPx / kWB;          // pixels per thread
static constexpr int kBoxRows = kWarpRows;
static constexpr int kBoxFloats = kBoxRows * kWarpPitch;  // LDS floats per staged box
#ifndef PF_WARP_BATCH
#define PF_WARP_BATCH 16
#endif
static constexpr int kNB = PF_WARP_BATCH;                // panoramas per block

__device__ __forceinline__ void world_to_sph(float p0, float p1, float p2, float& az,
                                             float& zen)
{  // Depth.cpp:2960-2971, Imath normalize/length; atan2 evaluated in fp64 and rounded
    float l2 = p0 * p0 + p1 * p1 + p2 * p2;
    float l;
    if (l2 < 2.0f * FLT_MIN) {
        float ax = fabsf(p0), ay = fabsf(p1), az_ = fabsf(p2);
        float mx = ax;
        if (mx < ay) mx = ay;
        if (mx < az_) mx = az_;
        if (mx == 0.0f) l = 0.0f;
        else { ax /= mx; ay /= mx; az_ /= mx; l = mx * sqrtf(ax * ax + ay * ay + az_ * az_); }
    } else
        l = sqrtf(l2);
    if (l != 0.0f) { p0 /= l; p1 /= l; p2 /= l; }
    float a = (float)atan2((double)p1, (double)p0);
    float azf = (float)fmod((double)a, 2 * PF_MYPI);
    if (azf < 0) azf = (float)((double)azf + 2 * PF_MYPI);
    float q2 = p0 * p0 + p1 * p1;
    float ql;
    if (q2 < 2.0f * FLT_MIN) {
        float ax = fabsf(p0), ay = fabsf(p1);
        float mx = ax < ay ? ay : ax;
        if (mx == 0.0f) ql = 0.0f;
        else { ax /= mx; ay /= mx; ql = mx * sqrtf(ax * ax + ay * ay); }
    } else
        ql = sqrtf(q2);
    az = azf;
    zen = (float)atan2((double)ql, (double)p2);
}

__device__ __forceinline__ uint32_t mix32(uint32_t x)
{  // lowbias32 finaliser (the oracle's pfo_hash32)
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    x ^= x >> 16;
    return x;
}

// Pass 1: bilinear corner and weights of every tile pixel; wxy = x0 | y0 << 16.
__global__ void __launch_bounds__(kWB) k_warp_coords(const TileGeom* __restrict__ geom, int pw,
                                                     int ph, uint32_t* __restrict__ wxy,
                                                     float2* __restrict__ wfxy)
{
    const int p = blockIdx.y;
    const TileGeom g = geom[p];
    long long npx = (long long)g.w * g.h;
    long long i = (long long)blockIdx.x * kWB + threadIdx.x;
    if (i >= npx) return;
    int Y = (int)(i / g.w), X = (int)(i - (long long)Y * g.w);
    float xf = (float)X / (float)(g.w - 1), yf = (float)Y / (float)(g.h - 1);
    float q0 = g.corner0[0] + g.hedge[0] * xf, q1 = g.corner0[1] + g.hedge[1] * xf,
          q2 = g.corner0[2] + g.hedge[2] * xf;
    q0 = q0 + g.vedge[0] * yf; q1 = q1 + g.vedge[1] * yf; q2 = q2 + g.vedge[2] * yf;
    float az, zen;
    world_to_sph(q0, q1, q2, az, zen);
    float px = (float)((double)az / (2 * PF_MYPI) * (double)(pw - 1));
    float py = (float)((double)zen / PF_MYPI * (double)(ph - 1));
    int x0 = (int)floorf(px), y0 = (int)floorf(py);
    float fx = px - (float)x0, fy = py - (float)y0;
    if (x0 < 0) { x0 = 0; fx = 0; }
    if (y0 < 0) { y0 = 0; fy = 0; }
    if (x0 > pw - 1) { x0 = pw - 1; fx = 0; }
    if (y0 > ph - 1) { y0 = ph - 1; fy = 0; }
    wxy[g.pix_off + i] = (uint32_t)x0 | ((uint32_t)y0 << 16);
    wfxy[g.pix_off + i] = make_float2(fx, fy);
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

struct WarpLanes {  // one thread's kPx pixels, all panorama-invariant
    uint32_t la[kPx];   // LDS float index of corner (x0, y0) in the box
    uint32_t oo[kPx];   // byte offset of the pixel inside one panorama's tile block; past the
                        // block (a dropped buffer store) for lanes without a pixel
    uint32_t hp[kPx];   // mix32(pixel index): the per-pixel half of the noise hash
    uint32_t rs[kPx];   // byte offset of the pixel's slot in one panorama's response row
    f2 wx[kPx], wy[kPx];  // (1-fx, fx), (1-fy, fy)
};

typedef uint32_t u4v __attribute__((ext_vector_type(4)));

// Stage the region box of kNB panoramas through LDS (double-buffered) and interpolate every
// pixel of the region for each.  U = floats per staging unit (4: 16-B loads of a box whose
// origin and row width are whole quads, pw % 4 == 0; 1 otherwise); NS = staging units per
// thread.  Every staging load is issued unconditionally (slots past the box reload a valid unit,
// panoramas past the chunk reload the last one), so the loads for panorama q+2 are in flight
// while panorama q is interpolated.
template <int NS, int U, bool RESP>
__device__ __forceinline__ void warp_region(float* box, const RespK* rk, const WarpRegion& R,
                                            int t, const WarpLanes& W,
                                            const float* __restrict__ pano, long long pstride,
                                            int pw, int ph, float* __restrict__ tiles,
                                            long long tstride, int bbeg, int nb)
{
    uint32_t goff[NS];  // unit e = t + 256*s of the box -> panorama byte offset
    uint32_t loff[NS];  // -> LDS float index
#pragma unroll
    for (int s = 0; s < NS; s++) {
        int e = t + s * kWB;
        e = e < R.units ? e : R.units - 1;
        const int r = e / R.bwu, c = (e - r * R.bwu) * U;
        int row = R.gy0 + r;
        row = row < ph ? row : ph - 1;  // only rows of zero-weight corners are clamped
        int col = R.gx0 + c;
        col = col < pw ? col : col - pw;  // the box wraps in azimuth (quads never straddle)
        goff[s] = (uint32_t)(row * pw + col) * 4u;
        loff[s] = (uint32_t)(r * kWarpPitch + c);
    }
    float stg[2][NS][U];
    const uint32_t pbytes = (uint32_t)(pstride * 4);
    auto fetch = [&](float (*dst)[U], int q) {
        const auto pr = rsrc(pano + (long long)(bbeg + (q < nb ? q : nb - 1)) * pstride, pbytes);
#pragma unroll
        for (int s = 0; s < NS; s++) {
            if constexpr (U == 4) {
                const u4v v = __builtin_amdgcn_raw_buffer_load_b128(pr, (int)goff[s], 0, 0);
#pragma unroll
                for (int j = 0; j < 4; j++) dst[s][j] = __uint_as_float(v[j]);
            } else {
                dst[s][0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(pr, (int)goff[s], 0, 0));
            }
        }
    };
    auto put = [&](float* bx, const float (*src)[U]) {
#pragma unroll
        for (int s = 0; s < NS; s++) {
            if constexpr (U == 4) {
                *(float4*)(bx + loff[s]) = make_float4(src[s][0], src[s][1], src[s][2], src[s][3]);
            } else {
                bx[loff[s]] = src[s][0];
            }
        }
    };
    auto iter = [&](auto parity, int q) {
        constexpr int PA = decltype(parity)::value;
        fetch(stg[PA], q + 2);  // panorama q was put into buffer PA last iteration: reuse stg[PA]
        const float* L = box + PA * kBoxFloats;
        const int b = bbeg + q;
        const auto orr = rsrc(tiles + b * tstride, (uint32_t)(tstride * 4));
        const char* rq = (const char*)(rk + q * kWarpSlots);
        float out[kPx];
#pragma unroll
        for (int k = 0; k < kPx; k += 2) {
            f2 v;
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const float* c = L + W.la[k + j];
                v[j] = bilinear(f2{c[0], c[1]}, f2{c[kWarpPitch], c[kWarpPitch + 1]},
                                W.wx[k + j], W.wy[k + j]);
            }
            if (RESP) {
                const RespK r0 = *(const RespK*)(rq + W.rs[k]);
                const RespK r1 = *(const RespK*)(rq + W.rs[k + 1]);
                const f2 u = f2{noise_top24(W.hp[k], r0.key), noise_top24(W.hp[k + 1], r1.key)};
                const f2 nz = __builtin_elementwise_fma(u, f2{0x1p-23f, 0x1p-23f},
                                                        f2{-1.0f, -1.0f});
                f2 tt = f2{r0.alpha, r1.alpha} * v;
                tt = tt + (f2{r0.kappa, r1.kappa} * v) * v;
                tt = tt + f2{r0.beta, r1.beta};
                v = pk_add_clamp01(tt, f2{r0.sigma, r1.sigma} * nz);
            }
            out[k] = v[0];
            out[k + 1] = v[1];
        }
#pragma unroll
        for (int k = 0; k < kPx; k++)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(out[k]), orr, (int)W.oo[k], 0, 0);
        put(box + (1 - PA) * kBoxFloats, stg[1 - PA]);  // panorama q+1 (past the chunk: unread)
        __syncthreads();
    };
    fetch(stg[0], 0);
    fetch(stg[1], 1);
    put(box, stg[0]);
    __syncthreads();
    for (int q = 0; q < nb; q += 2) {
        iter(std::integral_constant<int, 0>{}, q);
        if (q + 1 < nb) iter(std::integral_constant<int, 1>{}, q + 1);
    }
}

template <int NS, int U>
__device__ __forceinline__ void warp_region_sel(bool resp, float* box, const RespK* rk,
                                                const WarpRegion& R, int t, const WarpLanes& W,
                                                const float* pano, long long pstride, int pw,
                                                int ph, float* tiles, long long tstride, int bbeg,
                                                int nb)
{
    if (resp) warp_region<NS, U, true>(box, rk, R, t, W, pano, pstride, pw, ph, tiles, tstride,
                                       bbeg, nb);
    else warp_region<NS, U, false>(box, rk, R, t, W, pano, pstride, pw, ph, tiles, tstride, bbeg,
                                   nb);
}

__global__ void __launch_bounds__(kWB) k_warp_depth(const TileGeom* __restrict__ geom,
                                                    int ntiles,
                                                    const WarpRegion* __restrict__ regions,
                                                    int nregions,
                                                    const WarpEntry* __restrict__ entries,
                                                    const float* __restrict__ pano, int pw,
                                                    int ph, long long pstride,
                                                    const Resp* __restrict__ resp,
                                                    float* __restrict__ tiles,
                                                    long long tstride, int batch, int order)
{
    __shared__ __attribute__((aligned(16))) float box[2 * kBoxFloats];
    __shared__ RespK rk[kNB * kWarpSlots];  // published by the first barrier inside warp_region
    // the chunks of one region are adjacent, XCD-contiguous runs of regions (sorted by band,
    // then column): neighbouring boxes' shared rows/columns and a region's entries hit in L2
    const unsigned nchunk = (unsigned)((batch + kNB - 1) / kNB);
    const unsigned lb = xcd_remap(blockIdx.x, gridDim.x);
    // by reference: a private copy of tile[] would be indexed dynamically, i.e. live in scratch
    const WarpRegion& R = regions[order ? lb % (unsigned)nregions : lb / nchunk];
    const int chunk = (int)(order ? lb / (unsigned)nregions : lb % nchunk);
    const int t = threadIdx.x;
    const int bbeg = chunk * kNB;
    const int nb = min(kNB, batch - bbeg);

    WarpLanes W;
    int slot[kPx];
    bool ok[kPx];
#pragma unroll
    for (int k = 0; k < kPx; k++) {
        const int e = t + k * kWB;
        W.la[k] = 0; W.wx[k] = f2{1.0f, 0.0f}; W.wy[k] = f2{1.0f, 0.0f};
        W.hp[k] = 0; W.rs[k] = 0; W.oo[k] = 0xFFFFFFF0u;
        slot[k] = 0;
        ok[k] = false;
        if (e < R.n) {
            const WarpEntry E = entries[R.e0 + e];
            if (E.i != 0xFFFFFFFFu) {
                const uint32_t i = E.i & 0xFFFFFFu;
                slot[k] = (int)(E.i >> 24);
                ok[k] = true;
                const TileGeom& g = geom[R.tile[slot[k]]];
                W.la[k] = E.ls;
                W.oo[k] = (uint32_t)(g.off + (long long)i * g.c) * 4u;
                W.hp[k] = mix32(i);
                W.rs[k] = (uint32_t)(slot[k] * sizeof(RespK));
                W.wx[k] = f2{1.0f - E.fx, E.fx};
                W.wy[k] = f2{1.0f - E.fy, E.fy};
            }
        }
    }

    if (R.wide) {  // footprints too wide for a box (near a pole): direct corner gathers
        for (int q = 0; q < nb; q++) {
            const int b = bbeg + q;
            const float* pp = pano + b * pstride;
            float* out = tiles + b * tstride;
#pragma unroll
            for (int k = 0; k < kPx; k++) {
                if (!ok[k]) continue;
                const uint32_t o00 = W.la[k] & 0x3FFFFFFFu, dx = W.la[k] >> 31;
                const uint32_t o10 = o00 + (((W.la[k] >> 30) & 1u) ? (uint32_t)pw : 0u);
                float v = bilinear(f2{pp[o00], pp[o00 + dx]}, f2{pp[o10], pp[o10 + dx]},
                                   W.wx[k], W.wy[k]);
                if (resp) {
                    const RespK r = resp_key(resp, b, ntiles, R.tile[slot[k]]);
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

    if (t < nb * R.nslot) {
        const int q = t / R.nslot, s = t - q * R.nslot;
        rk[q * kWarpSlots + s] = resp_key(resp, bbeg + q, ntiles, R.tile[s]);
    }
    const bool rs = resp != nullptr;
    if ((pw & 3) == 0) {  // quad-aligned boxes: 16-B staging loads
        if (R.units <= kWB) warp_region_sel<1, 4>(rs, box, rk, R, t, W, pano, pstride, pw, ph,
                                                  tiles, tstride, bbeg, nb);
        else warp_region_sel<(kBoxFloats / 4 + kWB - 1) / kWB, 4>(
            rs, box, rk, R, t, W, pano, pstride, pw, ph, tiles, tstride, bbeg, nb);
    } else {
        if (R.units <= 4 * kWB) warp_region_sel<4, 1>(rs, box, rk, R, t, W, pano, pstride, pw, ph,
                                                      tiles, tstride, bbeg, nb);
        else warp_region_sel<(kBoxFloats + kWB - 1) / kWB, 1>(rs, box, rk, R, t, W, pano, pstride,
                                                              pw, ph, tiles, tstride, bbeg, nb);
    }
}

// Per region its pixels' entries (perm: the region's tile pixels as layout-wide pixel indices,
// strip by strip, 0xFFFFFFFF past a strip's end) with the corner's index in the region's box.
__global__ void __launch_bounds__(kWB) k_warp_entries(const TileGeom* __restrict__ geom,
                                                      const WarpRegion* __restrict__ regions,
                                                      const uint32_t* __restrict__ perm,
                                                      const uint32_t* __restrict__ wxy,
                                                      const float2* __restrict__ wfxy, int pw,
                                                      int ph, WarpEntry* __restrict__ entries)
{
    const WarpRegion& R = regions[blockIdx.x];
    for (int e = threadIdx.x; e < R.n; e += kWB) {
        const uint32_t p = perm[R.e0 + e];
        WarpEntry E{0xFFFFFFFFu, 0u, 0.0f, 0.0f};
        if (p != 0xFFFFFFFFu) {
            int slot = 0;
            for (int s = 1; s < R.nslot; s++)
                if ((long long)p >= geom[R.tile[s]].pix_off) slot = s;  // slots in tile order
            const TileGeom& g = geom[R.tile[slot]];
            const uint32_t m = wxy[p];
            const int x0 = (int)(m & 0xFFFFu), y0 = (int)(m >> 16);
            const float2 f = wfxy[p];
            E.i = (p - (uint32_t)g.pix_off) | ((uint32_t)slot << 24);
            if (R.wide) {
                E.ls = (uint32_t)(y0 * pw + x0) | (x0 < pw - 1 ? 1u << 31 : 0u) |
                       (y0 < ph - 1 ? 1u << 30 : 0u);
            } else {
                int dx = x0 - R.gx0;
                if (dx < 0) dx += pw;
                E.ls = (uint32_t)((y0 - R.gy0) * kWarpPitch + dx);
            }
            E.fx = f.x;
            E.fy = f.y;
        }
        entries[R.e0 + e] = E;
    }
}

// ---------------------------------------------------------------------------------------------
void launch_warp_coords(hipStream_t s, const TileGeom* geom, int ntiles, long long npix_max,
                        int pw, int ph, uint32_t* wxy, float* wfxy)
{
    dim3 g1((unsigned)((npix_max + kWB - 1) / kWB), ntiles);
    hipLaunchKernelGGL(k_warp_coords, g1, dim3(kWB), 0, s, geom, pw, ph, wxy, (float2*)wfxy);
}

void launch_warp_entries(hipStream_t s, const TileGeom* geom, const WarpRegion* regions,
                         int nregions, const uint32_t* perm, const uint32_t* wxy,
                         const float* wfxy, int pw, int ph, WarpEntry* entries)
{
    hipLaunchKernelGGL(k_warp_entries, dim3((unsigned)nregions), dim3(kWB), 0, s, geom, regions,
                       perm, wxy, (const float2*)wfxy, pw, ph, entries);
}

void launch_warp_depth(hipStream_t s, const TileGeom* geom, int ntiles, const WarpRegion* regions,
                       int nregions, const WarpEntry* entries, const float* pano, int pw, int ph,
                       long long pstride, const Resp* resp, float* tiles, long long tstride,
                       int batch)
{
    const long long n = (long long)nregions * ((batch + kNB - 1) / kNB);
    static const int order = getenv("PF_WARP_ORDER") ? atoi(getenv("PF_WARP_ORDER")) : 0;
    hipLaunchKernelGGL(k_warp_depth, dim3((unsigned)n), dim3(kWB), 0, s, geom, ntiles, regions,
                       nregions, entries, pano, pw, ph, pstride, resp, tiles, tstride, batch,
                       order);
}

}  // namespace pf
