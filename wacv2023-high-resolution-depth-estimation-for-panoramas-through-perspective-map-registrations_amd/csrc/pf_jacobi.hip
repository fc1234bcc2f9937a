// pf_jacobi.hip -- register-streaming, temporally blocked damped-Jacobi engine for gfx950.
//
// The reference runs `iters` sweeps per level, each a full read-modify-write of the buffer
// (Depth.cpp:1680-1717).  Here one launch ("pass") advances the band by T sweeps:
//
//  * A wave owns a vertical strip of 64*C virtual columns (C per lane) and streams down a chunk
//    of rows.  At step k it loads row k and, for every sweep level t = 1..T, produces row k-t of
//    level t from rows k-t-1..k-t+1 of level t-1, which it keeps in registers (two rows of
//    history per level).  Horizontal neighbours cross lanes with DPP wave_shr/wave_shl moves.
//    No LDS, no barriers: every step issues T*C independent updates.
//  * Columns are "virtual": virtual column x of row Y is linear pixel Y*w + x, so x < 0 or
//    x >= w wraps into the neighbouring row -- exactly the reference's buffer[yy*width + xx]
//    addressing (the seam quirk of SURVEY.md Appendix A item 5 comes out for free).
//  * Each strip carries a halo of Tp >= T virtual columns on both sides and each row chunk a halo
//    of T rows; values in the halo go stale sweep by sweep and are never stored.
//  * Only band pixels (h0*w <= i < (h1+1)*w) are stored.  A band pixel never reads a pixel
//    outside the band (covered pixels sit in rows h0+1..h1-1), so out-of-band cells may hold
//    anything.
//  * The first pass of a level reads its input straight from the level-0 seed (emap gather) or
//    the 2x nearest upsample of the previous level; the last pass of the last level writes the
//    u16 quantisation (Depth.cpp:1721-1736) instead of floats.
//
// Per pixel the arithmetic is the reference's, in its order, fp32, no contraction:
//   Lcur = ((((W*-1/4) + N*-1/4) + Ctr) + S*-1/4) + E*-1/4    (std::map key order)
//   t = b + (L - Lcur)*0.5;  b' = clamp01(t*(1-1e-4) + b*1e-4)
// with Lcur = L = 0 for an un-windowed pixel.  (The reference starts Lcur at 0; 0 + W*-1/4 can
// differ from W*-1/4 only in the sign of a zero, which cannot reach b' because b is never -0.)
#include "pf_internal.hpp"

#include <cstdlib>
#include <cstring>

#ifndef PF_JLAG_WAVES
#define PF_JLAG_WAVES 1  // __launch_bounds__ min waves per SIMD of the lagged kernel
#endif
#ifndef PF_JLAG_STAGEWISE
#define PF_JLAG_STAGEWISE 1
#endif
#ifndef PF_JLAG_LDSL
#define PF_JLAG_LDSL 1  // L rows through a per-wave LDS ring (1) or per-level registers (0)
#endif
#ifndef PF_JLAG_PF
#define PF_JLAG_PF 2  // steps of lead for the input and L row loads (1 or 2)
#endif
#ifndef PF_JLAG_TOUCH
#define PF_JLAG_TOUCH 0  // steps of lead for L2 touch loads (0 = off; measured slower)
#endif

namespace pf {

namespace {

__device__ __forceinline__ float dpp_from_left(float v)
{  // lane i <- lane i-1 (wave_shr:1)
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xF, 0xF, true));
}
__device__ __forceinline__ float dpp_from_right(float v)
{  // lane i <- lane i+1 (wave_shl:1)
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x130, 0xF, 0xF, true));
}

template <int C>
struct Row {
    float v[C];
};

// One damped-Jacobi update of a C-column row segment.
template <int C>
__device__ __forceinline__ Row<C> sweep_row(const Row<C>& n, const Row<C>& c, const Row<C>& s,
                                            const Row<C>& L)
{
    const float reg = (float)1e-4;
    const float reg_ = 1 - reg;
    float west0 = dpp_from_left(c.v[C - 1]);
    float eastC = dpp_from_right(c.v[0]);
    Row<C> o;
#pragma unroll
    for (int j = 0; j < C; j++) {
        float W = j == 0 ? west0 : c.v[j - 1];
        float E = j == C - 1 ? eastC : c.v[j + 1];
        float b = c.v[j];
        // Lcur = (((W*q + N*q) + b) + S*q) + E*q with q = -1/4.  Every product by q (and by 0.5
        // below) is exact -- a power-of-two scaling -- so fl(W*q + N*q) = q*fl(W+N) and
        // fl(a + x*q) = fma(x, q, a): the fused form rounds exactly where the reference rounds.
        // (Exact unless an operand is below 2^-124, which depths in [0,1] never reach here.)
        float cur = __builtin_fmaf(W + n.v[j], -0.25f, b);
        cur = __builtin_fmaf(s.v[j], -0.25f, cur);
        cur = __builtin_fmaf(E, -0.25f, cur);
        // un-windowed pixel (L = marker): Lcur = L = 0, so the step is exactly +0.  Masked
        // with an AND so the compiler keeps this straight-line (no exec-mask branch).
        float d = L.v[j] - cur;
        uint32_t m = __float_as_uint(L.v[j]) == PF_NAN_MARKER ? 0u : 0xFFFFFFFFu;
        d = __uint_as_float(__float_as_uint(d) & m);
        float t = __builtin_fmaf(d, 0.5f, b);  // b + (L - Lcur)*0.5, product exact
        float v = t * reg_ + b * reg;
        // clamp01: b is never -0 or NaN here, so med3 equals the reference's compare chain
        v = __builtin_amdgcn_fmed3f(v, 0.0f, 1.0f);
        o.v[j] = v;
    }
    return o;
}

}  // namespace

// Source of a pass's input rows.
enum { SRC_BUF = 0, SRC_UPSAMPLE = 1, SRC_SEED = 2 };

template <int C, int T, int SRC, bool OUT16>
__global__ void __launch_bounds__(256) k_jstream(JacobiPass P)
{
    const int lane = threadIdx.x & 63;
    const long long job = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (job >= (long long)P.nstrips * P.nchunks) return;  // wave-uniform
    const int b = blockIdx.y;
    const int strip = (int)(job % P.nstrips), chunk = (int)(job / P.nstrips);
    const int w = P.w;
    const int xs0 = strip * P.V - P.Tp + lane * C;  // this lane's first virtual column
    const int vlo = strip * P.V, vhi = min(vlo + P.V, w);
    const int r0 = P.h0 + chunk * P.rows_per_chunk;
    const int r1 = min(r0 + P.rows_per_chunk, P.h1 + 1);
    const long long npx = (long long)w * P.h;

    const float* src = P.src + b * P.sstride;
    const float* prev = P.prev + b * P.pstride;
    const float* emap = P.emap + b * P.estride;
    const float* lnorm = P.lnorm + b * P.lstride;
    float* dst = P.dst + b * P.dstride;
    uint16_t* out = P.out + b * P.ostride;

    auto load_b = [&](int k) {
        Row<C> r;
        if constexpr (SRC == SRC_BUF) {
            long long base = (long long)k * w + xs0;
            base = base < 0 ? 0 : (base > npx - C ? npx - C : base);
            if constexpr (C == 4) {
                float4 q = *reinterpret_cast<const float4*>(src + base);
                r.v[0] = q.x; r.v[1] = q.y; r.v[2] = q.z; r.v[3] = q.w;
            } else if constexpr (C == 2) {
                float2 q = *reinterpret_cast<const float2*>(src + base);
                r.v[0] = q.x; r.v[1] = q.y;
            } else {
#pragma unroll
                for (int j = 0; j < C; j++) r.v[j] = src[base + j];
            }
        } else {
#pragma unroll
            for (int j = 0; j < C; j++) {
                long long i = (long long)k * w + xs0 + j;
                float v = 0.0f;
                if (i >= 0 && i < npx) {
                    int Y = (int)(i / w);
                    int xr = (int)(i - (long long)Y * w);
                    if constexpr (SRC == SRC_UPSAMPLE) {
                        v = prev[(long long)(Y / 2) * (w / 2) + xr / 2];
                    } else if (Y >= P.h0 && Y <= P.h1) {  // level-0 seed (Depth.cpp:1442-1465)
                        v = emap[emap_index(P.cols[xr + 1].az, P.rows[Y + 1].zen, P.ew, P.eh, P.ec)];
                    }
                }
                r.v[j] = v;
            }
        }
        return r;
    };
    auto load_L = [&](int k) {
        Row<C> r;
        long long base = (long long)k * w + xs0;
        base = base < 0 ? 0 : (base > npx - C ? npx - C : base);
        if constexpr (C == 4) {
            float4 q = *reinterpret_cast<const float4*>(lnorm + base);
            r.v[0] = q.x; r.v[1] = q.y; r.v[2] = q.z; r.v[3] = q.w;
        } else if constexpr (C == 2) {
            float2 q = *reinterpret_cast<const float2*>(lnorm + base);
            r.v[0] = q.x; r.v[1] = q.y;
        } else {
#pragma unroll
            for (int j = 0; j < C; j++) r.v[j] = lnorm[base + j];
        }
        return r;
    };

    Row<C> hist[T][2];  // level t: rows (k-2-t, k-1-t) at the start of step k
    Row<C> Lr[T + 1];   // Lr[t] = L of row k-t
#pragma unroll
    for (int t = 0; t < T; t++)
#pragma unroll
        for (int j = 0; j < C; j++) { hist[t][0].v[j] = 0.0f; hist[t][1].v[j] = 0.0f; }
#pragma unroll
    for (int t = 0; t <= T; t++)
#pragma unroll
        for (int j = 0; j < C; j++) Lr[t].v[j] = 0.0f;

    const int kbeg = r0 - T, kend = r1 + T;  // input rows streamed: [kbeg, kend)
    Row<C> nb = load_b(kbeg), nl = load_L(kbeg);
    for (int k = kbeg; k < kend; k++) {
        Row<C> cb = nb;
#pragma unroll
        for (int t = T; t >= 1; t--) Lr[t] = Lr[t - 1];
        Lr[0] = nl;
        if (k + 1 < kend) {  // prefetch the next input row
            nb = load_b(k + 1);
            nl = load_L(k + 1);
        }
        Row<C> newr = cb;  // level 0 row k
#pragma unroll
        for (int t = 1; t <= T; t++) {
            // level t, row k-t, from level t-1 rows k-t-1, k-t, k-t+1
            Row<C> o = sweep_row<C>(hist[t - 1][0], hist[t - 1][1], newr, Lr[t]);
            hist[t - 1][0] = hist[t - 1][1];
            hist[t - 1][1] = newr;
            newr = o;
        }
        const int j = k - T;  // output row of the final level
        if (j >= r0) {
            const long long rowb = (long long)j * w;
#pragma unroll
            for (int q = 0; q < C; q++) {
                int x = xs0 + q;
                if (x >= vlo && x < vhi) {
                    if constexpr (OUT16) {
                        float v = newr.v[q];
                        if (v < 0) v = 0;
                        if (v > 1) v = 1;
                        out[rowb + x] = (uint16_t)(v * 65535.0f);
                    } else
                        dst[rowb + x] = newr.v[q];
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Lagged variant: sweep level t produces row k-2t at step k (two rows behind level t-1 instead
// of one), so every level reads only rows finished in earlier steps and the T*C updates of a
// step are independent (no intra-step dependency chain).  Level t keeps a 3-row ring; input
// rows and the L rows of the next step are loaded one step ahead into double buffers.  The step
// loop is unrolled by 6 (lcm of the ring period 3 and the double-buffer period 2) so every ring
// index is a compile-time constant and no register moves are needed.
template <int C, int T, int SRC, bool OUT16>
struct JLag {
    Row<C> H[T][3];   // H[t][r % 3] = level t row r
    // Input rows are loaded PF steps before their first use: row r lands in In[r % NB] (issued
    // at step r + 1 - PF, consumed at step r + 1).  NB divides the unroll factor 6.
    static constexpr int PF = PF_JLAG_PF, NB = PF_JLAG_PF + 1;
    Row<C> In[NB];
#if PF_JLAG_LDSL
    // L rows live in a per-wave LDS ring of R = 2T+1 rows (row r in slot r % R): each L row is
    // loaded from memory once (one step ahead, into Lin) and read T times from LDS, instead of
    // T global loads per step held in 2*T*C registers.
    static constexpr int R = 2 * T + 1;
    Row<C> Lin[NB];   // L row r lands in Lin[r % NB] (issued at step r - PF), stored to LDS at step r
    float* lring;     // this wave's ring: R rows of 64*C floats
    int lane_c;       // lane * C (LDS column offset)
#else
    Row<C> Lb[2][T];  // Lb[k & 1][t-1] = L row k-2t, for step k
#endif
#if PF_JLAG_TOUCH
    Row<C> Tch[2][2];      // touch-load landing registers (input row, L row)
    uint32_t touch_acc;    // keeps the touch loads alive; never meaningful
#endif
    const JacobiPass* P;
    int w, xs0, vlo, vhi, r0, r1;
    int colbase;   // virtual column of lane 0 (wave-uniform)
    int lo;        // lane * C
    int rlo, rhi;  // rows loads are clamped to (wave-uniform; the host guarantees every row a
                   // valid output depends on lies inside, so clamping only touches halo rows)
    long long npx;
    const float *src, *prev, *emap, *lnorm;
    float* dst;
    uint16_t* out;

    // Row k of a plane: a wave-uniform row pointer (SGPR arithmetic) plus the lane offset, so
    // the loads use the global_load saddr form with no per-lane address math.
    __device__ __forceinline__ Row<C> load_row(const float* base_ptr, int k) const
    {
        Row<C> r;
        int kc = k < rlo ? rlo : (k > rhi ? rhi : k);
        const float* rp = base_ptr + ((long long)kc * w + colbase);
        if constexpr (C == 2) {
            float2 q = *reinterpret_cast<const float2*>(rp + lo);
            r.v[0] = q.x; r.v[1] = q.y;
        } else if constexpr (C == 4) {
            float4 q = *reinterpret_cast<const float4*>(rp + lo);
            r.v[0] = q.x; r.v[1] = q.y; r.v[2] = q.z; r.v[3] = q.w;
        } else {
#pragma unroll
            for (int j = 0; j < C; j++) r.v[j] = rp[lo + j];
        }
        return r;
    }

    __device__ __forceinline__ Row<C> load_input(int k) const
    {
        if constexpr (SRC == SRC_BUF) {
            return load_row(src, k);
        } else {
            Row<C> r;
#pragma unroll
            for (int j = 0; j < C; j++) {
                long long i = (long long)k * w + xs0 + j;
                float v = 0.0f;
                if (i >= 0 && i < npx) {
                    int Y = (int)(i / w);
                    int xr = (int)(i - (long long)Y * w);
                    if constexpr (SRC == SRC_UPSAMPLE) {
                        v = prev[(long long)(Y / 2) * (w / 2) + xr / 2];
                    } else if (Y >= P->h0 && Y <= P->h1) {  // level-0 seed (Depth.cpp:1442-1465)
                        v = emap[emap_index(P->cols[xr + 1].az, P->rows[Y + 1].zen, P->ew, P->eh,
                                            P->ec)];
                    }
                }
                r.v[j] = v;
            }
            return r;
        }
    }

    static constexpr int slot(int ph, int a) { return ((ph - a) % 3 + 3) % 3; }

#if PF_JLAG_LDSL
    // LDS ring slot of row (group base + d); kb = group base mod R (wave-uniform, SALU).
    __device__ __forceinline__ float* lslot(int kb, int d) const
    {
        const int s = (kb + d + 2 * R) % R;  // d >= -2T > -2R
        return lring + s * (64 * C) + lane_c;
    }
    __device__ __forceinline__ void lds_put(float* p, const Row<C>& r) const
    {
        if constexpr (C == 2) *reinterpret_cast<float2*>(p) = make_float2(r.v[0], r.v[1]);
        else if constexpr (C == 4) *reinterpret_cast<float4*>(p) = make_float4(r.v[0], r.v[1], r.v[2], r.v[3]);
        else {
#pragma unroll
            for (int j = 0; j < C; j++) p[j] = r.v[j];
        }
    }
    __device__ __forceinline__ Row<C> lds_get(const float* p) const
    {
        Row<C> r;
        if constexpr (C == 2) {
            float2 q = *reinterpret_cast<const float2*>(p);
            r.v[0] = q.x; r.v[1] = q.y;
        } else if constexpr (C == 4) {
            float4 q = *reinterpret_cast<const float4*>(p);
            r.v[0] = q.x; r.v[1] = q.y; r.v[2] = q.z; r.v[3] = q.w;
        } else {
#pragma unroll
            for (int j = 0; j < C; j++) r.v[j] = p[j];
        }
        return r;
    }
#endif

    // Step k = (group base) + PH; kb = group base mod R (used by the LDS L ring only).
    template <int PH>
    __device__ __forceinline__ void step(int k, int kb)
    {
        // level-0 row k-1 (loaded last step) joins the ring
        H[0][slot(PH, 1)] = In[(PH + NB - 1) % NB];
#if PF_JLAG_LDSL
        // L row k (landed in Lin last step) goes to its ring slot; fetch L row k+1.  The slot
        // is reused by row k+R > k, after every level has read row k (last read at k + 2T).
        lds_put(lslot(kb, PH), Lin[PH % NB]);
        Lin[(PH + PF) % NB] = load_row(lnorm, k + PF);
        Row<C> Lv[T];
#pragma unroll
        for (int t = 1; t <= T; t++) Lv[t - 1] = lds_get(lslot(kb, PH - 2 * t));
#endif
#if PF_JLAG_TOUCH
        // Touch loads: bring the input and L rows PF_JLAG_TOUCH steps ahead into L2 (their
        // first use would otherwise wait on HBM with only one step of lead).  The values are
        // folded into a dummy one step later so the waits never land in this step.
        if constexpr (SRC == SRC_BUF) {
            touch_acc ^= __float_as_uint(Tch[(PH + 1) & 1][0].v[0]) ^
                         __float_as_uint(Tch[(PH + 1) & 1][1].v[0]);
            Tch[PH & 1][0] = load_row(src, k + PF_JLAG_TOUCH);
        } else {
            touch_acc ^= __float_as_uint(Tch[(PH + 1) & 1][1].v[0]);
        }
        Tch[PH & 1][1] = load_row(lnorm, k + PF_JLAG_TOUCH);
#endif
        // loads for the next step: input row k, L rows (k+1) - 2t
        In[(PH + PF - 1) % NB] = load_input(k + PF - 1);
#if !PF_JLAG_LDSL
#pragma unroll
        for (int t = 1; t <= T; t++) Lb[(PH + 1) & 1][t - 1] = load_row(lnorm, k + 1 - 2 * t);
        const Row<C>* Lv = Lb[PH & 1];
#endif
        Row<C> nw[T];
#if PF_JLAG_STAGEWISE
        // Stage-wise over the T*C independent updates of this step, so consecutive VALU
        // instructions belong to different updates (hides the dependent-issue latency).
        float Wl[T], Er[T];
#pragma unroll
        for (int t = 1; t <= T; t++) {
            Wl[t - 1] = dpp_from_left(H[t - 1][slot(PH, 2 * t)].v[C - 1]);
            Er[t - 1] = dpp_from_right(H[t - 1][slot(PH, 2 * t)].v[0]);
        }
        float cur[T][C];
#pragma unroll
        for (int t = 1; t <= T; t++)
#pragma unroll
            for (int j = 0; j < C; j++) {
                const Row<C>& c = H[t - 1][slot(PH, 2 * t)];
                float W = j == 0 ? Wl[t - 1] : c.v[j - 1];
                cur[t - 1][j] = W + H[t - 1][slot(PH, 2 * t + 1)].v[j];
            }
#pragma unroll
        for (int t = 1; t <= T; t++)
#pragma unroll
            for (int j = 0; j < C; j++)
                cur[t - 1][j] = __builtin_fmaf(cur[t - 1][j], -0.25f, H[t - 1][slot(PH, 2 * t)].v[j]);
#pragma unroll
        for (int t = 1; t <= T; t++)
#pragma unroll
            for (int j = 0; j < C; j++)
                cur[t - 1][j] = __builtin_fmaf(H[t - 1][slot(PH, 2 * t - 1)].v[j], -0.25f, cur[t - 1][j]);
#pragma unroll
        for (int t = 1; t <= T; t++)
#pragma unroll
            for (int j = 0; j < C; j++) {
                const Row<C>& c = H[t - 1][slot(PH, 2 * t)];
                float E = j == C - 1 ? Er[t - 1] : c.v[j + 1];
                cur[t - 1][j] = __builtin_fmaf(E, -0.25f, cur[t - 1][j]);
            }
#pragma unroll
        for (int t = 1; t <= T; t++)
#pragma unroll
            for (int j = 0; j < C; j++) {
                const float Lx = Lv[t - 1].v[j];
                float d = Lx - cur[t - 1][j];
                uint32_t m = __float_as_uint(Lx) == PF_NAN_MARKER ? 0u : 0xFFFFFFFFu;
                cur[t - 1][j] = __uint_as_float(__float_as_uint(d) & m);
            }
#pragma unroll
        for (int t = 1; t <= T; t++)
#pragma unroll
            for (int j = 0; j < C; j++) {
                const float b = H[t - 1][slot(PH, 2 * t)].v[j];
                float tt = __builtin_fmaf(cur[t - 1][j], 0.5f, b);
                float v = tt * (1 - (float)1e-4) + b * (float)1e-4;
                nw[t - 1].v[j] = __builtin_amdgcn_fmed3f(v, 0.0f, 1.0f);
            }
#else
#pragma unroll
        for (int t = 1; t <= T; t++)
            nw[t - 1] = sweep_row<C>(H[t - 1][slot(PH, 2 * t + 1)], H[t - 1][slot(PH, 2 * t)],
                                     H[t - 1][slot(PH, 2 * t - 1)], Lv[t - 1]);
#endif
#pragma unroll
        for (int t = 1; t < T; t++) H[t][slot(PH, 2 * t)] = nw[t - 1];
        const int j = k - 2 * T;  // final-level row finished this step
        if (j >= r0 && j < r1) {
            const long long rowb = (long long)j * w + colbase;
#pragma unroll
            for (int q = 0; q < C; q++) {
                int x = xs0 + q;
                if (x >= vlo && x < vhi) {
                    if constexpr (OUT16) {
                        float v = nw[T - 1].v[q];
                        if (v < 0) v = 0;
                        if (v > 1) v = 1;
                        (out + rowb)[lo + q] = (uint16_t)(v * 65535.0f);
                    } else {
                        (dst + rowb)[lo + q] = nw[T - 1].v[q];
                    }
                }
            }
        }
    }
};

template <int C, int T, int SRC, bool OUT16>
__global__ void __launch_bounds__(256, PF_JLAG_WAVES) k_jlag(JacobiPass P)
{
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int job = blockIdx.x * 4 + wave;
    if (job >= P.nstrips * P.nchunks) return;  // wave-uniform
    const int b = blockIdx.y;
    const int strip = job % P.nstrips, chunk = job / P.nstrips;
    JLag<C, T, SRC, OUT16> S;
    S.P = &P;
    S.w = P.w;
    S.colbase = strip * P.V - P.Tp;
    S.lo = lane * C;
    S.rlo = 1;
    S.rhi = P.h - 2;
    S.xs0 = strip * P.V - P.Tp + lane * C;
    S.vlo = strip * P.V;
    S.vhi = min(S.vlo + P.V, P.w);
    S.r0 = P.h0 + chunk * P.rows_per_chunk;
    S.r1 = min(S.r0 + P.rows_per_chunk, P.h1 + 1);
    S.npx = (long long)P.w * P.h;
    S.src = P.src + b * P.sstride;
    S.prev = P.prev + b * P.pstride;
    S.emap = P.emap + b * P.estride;
    S.lnorm = P.lnorm + b * P.lstride;
    S.dst = P.dst + b * P.dstride;
    S.out = P.out + b * P.ostride;
#pragma unroll
    for (int t = 0; t < T; t++)
#pragma unroll
        for (int q = 0; q < 3; q++)
#pragma unroll
            for (int j = 0; j < C; j++) S.H[t][q].v[j] = 0.0f;
    constexpr int NB = JLag<C, T, SRC, OUT16>::NB;
#pragma unroll
    for (int q = 0; q < NB; q++) {
#pragma unroll
        for (int j = 0; j < C; j++) S.In[q].v[j] = 0.0f;
#if PF_JLAG_LDSL
#pragma unroll
        for (int j = 0; j < C; j++) S.Lin[q].v[j] = 0.0f;
#endif
    }
#if !PF_JLAG_LDSL
#pragma unroll
    for (int q = 0; q < 2; q++)
#pragma unroll
        for (int t = 0; t < T; t++)
#pragma unroll
            for (int j = 0; j < C; j++) S.Lb[q][t].v[j] = 0.0f;
#endif
#if PF_JLAG_LDSL
    constexpr int R = JLag<C, T, SRC, OUT16>::R;
    __shared__ float lds_l[4 * R * 64 * C];  // per-wave private rings, no barriers needed
    S.lring = lds_l + wave * (R * 64 * C);
    S.lane_c = lane * C;
#endif
#if PF_JLAG_TOUCH
    S.touch_acc = 0;
#pragma unroll
    for (int q = 0; q < 2; q++)
#pragma unroll
        for (int r = 0; r < 2; r++)
#pragma unroll
            for (int j = 0; j < C; j++) S.Tch[q][r].v[j] = 0.0f;
#endif
    // steps k0 .. kend: level 0 needs rows from r0 - T, the last output row r1-1 finishes at
    // step r1 - 1 + 2T; k0 is rounded down to a multiple of 6 so ring slots are static.
    int kfirst = S.r0 - T - 1;
    int k0 = kfirst - (((kfirst % 6) + 6) % 6);
    int kend = S.r1 + 2 * T;
    // prime the rows the first steps consume before their in-loop loads land (the rest are
    // loaded PF steps ahead inside step()).  With the LDS ring the slots of rows before k0 stay
    // unwritten: they only feed halo/stale cells, exactly like the zero-initialised level rows.
    // k0 is a multiple of 6, so row k0 + r sits in buffer r.
#pragma unroll
    for (int r = 0; r + 1 < JLag<C, T, SRC, OUT16>::PF; r++) S.In[r] = S.load_input(k0 + r);
#if PF_JLAG_LDSL
#pragma unroll
    for (int r = 0; r < JLag<C, T, SRC, OUT16>::PF; r++) S.Lin[r] = S.load_row(S.lnorm, k0 + r);
    int kb = ((k0 % R) + R) % R;
#else
#pragma unroll
    for (int t = 1; t <= T; t++) S.Lb[0][t - 1] = S.load_row(S.lnorm, k0 - 2 * t);
    const int kb = 0;
#endif
    for (int k = k0; k < kend; k += 6) {
        S.template step<0>(k, kb);
        S.template step<1>(k + 1, kb);
        S.template step<2>(k + 2, kb);
        S.template step<3>(k + 3, kb);
        S.template step<4>(k + 4, kb);
        S.template step<5>(k + 5, kb);
#if PF_JLAG_LDSL
        kb = (kb + 6) % R;
#endif
    }
#if PF_JLAG_TOUCH
    // never true for real data (P.w > 0); keeps the touch loads from being optimised away
    if (S.touch_acc == 0x7FBADBAEu && P.w < 0) S.dst[0] = 0.0f;
#endif
}

// Out-of-band rows of a level: 0 (level 0, Depth.cpp:1449-1452) or the nearest upsample of the
// previous level (Depth.cpp:1467-1485); stored to both ping-pong buffers, or quantised into the
// u16 output on the last level.
__global__ void __launch_bounds__(256) k_border(const float* __restrict__ prev, long long pstride,
                                                LevelDims L, float* __restrict__ a,
                                                float* __restrict__ bb, long long stride,
                                                uint16_t* __restrict__ out, long long ostride)
{
    const long long top = (long long)L.h0 * L.w;
    const long long bot = (long long)(L.h - 1 - L.h1) * L.w;
    long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= top + bot) return;
    const int b = blockIdx.y;
    long long o = i < top ? i : (long long)(L.h1 + 1) * L.w + (i - top);
    int y = (int)(o / L.w), x = (int)(o - (long long)y * L.w);
    float v = 0.0f;
    if (prev) v = prev[b * pstride + (long long)(y / 2) * (L.w / 2) + x / 2];
    if (out) {
        float q = v;
        if (q < 0) q = 0;
        if (q > 1) q = 1;
        out[b * ostride + o] = (uint16_t)(q * 65535.0f);
    } else {
        a[b * stride + o] = v;
        bb[b * stride + o] = v;
    }
}

// ---------------------------------------------------------------------------------------------
template <int C, int T, int SRC, bool OUT16>
static void launch_pass_cts(hipStream_t s, const JacobiPass& P, int batch)
{
    static const bool lag = !(getenv("PF_JKERNEL") && strcmp(getenv("PF_JKERNEL"), "stream") == 0);
    long long jobs = (long long)P.nstrips * P.nchunks;
    dim3 grid((unsigned)((jobs + 3) / 4), batch);
    if (lag) hipLaunchKernelGGL((k_jlag<C, T, SRC, OUT16>), grid, dim3(256), 0, s, P);
    else hipLaunchKernelGGL((k_jstream<C, T, SRC, OUT16>), grid, dim3(256), 0, s, P);
}

template <int C, int T>
static void launch_pass_ct(hipStream_t s, const JacobiPass& P, int batch)
{
    if (P.out_mode) {
        if (P.src_mode == SRC_BUF) launch_pass_cts<C, T, SRC_BUF, true>(s, P, batch);
        else if (P.src_mode == SRC_UPSAMPLE) launch_pass_cts<C, T, SRC_UPSAMPLE, true>(s, P, batch);
        else launch_pass_cts<C, T, SRC_SEED, true>(s, P, batch);
    } else {
        if (P.src_mode == SRC_BUF) launch_pass_cts<C, T, SRC_BUF, false>(s, P, batch);
        else if (P.src_mode == SRC_UPSAMPLE) launch_pass_cts<C, T, SRC_UPSAMPLE, false>(s, P, batch);
        else launch_pass_cts<C, T, SRC_SEED, false>(s, P, batch);
    }
}

template <int C>
static void launch_pass_c(hipStream_t s, const JacobiPass& P, int T, int batch)
{
    switch (T) {
        case 1: launch_pass_ct<C, 1>(s, P, batch); break;
        case 2: launch_pass_ct<C, 2>(s, P, batch); break;
        case 4: launch_pass_ct<C, 4>(s, P, batch); break;
        case 5: launch_pass_ct<C, 5>(s, P, batch); break;
        case 8: launch_pass_ct<C, 8>(s, P, batch); break;
        default: launch_pass_ct<C, 10>(s, P, batch); break;
    }
}

bool jstream_supported_T(int T) { return T == 1 || T == 2 || T == 4 || T == 5 || T == 8 || T == 10; }

template <int T>
static int waves_per_cu_t()
{
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &nb, reinterpret_cast<const void*>(k_jlag<2, T, SRC_BUF, false>), 256, 0) != hipSuccess)
        nb = 1;
    return nb * 4;
}

// Resident waves per CU of the pass kernel at depth T (used to size the grid to whole rounds).
int jstream_waves_per_cu(int T)
{
    static int cache[11] = {0};
    if (T < 1 || T > 10) return 4;
    if (!cache[T]) {
        switch (T) {
            case 1: cache[T] = waves_per_cu_t<1>(); break;
            case 2: cache[T] = waves_per_cu_t<2>(); break;
            case 4: cache[T] = waves_per_cu_t<4>(); break;
            case 5: cache[T] = waves_per_cu_t<5>(); break;
            case 8: cache[T] = waves_per_cu_t<8>(); break;
            default: cache[T] = waves_per_cu_t<10>(); break;
        }
    }
    return cache[T];
}

void launch_jstream(hipStream_t s, const JacobiPass& P, int C, int T, int batch)
{
#if PF_JACOBI_C4
    if (C == 4) { launch_pass_c<4>(s, P, T, batch); return; }
#endif
    (void)C;
    launch_pass_c<2>(s, P, T, batch);
}

void launch_border(hipStream_t s, const float* prev, long long pstride, LevelDims L, float* a,
                   float* b, long long stride, uint16_t* out, long long ostride, int batch)
{
    long long n = (long long)(L.h0 + (L.h - 1 - L.h1)) * L.w;
    if (n <= 0) return;
    dim3 grid((unsigned)((n + 255) / 256), batch);
    hipLaunchKernelGGL(k_border, grid, dim3(256), 0, s, prev, pstride, L, a, b, stride, out,
                       ostride);
}

}  // namespace pf
