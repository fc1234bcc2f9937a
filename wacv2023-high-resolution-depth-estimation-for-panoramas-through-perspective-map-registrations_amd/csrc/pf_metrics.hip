// Accuracy metrics of a fused panorama against ground truth:
// ErrorData (Depth.cpp:1980-2213, the u16 result) and ErrorEmap (Depth.cpp:2215-2458, a float
// equirectangular map such as the baseline), with the median-shift (align_way 1) and
// least-squares (align_way 2) alignments.
//
// The reference sorts two std::lists per panorama for the medians and accumulates in fp32 on one
// core.  Here every panorama of a batch is one slice of the grid:
//   * exact medians by a three-pass radix select over order-preserving float keys (11/11/10
//     bits): each pass histograms one digit in LDS (16 KB per block for the two streams gt and
//     given), merges the non-empty bins into a per-panorama global histogram, and one block per
//     (panorama, stream) scans it to fix the digit and the remaining rank.  The result is the
//     element at index n/2 of the sorted list, bit for bit (Depth.cpp:2061-2086);
//   * the error sums in fp64 per block, reduced in a fixed order by one block per panorama, so
//     the result is deterministic (the reference's sequential fp32 sums carry ~1e-5 relative
//     rounding of their own: the parity bar for the means is a tolerance, for the counts and the
//     deltas it is exact).  align_way 2 solves its normal equations in fp64: the reference's
//     fp32 sums drift by percents at 1M samples, so {s, o} are pinned to an fp64 solve.
// Per pixel the work is HBM-bound byte movement (one gt read + one u16/f32 read per pass); no
// MFMA.
#include "pf_internal.hpp"

#include <cstdlib>

namespace pf {

namespace {

constexpr int MB = 256;        // threads per block
constexpr int MNBLK = 128;     // blocks per panorama (fixed: the fp64 reduction order is fixed)
constexpr int HBINS = 2048;    // bins of one radix digit (11 bits)
#ifndef PF_MED_RUN
#define PF_MED_RUN 1           // first-digit histogram: per-thread run counts (else wave ballots)
#endif

struct MArgs {
    const float* gt;
    int gw, gh, gc;
    long long gstride;
    const float* gv;          // ErrorEmap: the given map (channel 0 of gvc)
    const uint16_t* gv16;     // ErrorData: the u16 result
    int w, h, gvc;
    long long vstride;
    int h0, h1;               // rows [h0, h1] inclusive, already clipped to [0, h-1]
    float rx, ry;             // (float)gt.width / (float)w, (float)gt.height / (float)h
    int cap;
    float depth_max;
    int abs_median;           // ErrorEmap skips abs(val0) < 1e-4 in its median pass
    int fast;                 // gt and result share the geometry, 1 channel, 16 B rows: 4 px
                              // per thread with vector loads
};

// Depth.cpp:2033-2053 (ErrorData) / :2248-2268 (ErrorEmap): band row, nearest gt pixel, skip
// invalid gt, cap at 10 m.
// (float)u / 65535.0f, correctly rounded, without the division sequence: one multiply by the
// reciprocal and one fma refinement.  Exhaustively equal to the division for every u in
// [0, 65535] (checked on the host with glibc fmaf: tests/test_oracle_metrics.py).
__device__ __forceinline__ float u16_unit(uint32_t u)
{
    const float rcp = 1.0f / 65535.0f;
    const float x = (float)u;
    const float q = x * rcp;
    return fmaf(fmaf(-q, 65535.0f, x), rcp, q);
}

__device__ __forceinline__ bool finish_px(const MArgs& a, bool abs_skip, float& v0, float& v1)
{
    const float t = abs_skip ? fabsf(v0) : v0;
    if ((double)t < 1e-4) return false;
    if (a.cap) {
        v0 = v0 < a.depth_max ? v0 : a.depth_max;  // MIN2(val, depth_max)
        v1 = v1 < a.depth_max ? v1 : a.depth_max;
    }
    return true;
}

__device__ __forceinline__ bool eval_px(const MArgs& a, int b, int x, int y, bool abs_skip,
                                        float& v0, float& v1)
{
    int X = (int)((float)x * a.rx);
    int Y = (int)((float)y * a.ry);
    X = X < a.gw - 1 ? X : a.gw - 1;
    Y = Y < a.gh - 1 ? Y : a.gh - 1;
    v0 = a.gt[(long long)b * a.gstride + ((long long)Y * a.gw + X) * a.gc];
    if (a.gv16)
        v1 = u16_unit(a.gv16[(long long)b * a.vstride + (long long)y * a.w + x]);
    else
        v1 = a.gv[(long long)b * a.vstride + ((long long)y * a.w + x) * a.gvc];
    return finish_px(a, abs_skip, v0, v1);
}

// Pixels x .. x+3 of row y (x a multiple of 4).  Fast form: one 16 B gt load and one 8 B (u16)
// or 16 B (f32) result load; X == x and Y == y there because the ratios are exactly 1.
__device__ __forceinline__ void eval4(const MArgs& a, int b, int x, int y, bool abs_skip,
                                      float v0[4], float v1[4], bool ok[4])
{
    if (a.fast) {
        if (x >= a.w) {
            for (int k = 0; k < 4; ++k) ok[k] = false, v0[k] = v1[k] = 0.0f;
            return;
        }
        const long long gi = (long long)b * a.gstride + (long long)y * a.w + x;
        const float4 g = *reinterpret_cast<const float4*>(a.gt + gi);
        v0[0] = g.x, v0[1] = g.y, v0[2] = g.z, v0[3] = g.w;
        const long long vi = (long long)b * a.vstride + (long long)y * a.w + x;
        if (a.gv16) {
            const ushort4 u = *reinterpret_cast<const ushort4*>(a.gv16 + vi);
            v1[0] = u16_unit(u.x), v1[1] = u16_unit(u.y);
            v1[2] = u16_unit(u.z), v1[3] = u16_unit(u.w);
        } else {
            const float4 f = *reinterpret_cast<const float4*>(a.gv + vi);
            v1[0] = f.x, v1[1] = f.y, v1[2] = f.z, v1[3] = f.w;
        }
        for (int k = 0; k < 4; ++k) ok[k] = finish_px(a, abs_skip, v0[k], v1[k]);
        return;
    }
    for (int k = 0; k < 4; ++k) {
        v0[k] = v1[k] = 0.0f;
        ok[k] = x + k < a.w && eval_px(a, b, x + k, y, abs_skip, v0[k], v1[k]);
    }
}

__device__ __forceinline__ uint32_t fkey(float v)
{
    uint32_t u = __float_as_uint(v);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ float fkey_inv(uint32_t k)
{
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// Per (panorama, stream): prefix digits so far, remaining rank, element count, final key.
struct SelState {
    uint32_t prefix, rank, n, key;
};

__device__ __forceinline__ int digit_shift(int pass) { return pass == 0 ? 21 : (pass == 1 ? 10 : 0); }
__device__ __forceinline__ uint32_t digit_mask(int pass) { return pass == 2 ? 0x3FFu : 0x7FFu; }

// Histogram increment aggregated over the wave: the top digits of depths cluster in a few bins,
// so when every active lane of the wave hits one bin a single lane adds the count (LDS atomics
// to one address would otherwise serialise 64-fold).  Measured at C3: a loop over up to 4
// distinct bins per wave was slower (298 vs 243 us per pass): the ballots cost more than the
// conflicts they save.
__device__ __forceinline__ void agg_add(uint32_t* h, uint32_t bin, bool active)
{
    const uint64_t m = __ballot(active);
    if (!m) return;
    const int leader = __ffsll((unsigned long long)m) - 1;
    const uint32_t lb = __shfl(bin, leader);
    const uint64_t same = __ballot(active && bin == lb);
    if (same == m) {
        if ((int)(threadIdx.x & 63) == leader) atomicAdd(&h[lb], (uint32_t)__popcll(m));
    } else if (active) {
        atomicAdd(&h[bin], 1u);
    }
}

__global__ __launch_bounds__(MB) void k_med_hist(MArgs a, int pass, const SelState* st,
                                                 uint32_t* hist)
{
    __shared__ uint32_t h[2][HBINS];
    const int b = blockIdx.y;
    for (int i = threadIdx.x; i < 2 * HBINS; i += MB) (&h[0][0])[i] = 0;
    __syncthreads();
    const int sh = digit_shift(pass);
    const uint32_t msk = digit_mask(pass);
    uint32_t pre[2] = {0, 0};
    if (pass > 0) {
        pre[0] = st[b * 2 + 0].prefix;
        pre[1] = st[b * 2 + 1].prefix;
    }
    const int psh = pass == 1 ? 21 : 10;
    // PF_MED_RUN: the top digit of a depth map is spatially coherent, so each thread counts a run
    // of equal bins in a register and adds it to LDS when the bin changes (and once at the end)
    uint32_t rb[2] = {0u, 0u}, rc[2] = {0u, 0u};
    auto run_add = [&](int st, uint32_t bin, bool act) {
        if (!act) return;
        if (rc[st] && bin == rb[st]) {
            ++rc[st];
        } else {
            if (rc[st]) atomicAdd(&h[st][rb[st]], rc[st]);
            rb[st] = bin;
            rc[st] = 1u;
        }
    };
    // rows of the band round-robin over the blocks of this panorama, a row's pixels over the
    // threads; block-uniform trip counts so the wave-aggregated atomics see whole waves
    for (int y = a.h0 + blockIdx.x; y <= a.h1; y += gridDim.x)
        for (int x0 = 0; x0 < a.w; x0 += 4 * MB) {
            float v0[4], v1[4];
            bool ok[4];
            eval4(a, b, x0 + 4 * threadIdx.x, y, a.abs_median != 0, v0, v1, ok);
            for (int k = 0; k < 4; ++k) {
                const uint32_t k0 = fkey(v0[k]), k1 = fkey(v1[k]);
                const bool a0 = ok[k] && (pass == 0 || (k0 >> psh) == pre[0]);
                const bool a1 = ok[k] && (pass == 0 || (k1 >> psh) == pre[1]);
                if (pass == 0 && PF_MED_RUN) {
                    run_add(0, (k0 >> sh) & msk, a0);
                    run_add(1, (k1 >> sh) & msk, a1);
                } else if (pass == 0) {  // the top digit clusters: aggregate over the wave
                    agg_add(h[0], (k0 >> sh) & msk, a0);
                    agg_add(h[1], (k1 >> sh) & msk, a1);
                } else {          // lower digits spread: plain LDS atomics
                    if (a0) atomicAdd(&h[0][(k0 >> sh) & msk], 1u);
                    if (a1) atomicAdd(&h[1][(k1 >> sh) & msk], 1u);
                }
            }
        }
    if (rc[0]) atomicAdd(&h[0][rb[0]], rc[0]);
    if (rc[1]) atomicAdd(&h[1][rb[1]], rc[1]);
    __syncthreads();
    uint32_t* g = hist + (long long)b * 2 * HBINS;
    for (int i = threadIdx.x; i < 2 * HBINS; i += MB) {
        const uint32_t v = (&h[0][0])[i];
        if (v) atomicAdd(&g[i], v);
    }
}

// One block per (panorama, stream): find the bin holding the element of rank `rank`.
__global__ __launch_bounds__(MB) void k_med_scan(int pass, uint32_t* hist, SelState* st)
{
    constexpr int PER = HBINS / MB;  // 8 bins per thread
    __shared__ uint32_t part[MB];
    const int s = blockIdx.x;  // b * 2 + stream
    uint32_t* g = hist + (long long)s * HBINS;
    const int nb = pass == 2 ? 1024 : HBINS;
    uint32_t loc[PER], sum = 0;
    for (int j = 0; j < PER; ++j) {
        const int bin = threadIdx.x * PER + j;
        loc[j] = bin < nb ? g[bin] : 0u;
        sum += loc[j];
    }
    // the next pass histograms into the same bins: each thread clears the bins it read (all
    // HBINS, so the workspace leaves the last pass zeroed as well)
    for (int j = 0; j < PER; ++j) g[threadIdx.x * PER + j] = 0u;
    part[threadIdx.x] = sum;
    __syncthreads();
    // inclusive Hillis-Steele scan over 256 partial sums
    for (int off = 1; off < MB; off <<= 1) {
        const uint32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0u;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    const uint32_t total = part[MB - 1];
    SelState S = st[s];
    if (pass == 0) {
        S.n = total;
        S.rank = total / 2;  // Depth.cpp:2065 count == size()/2
        S.prefix = 0;
    }
    if (S.n == 0) {  // empty list: the reference's median stays 0
        if (threadIdx.x == 0) {
            S.key = fkey(0.0f);
            st[s] = S;
        }
        return;
    }
    const uint32_t excl = threadIdx.x ? part[threadIdx.x - 1] : 0u;
    if (S.rank >= excl && S.rank < part[threadIdx.x]) {
        uint32_t c = excl;
        for (int j = 0; j < PER; ++j) {
            if (S.rank < c + loc[j]) {
                const uint32_t bin = threadIdx.x * PER + j;
                S.rank -= c;
                S.prefix = pass == 0 ? bin : ((S.prefix << (pass == 2 ? 10 : 11)) | bin);
                if (pass == 2) S.key = S.prefix;
                st[s] = S;
                break;
            }
            c += loc[j];
        }
    }
}

__device__ __forceinline__ double wave_sum(double v)
{
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// Depth.cpp:2096-2134 / :2315-2352: least-squares sums (fp64 accumulation of the fp32 terms).
constexpr int NLS = 5;
__global__ __launch_bounds__(MB) void k_ls_sums(MArgs a, double* part)
{
    const int b = blockIdx.y;
    double s[NLS] = {0, 0, 0, 0, 0};
    for (int y = a.h0 + blockIdx.x; y <= a.h1; y += gridDim.x)
    for (int x0 = 4 * threadIdx.x; x0 < a.w; x0 += 4 * MB) {
      float V0[4], V1[4];
      bool ok[4];
      eval4(a, b, x0, y, false, V0, V1, ok);
      for (int k = 0; k < 4; ++k) {
        if (!ok[k]) continue;
        const float v0 = V0[k], v1 = V1[k];
        s[0] += (double)(v1 * v1);
        s[1] += (double)v1;
        s[2] += 1.0;
        s[3] += (double)(v0 * v1);
        s[4] += (double)v0;
      }
    }
    __shared__ double red[MB / 64][NLS];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int k = 0; k < NLS; ++k) {
        const double v = wave_sum(s[k]);
        if (lane == 0) red[wv][k] = v;
    }
    __syncthreads();
    if (threadIdx.x < NLS) {
        double v = 0;
        for (int w = 0; w < MB / 64; ++w) v += red[w][threadIdx.x];
        part[((long long)b * gridDim.x + blockIdx.x) * NLS + threadIdx.x] = v;
    }
}

// Per panorama: the alignment parameters (median shift or {s, o}) in the reference's fp32 forms.
struct Align {
    float shift, s, o, gt_med, gv_med;
};

__global__ __launch_bounds__(64) void k_align(int align_way, const SelState* st,
                                              const double* lspart, int nblk, Align* al)
{
    const int b = blockIdx.x;
    __shared__ double col[NLS];
    if (align_way == 2 && threadIdx.x < NLS) {
        double v = 0;
        for (int i = 0; i < nblk; ++i) v += lspart[((long long)b * nblk + i) * NLS + threadIdx.x];
        col[threadIdx.x] = v;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    Align A{1.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    if (align_way == 1) {
        A.gt_med = fkey_inv(st[b * 2 + 0].key);
        A.gv_med = fkey_inv(st[b * 2 + 1].key);
        A.shift = A.gt_med / A.gv_med;  // Depth.cpp:2088
    } else if (align_way == 2) {
        const double* acc = col;
        // Depth.cpp:2121-2126 in fp64 (the reference's fp32 forms cancel badly at ~1M samples),
        // rounded to the reference's float {s, o}
        const double a00 = acc[0], a01 = acc[1], a11 = acc[2], b0 = acc[3], b1 = acc[4];
        const double det = a00 * a11 - a01 * a01;
        A.s = (float)((a11 * b0 - a01 * b1) / det);
        A.o = (float)((-a01 * b0 + a00 * b1) / det);
    }
    al[b] = A;
}

// Depth.cpp:2140-2203 / :2358-2420: the error terms.
constexpr int NSUM = 8;  // mse, mae, mre, mselog, n, nlog, fail1, fail2 (fail3 in slot 8)
__global__ __launch_bounds__(MB) void k_err_sums(MArgs a, int align_way, const Align* al,
                                                 double* part)
{
    const int b = blockIdx.y;
    const Align A = al[b];
    double s[NSUM + 1] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t cn[5] = {0, 0, 0, 0, 0};  // s[4..8] are counts: integer adds per thread
    for (int y = a.h0 + blockIdx.x; y <= a.h1; y += gridDim.x)
    for (int x0 = 4 * threadIdx.x; x0 < a.w; x0 += 4 * MB) {
      float V0[4], V1[4];
      bool ok[4];
      eval4(a, b, x0, y, false, V0, V1, ok);
      for (int k = 0; k < 4; ++k) {
        if (!ok[k]) continue;
        const float v0 = V0[k];
        float v1 = V1[k];
        if (align_way == 1)
            v1 *= A.shift;
        else if (align_way == 2)
            v1 = v1 * A.s + A.o;
        const float d = v0 - v1;
        s[0] += (double)d * (double)d;          // pow(val0 - val1, 2)
        s[1] += (double)fabsf(d);
        s[2] += (double)(fabsf(d) / v0);
        if ((double)v0 > 1e-4 && (double)v1 > 1e-4) {
            const float lg = log10f(v0) - log10f(v1);
            s[3] += (double)lg * (double)lg;
            ++cn[1];
        }
        if (v0 > 0 && v1 > 0) {
            // MAX2(v0 / v1, v1 / v0) with one division: the quotient of the larger by the
            // smaller is >= 1 and the other <= 1 after rounding (rounding is monotonic), so the
            // max is exactly fl(larger / smaller)
            const float rm = v0 > v1 ? v0 / v1 : v1 / v0;
            cn[2] += (double)rm >= 1.25;
            cn[3] += (double)rm >= 1.5625;
            cn[4] += (double)rm >= 1.953125;
        }
        ++cn[0];
      }
    }
    for (int k = 0; k < 5; ++k) s[4 + k] = (double)cn[k];
    __shared__ double red[MB / 64][NSUM + 1];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int k = 0; k <= NSUM; ++k) {
        const double v = wave_sum(s[k]);
        if (lane == 0) red[wv][k] = v;
    }
    __syncthreads();
    if (threadIdx.x <= NSUM) {
        double v = 0;
        for (int w = 0; w < MB / 64; ++w) v += red[w][threadIdx.x];
        part[((long long)b * gridDim.x + blockIdx.x) * (NSUM + 1) + threadIdx.x] = v;
    }
}

__global__ __launch_bounds__(MB) void k_err_final(const double* part, int nblk, const Align* al,
                                                  pf_metrics* out)
{
    const int b = blockIdx.x;
    __shared__ double col[NSUM + 1];
    // column k summed by the 64 lanes of wave k (strided, then a fixed-shape tree): the order
    // is fixed, so the result is deterministic
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int k = wv; k <= NSUM; k += blockDim.x >> 6) {
        double v = 0;
        for (int i = lane; i < nblk; i += 64) v += part[((long long)b * nblk + i) * (NSUM + 1) + k];
        v = wave_sum(v);
        if (lane == 0) col[k] = v;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    double acc[NSUM + 1];
    for (int k = 0; k <= NSUM; ++k) acc[k] = col[k];
    const int n = (int)acc[4], nlog = (int)acc[5];
    const int f1 = (int)acc[6], f2 = (int)acc[7], f3 = (int)acc[8];
    pf_metrics m;
    m.mse = (float)acc[0] / (float)n;  // Depth.cpp:2206-2212
    m.mae = (float)acc[1] / (float)n;
    m.mre = (float)acc[2] / (float)n;
    m.mselog = (float)acc[3] / (float)nlog;
    m.delta1 = (float)(n - f1) / (float)n;
    m.delta2 = (float)(n - f2) / (float)n;
    m.delta3 = (float)(n - f3) / (float)n;
    const Align A = al[b];
    m.median_shift = A.shift;
    m.ls_s = A.s;
    m.ls_o = A.o;
    m.gt_median = A.gt_med;
    m.given_median = A.gv_med;
    m.n = n;
    m.nlog = nlog;
    m.reserved[0] = m.reserved[1] = 0;
    out[b] = m;
}

// ---------------------------------------------------------------------------------------------
// The reference's own summation order (pf_set_metrics_order(PF_METRICS_SEQUENTIAL)).  The
// reference accumulates in row-major order into floats: mse and mselog through a double
// (`mse += pow(val0 - val1, 2)` is float = (float)((double)float + double)), mae and mre in
// float, the least-squares sums a_00..b_1 in float (Depth.cpp:2119-2123, 2178-2186).  Each
// pixel's terms are computed in parallel (k_seq_terms) and written in that order; one lane per
// plane then adds them in sequence (k_ls_seq / k_err_seq, below).  A pixel that the reference skips
// contributes exact zeros (x + 0 == x for every finite x >= 0), so the lanes need no masks; the
// counts (n, nlog, delta fails) are integers and stay in the parallel pass (k_err_sums).
struct SeqTerms {  // four planes per panorama: component k of band pixel i = (y - h0) * w + x of
                  // panorama b at t[(b * 4 + k) * bandp + i] (bandp = band rounded up to 4)
    float* t;     // ERR: {d, |d|, |d| / v0, lg} (d, lg = 0 where skipped; the double squares
                  //      (double)d * (double)d and (double)lg * (double)lg are exact);
                  // LS:  {v1 * v1, v1, v0 * v1, v0} (0 where skipped; v0 > 0 where compared)
    long long bandp;
};

// one pixel's four terms (the SeqTerms plane layout), v0 / v1 / ok from eval4
template <bool LS>
__device__ __forceinline__ float4 seq_px(float v0, float v1, bool ok, int align_way, const Align& A)
{
    float4 o = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (LS) {
        if (ok) o = make_float4(v1 * v1, v1, v0 * v1, v0);
    } else if (ok) {
        if (align_way == 1)
            v1 *= A.shift;
        else if (align_way == 2)
            v1 = v1 * A.s + A.o;
        const float d = v0 - v1;
        o.x = d;
        o.y = fabsf(d);
        o.z = fabsf(d) / v0;
        if ((double)v0 > 1e-4 && (double)v1 > 1e-4) o.w = log10f(v0) - log10f(v1);
    }
    return o;
}

template <bool LS>
__global__ __launch_bounds__(MB) void k_seq_terms(MArgs a, int align_way, const Align* al,
                                                  SeqTerms T, long long band)
{
    const int b = blockIdx.y;
    const Align A = al ? al[b] : Align{1.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    for (int y = a.h0 + blockIdx.x; y <= a.h1; y += gridDim.x)
    for (int x0 = 4 * threadIdx.x; x0 < a.w; x0 += 4 * MB) {
      float V0[4], V1[4];
      bool ok[4];
      eval4(a, b, x0, y, false, V0, V1, ok);
      float* pl = T.t + (long long)b * 4 * T.bandp;
      for (int k = 0; k < 4 && x0 + k < a.w; ++k) {
        const long long i = (long long)(y - a.h0) * a.w + x0 + k;
        const float4 o = seq_px<LS>(V0[k], V1[k], ok[k], align_way, A);
        pl[i] = o.x;
        pl[T.bandp + i] = o.y;
        pl[2 * T.bandp + i] = o.z;
        pl[3 * T.bandp + i] = o.w;
      }
    }
}

// The sequential sums.  The reference's accumulators are floats: for a float term the double sum
// rounded to float IS the float sum (double rounding is innocuous for + of two floats), so mae,
// mre and the least-squares sums are one dependent fp32 add per pixel.  mse and mselog add an
// exact double square, acc = (float)((double)acc + (double)v * (double)v), whose cvt/add-f64/cvt
// chain costs ~38 cycles per pixel; there the wave runs the single-rounding fma(v, v, acc) -- equal
// to the reference except when the double sum lands exactly on a float tie -- and then checks
// every step of the chunk in parallel (lane l recomputes the reference's step j = l, l + 64, ...
// from the stored previous value).  All steps before the first mismatch are exact by induction;
// from a mismatch on (rare: ~2^-29 per step) the lane recomputes the rest of the chunk with the
// reference's formula, so the result is the reference's in every case.
//
// One wave streams NPL of the panorama's term planes through LDS in chunks of SCH pixels (16 B
// per lane per load, the next chunk's loads in flight while the current one is added); lane
// k < NPL adds plane pid[k] in row-major order.
#ifndef PF_SEQ_SB
#define PF_SEQ_SB 0  // schedule barrier after the chain's next-group LDS reads (A/B knob)
#endif
#ifndef PF_SEQ_GRP
#define PF_SEQ_GRP 64  // pixels per chain group (one LDS round trip each; one checked per lane)
#endif
constexpr int SCH = 1024, SPS = SCH + 16;  // LDS plane stride: the lanes' planes in different banks

__device__ __forceinline__ void wave_sync()
{  // one wave's LDS operations complete in order: wait for this lane's LDS operations and keep
   // the compiler from moving memory operations across.  A wavefront-scope fence would also
   // wait for the next chunk's global loads in flight (vmcnt(0)), stalling every chunk.
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ float sq_step(float acc, float v)
{  // the reference's step for a squared term (Depth.cpp:2178-2186: mse += pow(d, 2))
    const double t = (double)v;
    return (float)((double)acc + t * t);
}

// SQ: NPL == 2 squared planes (fast fma chain + verification, accb = 2 x SCH floats of LDS);
// else plain float adds.  cnt (all lanes): number of positive terms of plane pid[NPL - 1].
// SQ (NPL == 1): one squared plane per wave, every lane runs the same chain; lane g keeps the
// chain's value at the end of GRP-pixel group g of the chunk, so the check is one group per lane
// (from the previous group's end value, the reference's GRP steps must reach this group's end
// value) with no LDS writes on the chain's path.  Matching group ends make the chunk's result
// the reference's by induction, whatever the steps inside did.  force (tests): one group per
// chunk counts as a mismatch, so the exact redo path runs.
constexpr int SNM = SCH / 256;  // 4-pixel groups per lane per chunk

// Where a chain's chunks come from.  PlaneSrc: the term planes k_seq_terms wrote (any geometry).
// InputSrc (round 6, MArgs::fast geometry): the terms computed from the inputs in the staging
// step -- the chunk's gt / result loads are issued a chunk ahead (load) and the terms formed as
// the chunk is staged to LDS (put) -- so no term planes are written or re-read (3.8 GB -> the
// inputs' 6-8 B per pixel at C3).  Both stage band pixel c * SCH + u * 256 + lane * 4 + k of
// plane pid[p] at L[p * SPS + u * 256 + lane * 4 + k], zeros past the band.
template <int NPL>
struct PlaneSrc {
    static constexpr int NBUF = NPL;  // planes per LDS buffer (the wave's own)
    const float* pl;
    long long bandp;
    float4 R[NPL][SNM];
    __device__ __forceinline__ int boff(int p, const int (&)[NPL]) const { return p; }
    __device__ __forceinline__ void sync() const { wave_sync(); }
    __device__ __forceinline__ void load(long long c, const int (&pid)[NPL], int lane)
    {
#pragma unroll
        for (int p = 0; p < NPL; ++p)
#pragma unroll
            for (int u = 0; u < SNM; ++u) {
                const long long off = c * SCH + u * 256 + lane * 4;  // < bandp => off + 3 < bandp
                R[p][u] = off < bandp ? *reinterpret_cast<const float4*>(pl + pid[p] * bandp + off)
                                      : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            }
    }
    __device__ __forceinline__ void put(float* L, const int (&pid)[NPL], int lane) const
    {
#pragma unroll
        for (int p = 0; p < NPL; ++p)
#pragma unroll
            for (int u = 0; u < SNM; ++u)
                *reinterpret_cast<float4*>(L + p * SPS + u * 256 + lane * 4) = R[p][u];
    }
};

// SharedSrc: the block's producer waves (seq_produce) stage all four term planes of each chunk
// in a shared double buffer; the chain waves read their planes from it and sync with the block
template <int NPL>
struct SharedSrc {
    static constexpr int NBUF = 4;
    __device__ __forceinline__ void load(long long, const int (&)[NPL], int) {}
    __device__ __forceinline__ void put(float*, const int (&)[NPL], int) const {}
    __device__ __forceinline__ int boff(int p, const int (&pid)[NPL]) const { return pid[p]; }
    __device__ __forceinline__ void sync() const { __syncthreads(); }
};

// Producer wave pw of NP: the terms of chunk c (band pixels c * SCH ..), computed from gt and the
// result (MArgs::fast: 16-B gt rows, w % 4 == 0, so a lane's 4 pixels share a row), all four
// planes at L[k * SPS + u * 256 + lane * 4 + j]; zeros past the band.  Same per-pixel
// arithmetic as k_seq_terms (eval4's fast form + seq_px), so the terms are bit-identical.
template <bool LS>
__device__ __forceinline__ void seq_produce(const MArgs& m, int b, int align_way, const Align& A,
                                            long long band, long long c, float* L, int pw, int np,
                                            int lane)
{
    for (int u = pw; u < SNM; u += np) {
        const long long i0 = c * SCH + u * 256 + lane * 4;
        float4 o[4];
        if (i0 < band) {
            const int r = (int)(i0 / m.w);
            const long long px = (long long)(m.h0 + r) * m.w + (i0 - (long long)r * m.w);
            const float4 g = *reinterpret_cast<const float4*>(m.gt + (long long)b * m.gstride + px);
            const float G[4] = {g.x, g.y, g.z, g.w};
            float V[4];
            if (m.gv16) {
                const uint2 q = *reinterpret_cast<const uint2*>(m.gv16 + (long long)b * m.vstride + px);
                V[0] = u16_unit(q.x & 0xFFFFu), V[1] = u16_unit(q.x >> 16);
                V[2] = u16_unit(q.y & 0xFFFFu), V[3] = u16_unit(q.y >> 16);
            } else {
                const float4 f = *reinterpret_cast<const float4*>(m.gv + (long long)b * m.vstride + px);
                V[0] = f.x, V[1] = f.y, V[2] = f.z, V[3] = f.w;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float v0 = G[j], v1 = V[j];
                const bool ok = finish_px(m, false, v0, v1);
                o[j] = seq_px<LS>(v0, v1, ok, align_way, A);
            }
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        }
        float* q = L + u * 256 + lane * 4;
        *reinterpret_cast<float4*>(q) = make_float4(o[0].x, o[1].x, o[2].x, o[3].x);
        *reinterpret_cast<float4*>(q + SPS) = make_float4(o[0].y, o[1].y, o[2].y, o[3].y);
        *reinterpret_cast<float4*>(q + 2 * SPS) = make_float4(o[0].z, o[1].z, o[2].z, o[3].z);
        *reinterpret_cast<float4*>(q + 3 * SPS) = make_float4(o[0].w, o[1].w, o[2].w, o[3].w);
    }
}

// the producer waves' side of seq_chain's loop: one barrier before the first chunk and one per
// chunk, as the chain waves (SharedSrc::sync)
template <bool LS>
__device__ __forceinline__ void seq_producers(const MArgs& m, int b, int align_way, const Align& A,
                                              long long band, float* lds, int pw, int np, int lane)
{
    const long long nch = (band + SCH - 1) / SCH;
    if (nch == 0) return;
    seq_produce<LS>(m, b, align_way, A, band, 0, lds, pw, np, lane);
    __syncthreads();
    for (long long c = 0; c < nch; ++c) {
        if (c + 1 < nch)
            seq_produce<LS>(m, b, align_way, A, band, c + 1, lds + ((c + 1) & 1) * (4 * SPS), pw,
                            np, lane);
        __syncthreads();
    }
}

template <int NPL, bool SQ, class Src>
__device__ __forceinline__ float seq_chain(Src& src, long long band, const int (&pid)[NPL],
                                           float* lds, uint32_t* cnt, int force = 0)
{
    static_assert(!SQ || NPL == 1, "one squared chain per wave");
    constexpr int GRP = PF_SEQ_GRP, GQ = GRP / 4;  // pixels, float4 reads per group
    static_assert(SCH % GRP == 0 && SCH / GRP <= 64, "at most one group per lane");
    const int lane = threadIdx.x & 63;
    auto load = [&](long long c) { src.load(c, pid, lane); };
    auto put = [&](float* L) { src.put(L, pid, lane); };
    const int my = lane < NPL ? lane : 0;
    float acc = 0.0f;
    uint32_t pos = 0;
    const long long nch = (band + SCH - 1) / SCH;
    if (nch == 0) {
        if (cnt) *cnt = 0;
        return acc;
    }
    load(0);
    put(lds);
    src.sync();
    for (long long c = 0; c < nch; ++c) {
        if (c + 1 < nch) load(c + 1);
        const float* L = lds + (c & 1) * (Src::NBUF * SPS);
        const float* Lm = L + src.boff(my, pid) * SPS;
        const int n = (int)(band - c * SCH < SCH ? band - c * SCH : SCH);
        if (SQ && n < SCH) {  // the band's last, partial chunk: the reference's steps directly
            for (int j = 0; j < n; ++j) acc = sq_step(acc, Lm[j]);
        } else {
            const float st = acc;
            float mine = 0.0f;  // SQ: lane g holds the value at the end of group g
            // 16 pixels per group; the next group's LDS reads are issued before this group's
            // chain.  Reads past n stay inside the SPS-padded planes.
            int j = 0;
            if (n >= GRP) {
                float4 cur[GQ];
#pragma unroll
                for (int k = 0; k < GQ; ++k) cur[k] = *reinterpret_cast<const float4*>(Lm + 4 * k);
                for (; j + GRP <= n; j += GRP) {
                    float4 nxt[GQ];
#pragma unroll
                    for (int k = 0; k < GQ; ++k)  // the last group's reads run past n: inside
                        nxt[k] = *reinterpret_cast<const float4*>(  // the padded LDS region
                            Lm + (j + GRP < SCH ? j + GRP : 0) + 4 * k);
#if PF_SEQ_SB
                    __builtin_amdgcn_sched_barrier(0);  // keep the reads a whole group ahead
#endif
#pragma unroll
                    for (int k = 0; k < GQ; ++k) {
                        const float4 v = cur[k];
                        if constexpr (SQ) {
                            acc = __builtin_fmaf(v.x, v.x, acc);
                            acc = __builtin_fmaf(v.y, v.y, acc);
                            acc = __builtin_fmaf(v.z, v.z, acc);
                            acc = __builtin_fmaf(v.w, v.w, acc);
                        } else {
                            acc = acc + v.x;
                            acc = acc + v.y;
                            acc = acc + v.z;
                            acc = acc + v.w;
                        }
                    }
                    if constexpr (SQ) mine = lane == j / GRP ? acc : mine;
#pragma unroll
                    for (int k = 0; k < GQ; ++k) cur[k] = nxt[k];
                }
            }
            for (; j < n; ++j) acc = acc + Lm[j];  // plain chains only (SQ chunks here are full)
            if constexpr (SQ) {
                // lane g: the reference's GRP steps of group g from the end of group g - 1
                constexpr int NG = SCH / GRP;
                const float up = __shfl_up(mine, 1);
                float e = lane ? up : st;
                const float4* G = reinterpret_cast<const float4*>(Lm + GRP * (lane < NG ? lane : 0));
#pragma unroll
                for (int k = 0; k < GQ; ++k) {
                    const float4 v = G[k];
                    e = sq_step(e, v.x);
                    e = sq_step(e, v.y);
                    e = sq_step(e, v.z);
                    e = sq_step(e, v.w);
                }
                const int fg = force ? (int)((c * 613) % NG) : -1;
                const uint64_t m = __ballot(lane < NG && (__float_as_uint(e) != __float_as_uint(mine) ||
                                                          lane == fg));
                if (m) {  // rare: redo from the first bad group the reference's way
                    const int g0 = __ffsll((unsigned long long)m) - 1;
                    float a = g0 ? __shfl(mine, g0 - 1) : st;
                    for (int i = GRP * g0; i < n; ++i) a = sq_step(a, Lm[i]);
                    acc = a;
                }
            }
        }
        if (cnt) {
            const float* Lc = L + src.boff(NPL - 1, pid) * SPS;
            for (int i = lane; i < n; i += 64) pos += Lc[i] > 0.0f ? 1u : 0u;
        }
        if (c + 1 < nch) put(lds + ((c + 1) & 1) * (Src::NBUF * SPS));
        src.sync();
    }
    if (cnt) {
        for (int o = 32; o > 0; o >>= 1) pos += __shfl_xor(pos, o);
        *cnt = pos;
    }
    return acc;
}

// Depth.cpp:2119-2134 in the reference's float order, one wave per panorama: lanes 0..3 add
// a00 (v1*v1), a01 (v1), b0 (v0*v1), b1 (v0); a11 counts the compared pixels in a float, which
// is the count itself up to 2^24 and stays at 2^24 after (2^24 + 1 rounds to even).
// FUSED (round 6, MArgs::fast geometry): the block's SEQ_NP producer waves form the terms from
// gt and the result chunk by chunk into a shared LDS double buffer (seq_producers) while the
// chain waves add the previous chunk -- no term planes in HBM (k_seq_terms wrote 2.25 GB of them
// per C3 batch and the chains re-read 1.53 GB).  Else the chains read k_seq_terms' planes.
#ifndef PF_SEQ_NP
// producer waves per block; round 6 A/B on the C3 batch (whole sequential call): 1 -> 8.06,
// 2 -> 7.32-7.38, 4 -> 7.34-7.40 ms
#define PF_SEQ_NP 4
#endif
constexpr int SEQ_NP = PF_SEQ_NP;

template <bool FUSED>
__global__ __launch_bounds__(64 * (1 + SEQ_NP)) void k_ls_seq(MArgs a, SeqTerms T, long long band,
                                                               Align* al)
{
    __shared__ float lds[2 * 4 * SPS];
    const int b = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int pid[4] = {0, 1, 2, 3};
    uint32_t n = 0;
    float r;
    if constexpr (FUSED) {
        if (wv > 0) {
            seq_producers<true>(a, b, 0, Align{1.0f, 0.0f, 0.0f, 0.0f, 0.0f}, band, lds, wv - 1,
                                SEQ_NP, lane);
            return;
        }
        SharedSrc<4> src;
        r = seq_chain<4, false>(src, band, pid, lds, &n);
    } else {
        PlaneSrc<4> src{T.t + (long long)b * 4 * T.bandp, T.bandp};
        r = seq_chain<4, false>(src, band, pid, lds, &n);
    }
    const float a00 = __shfl(r, 0), a01 = __shfl(r, 1), b0 = __shfl(r, 2), b1 = __shfl(r, 3);
    const float a11 = (float)(n < (1u << 24) ? n : (1u << 24));
    if (lane != 0) return;
    const float det = a00 * a11 - a01 * a01;
    Align A{1.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    A.s = (a11 * b0 - a01 * b1) / det;
    A.o = (-a01 * b0 + a00 * b1) / det;
    al[b] = A;
}

// one chain wave of k_err_seq over the planes PIDS
template <bool FUSED, bool SQ, int... PIDS>
__device__ __forceinline__ float err_chain(const SeqTerms& T, long long band, int b, float* lds,
                                           int force)
{
    constexpr int NPL = sizeof...(PIDS);
    const int pid[NPL] = {PIDS...};
    if constexpr (FUSED) {
        SharedSrc<NPL> src;
        return seq_chain<NPL, SQ>(src, band, pid, lds, nullptr, force);
    } else {
        PlaneSrc<NPL> src{T.t + (long long)b * 4 * T.bandp, T.bandp};
        return seq_chain<NPL, SQ>(src, band, pid, lds, nullptr, force);
    }
}

// Depth.cpp:2178-2186, 2207-2210 in the reference's order, three chain waves per panorama: mse
// (plane 0) and mselog (plane 3) through the double square, one wave each; mae (plane 1) and mre
// (plane 2) in float, lanes 0 and 1 of the third; the integer counts come from the parallel
// pass's part[] (exact in any order).  FUSED: waves 3.. produce the terms (one shared buffer for
// the three chains), else each chain wave stages its planes from k_seq_terms' output.
template <bool FUSED>
__global__ __launch_bounds__(64 * (3 + SEQ_NP)) void k_err_seq(MArgs a, int align_way, SeqTerms T,
                                                                long long band, const double* part,
                                                                int nblk, const Align* al,
                                                                pf_metrics* out, int force)
{
    constexpr int BUF = FUSED ? 2 * 4 * SPS : 2 * SPS;
    __shared__ float lds_sq[FUSED ? 1 : 2][BUF];
    __shared__ float lds_pl[FUSED ? 1 : 2 * 2 * SPS];
    __shared__ float res[4];
    const int b = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float* l0 = lds_sq[0];
    float* l1 = FUSED ? lds_sq[0] : lds_sq[FUSED ? 0 : 1];  // (the index is valid in both forms)
    float* l2 = FUSED ? lds_sq[0] : lds_pl;
    // the branches are wave-uniform, and in the FUSED form every wave -- chain or producer --
    // passes the same 1 + nch workgroup barriers (seq_chain's SharedSrc::sync, seq_producers)
    if (wv == 0) {
        const float r = err_chain<FUSED, true, 0>(T, band, b, l0, force);
        if (lane == 0) res[0] = r;
    } else if (wv == 1) {
        const float r = err_chain<FUSED, true, 3>(T, band, b, l1, force);
        if (lane == 0) res[3] = r;
    } else if (wv == 2) {
        const float r = err_chain<FUSED, false, 1, 2>(T, band, b, l2, 0);
        if (lane < 2) res[lane + 1] = r;
    } else if constexpr (FUSED) {
        seq_producers<false>(a, b, align_way, al[b], band, lds_sq[0], wv - 3, SEQ_NP, lane);
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    const float mse = res[0], mae = res[1], mre = res[2], mselog = res[3];
    double cnt[5] = {0, 0, 0, 0, 0};  // n, nlog, fail1..3: integer-valued, order-free
    for (int i = 0; i < nblk; ++i)
        for (int k = 0; k < 5; ++k) cnt[k] += part[((long long)b * nblk + i) * (NSUM + 1) + 4 + k];
    const int n = (int)cnt[0], nlog = (int)cnt[1];
    const int f1 = (int)cnt[2], f2 = (int)cnt[3], f3 = (int)cnt[4];
    pf_metrics mt;
    mt.mse = mse / (float)n;
    mt.mae = mae / (float)n;
    mt.mre = mre / (float)n;
    mt.mselog = mselog / (float)nlog;
    mt.delta1 = (float)(n - f1) / (float)n;
    mt.delta2 = (float)(n - f2) / (float)n;
    mt.delta3 = (float)(n - f3) / (float)n;
    const Align A = al[b];
    mt.median_shift = A.shift;
    mt.ls_s = A.s;
    mt.ls_o = A.o;
    mt.gt_median = A.gt_med;
    mt.given_median = A.gv_med;
    mt.n = n;
    mt.nlog = nlog;
    mt.reserved[0] = mt.reserved[1] = 0;
    out[b] = mt;
}

}  // namespace

static size_t seq_bytes(long long band, int batch)
{  // SeqTerms: four planes of band (rounded up to 4) floats per panorama
    return (size_t)((band + 3) & ~3LL) * 4 * batch * sizeof(float) + 256;
}

// MArgs::fast: gt and the result share the geometry, one channel, 16-B aligned 4-pixel groups
static bool metrics_fast(const MetricsJob& j)
{
    const int gvc = j.given16 ? 1 : j.gc_given;
    return j.gw == j.w && j.gh == j.h && j.gc == 1 && gvc == 1 && j.w % 4 == 0 &&
           ((uintptr_t)j.gt & 15) == 0 &&
           (j.given16 ? ((uintptr_t)j.given16 & 7) == 0 : ((uintptr_t)j.given & 15) == 0);
}

// the sequential order's terms: formed in the chain kernels (fast geometry), else term planes
// in the workspace (k_seq_terms; PF_METRICS_SEQ_PLANES=1 forces them: tests / A/B)
static bool metrics_seq_planes(const MetricsJob& j)
{
    const char* sp = getenv("PF_METRICS_SEQ_PLANES");
    return j.sequential && (!metrics_fast(j) || (sp && sp[0] == '1'));
}

size_t metrics_workspace_bytes(const MetricsJob& j)
{
    const int batch = j.batch;
    const long long band = (long long)(j.h1 - j.h0 + 1) * j.w;
    const bool sequential = metrics_seq_planes(j);
    const size_t hist = sizeof(uint32_t) * 2 * HBINS * batch;
    const size_t st = sizeof(SelState) * 2 * batch;
    const size_t part = sizeof(double) * (NSUM + 1) * MNBLK * batch;
    const size_t al = sizeof(Align) * batch;
    return ((hist + 255) & ~(size_t)255) + ((st + 255) & ~(size_t)255) +
           ((part + 255) & ~(size_t)255) + ((al + 255) & ~(size_t)255) + 256 +
           (sequential ? seq_bytes(band, batch) : 0);
}

void launch_metrics(hipStream_t s, const MetricsJob& j, void* ws, pf_metrics* out)
{
    MArgs a;
    a.gt = j.gt;
    a.gw = j.gw;
    a.gh = j.gh;
    a.gc = j.gc;
    a.gstride = (long long)j.gw * j.gh * j.gc;
    a.gv = j.given;
    a.gv16 = j.given16;
    a.w = j.w;
    a.h = j.h;
    a.gvc = j.given16 ? 1 : j.gc_given;
    a.vstride = (long long)j.w * j.h * a.gvc;
    a.h0 = j.h0;
    a.h1 = j.h1;
    a.rx = (float)j.gw / (float)j.w;
    a.ry = (float)j.gh / (float)j.h;
    a.cap = j.cap_depth;
    const float to_matterport = 65535.0f / 4000.0f;  // Depth.cpp:1999-2000
    a.depth_max = 10.0f / to_matterport;
    a.abs_median = j.given16 ? 0 : 1;
    a.fast = metrics_fast(j) ? 1 : 0;

    char* p = (char*)ws;
    auto carve = [&](size_t bytes) {
        char* r = p;
        p += (bytes + 255) & ~(size_t)255;
        return (void*)r;
    };
    uint32_t* hist = (uint32_t*)carve(sizeof(uint32_t) * 2 * HBINS * j.batch);
    SelState* st = (SelState*)carve(sizeof(SelState) * 2 * j.batch);
    double* part = (double*)carve(sizeof(double) * (NSUM + 1) * MNBLK * j.batch);
    Align* al = (Align*)carve(sizeof(Align) * j.batch);
    const long long band = (long long)(j.h1 - j.h0 + 1) * j.w;
    // tests only: PF_METRICS_SEQ_FORCE_FIX=1 sends one step per chunk down the exact redo path
    const char* ff = getenv("PF_METRICS_SEQ_FORCE_FIX");
    const int seq_force = ff && ff[0] == '1' ? 1 : 0;
    const bool fused = !metrics_seq_planes(j);  // (sequential order only)
    SeqTerms T{};
    if (j.sequential && !fused) {
        T.bandp = (band + 3) & ~3LL;
        T.t = (float*)carve(sizeof(float) * 4 * T.bandp * j.batch);
    }

    // Panoramas in chunks (all at once by default).  Chunks sized to the 256 MB Infinity Cache
    // were measured slower at C3 (1.47 vs 1.42 ms for 64 panoramas): the passes are not
    // HBM-bound, and smaller grids fill the chip worse.
    const int chunk = j.batch;
    for (int b0 = 0; b0 < j.batch; b0 += chunk) {
        const int nb = j.batch - b0 < chunk ? j.batch - b0 : chunk;
        MArgs c = a;
        c.gt = a.gt + (long long)b0 * a.gstride;
        if (c.gv) c.gv = a.gv + (long long)b0 * a.vstride;
        if (c.gv16) c.gv16 = a.gv16 + (long long)b0 * a.vstride;
        uint32_t* hc = hist + (long long)b0 * 2 * HBINS;
        SelState* sc = st + 2 * b0;
        double* pc = part + (long long)b0 * (NSUM + 1) * MNBLK;
        Align* ac = al + b0;
        SeqTerms Tc = T;
        if (Tc.t) Tc.t += (long long)b0 * 4 * T.bandp;
        const dim3 grid(MNBLK, nb);
        if (j.align_way == 1) {
            (void)hipMemsetAsync(hc, 0, sizeof(uint32_t) * 2 * HBINS * nb, s);
            for (int pass = 0; pass < 3; ++pass) {  // k_med_scan re-zeroes the bins it read
                hipLaunchKernelGGL(k_med_hist, grid, dim3(MB), 0, s, c, pass, sc, hc);
                hipLaunchKernelGGL(k_med_scan, dim3(2 * nb), dim3(MB), 0, s, pass, hc, sc);
            }
        } else if (j.align_way == 2 && !j.sequential) {
            hipLaunchKernelGGL(k_ls_sums, grid, dim3(MB), 0, s, c, pc);
        }
        if (j.align_way == 2 && j.sequential) {  // least squares in the reference's float order
            if (fused) {
                hipLaunchKernelGGL(k_ls_seq<true>, dim3(nb), dim3(64 * (1 + SEQ_NP)), 0, s, c, Tc,
                                   band, ac);
            } else {
                hipLaunchKernelGGL(k_seq_terms<true>, grid, dim3(MB), 0, s, c, 0,
                                   (const Align*)nullptr, Tc, band);
                hipLaunchKernelGGL(k_ls_seq<false>, dim3(nb), dim3(64), 0, s, c, Tc, band, ac);
            }
        } else {
            hipLaunchKernelGGL(k_align, dim3(nb), dim3(64), 0, s, j.align_way, sc, pc, MNBLK, ac);
        }
        hipLaunchKernelGGL(k_err_sums, grid, dim3(MB), 0, s, c, j.align_way, ac, pc);
        if (j.sequential && fused) {
            hipLaunchKernelGGL(k_err_seq<true>, dim3(nb), dim3(64 * (3 + SEQ_NP)), 0, s, c,
                               j.align_way, Tc, band, pc, MNBLK, ac, out + b0, seq_force);
        } else if (j.sequential) {
            hipLaunchKernelGGL(k_seq_terms<false>, grid, dim3(MB), 0, s, c, j.align_way, ac, Tc,
                               band);
            hipLaunchKernelGGL(k_err_seq<false>, dim3(nb), dim3(192), 0, s, c, j.align_way, Tc,
                               band, pc, MNBLK, ac, out + b0, seq_force);
        } else {
            hipLaunchKernelGGL(k_err_final, dim3(nb), dim3(MB), 0, s, pc, MNBLK, ac, out + b0);
        }
    }
}

}  // namespace pf
