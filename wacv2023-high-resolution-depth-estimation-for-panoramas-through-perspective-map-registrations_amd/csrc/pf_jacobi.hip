// pf_jacobi.hip -- register-streaming, temporally blocked damped-Jacobi engine for gfx950.
//
// The reference runs `iters` sweeps per level, each a full read-modify-write of the buffer
// (Depth.cpp:1680-1717).  Here one launch ("pass") advances the band by T sweeps:
//
//  * A wave owns a vertical strip of 64*C virtual columns (C per lane) and streams down a chunk
//    of rows.  At step k it loads row k and, for every sweep level t = 1..T, produces row k-2t of
//    level t from rows k-2t-1..k-2t+1 of level t-1, which it keeps in registers (a 3-row ring per
//    level).  Horizontal neighbours cross lanes with DPP wave_shr/wave_shl moves.  L rows come
//    through a per-wave LDS ring; no barriers.
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

#ifndef PF_JNT
// nt stores of the streamed passes' finished rows: 3.03 / 3.10 ms against 3.16 / 3.08 for the
// plain stores in two alternating rounds (profiles/r03/tgt and profiles/r03/jnt; recipe: tools/gpu_round.sh ab, profiles/r03/jnt/): within the noise
#define PF_JNT 0
#endif

#include <cstdlib>
#include <cstring>

#ifndef PF_JACOBI_C4
#define PF_JACOBI_C4 0   // general (scalar) form at 4 columns per lane
#endif
#ifndef PF_JACOBI_C4P
#define PF_JACOBI_C4P 0  // packed form at 4 columns per lane
#endif
#ifndef PF_JACOBI_C3
// packed form at 3 columns per lane (round 6; built, bit-exact, measured slower than C = 2 on
// MI355X: DESIGN.md §3; off in the default build, which it would double; a build with
// -DPF_JACOBI_C3=1 takes it under PF_JC=3)
#define PF_JACOBI_C3 0
#endif
#ifndef PF_JLAG_WAVES
#define PF_JLAG_WAVES 1  // __launch_bounds__ min waves per SIMD of the lagged kernel
#endif
#ifndef PF_JPK_GROUP
#define PF_JPK_GROUP 3  // levels per stage-wise group of the packed form (VGPR bound: 3 waves/SIMD)
#endif
#ifndef PF_JGATE
#define PF_JGATE 0  // skip the sweep levels a step does not need (JLag::sweep_packed)
#endif
#ifndef PF_JFILL
// the first PF_JFILL 6-step groups of a row chunk's lagged fill run as their own unrolled steps
// with the levels they do not need compiled out (JLag::fill_from); 0 = off, -1 = per depth
#define PF_JFILL -1
#endif
#ifndef PF_JDRAIN
// the last PF_JDRAIN 6-step groups of a row chunk with the idle shallow levels compiled out (the
// last group alone holds 39 of the 45 idle level-steps at T = 10); 0 = off
#define PF_JDRAIN 1
#endif
#ifndef PF_JLAG_WAVES_FAST
// the packed passes: 3 waves per SIMD (<= 168 VGPRs).  With the drain compiled out (PF_JDRAIN)
// hipcc's free allocation lands at 168-171 (checked in the ISA); the bound holds it at 168
#define PF_JLAG_WAVES_FAST 3
#endif
#ifndef PF_JDRAIN_BIN
#define PF_JDRAIN_BIN 0
#endif
#ifndef PF_JDRAIN_ROT
#define PF_JDRAIN_ROT 1  // the drain as one copy after rotating the L ring to its group
#endif
#ifndef PF_JPIPE_FILL
#define PF_JPIPE_FILL 3  // fill groups of the pipelined engine (PF_JFILL = -1)
#endif
#ifndef PF_JLAG_PF
// steps of lead for the input and L row loads: 1 or 2 -- the step loop is unrolled by 6, so the
// load-buffer period PF + 1 must divide 6 (PF = 3 would need a 12-step unroll)
#define PF_JLAG_PF 2
#endif
static_assert(6 % (PF_JLAG_PF + 1) == 0, "the 6-step unroll needs a load-buffer period dividing 6");
#ifndef PF_JLREG_T
// passes of depth <= this keep their L ring in registers instead of LDS.  Round 4: at T = 10 the
// register ring takes the packed pass from 132 VGPRs + 48 KB of LDS per 4-wave workgroup to
// 166-167 VGPRs and no LDS -- the same 3 waves per SIMD -- and drops the T LDS reads per step:
// C3 Jacobi stage 3.37-3.38 -> 3.19-3.24 ms, 14.10-14.35k -> 14.75-14.81k panoramas/s (three
// alternating rounds on one MI355X, profiles/r04/ab_lreg; recipe: tools/gpu_round.sh ab)
#define PF_JLREG_T 10
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

typedef float f2 __attribute__((ext_vector_type(2)));

template <int C>
struct Row {
    float v[C];
};
// A lane's column pair as one vector value: element access .v[j] as for any C, and the packed
// form operates on .v directly (an array member here defeats scalar replacement of the level
// rings and sends them to scratch).
template <>
struct Row<2> {
    f2 v;
};
typedef float f4 __attribute__((ext_vector_type(4)));
template <>
struct Row<4> {  // the packed form works on the pairs .lo = columns 0,1 and .hi = columns 2,3
    f4 v;
};
typedef float f3 __attribute__((ext_vector_type(3)));
template <>
struct Row<3> {  // the packed form works on the pair .xy = columns 0,1 and the scalar .z
    f3 v;
};

}  // namespace

// Source of a pass's input rows.
enum { SRC_BUF = 0, SRC_UPSAMPLE = 1, SRC_SEED = 2 };

// ---------------------------------------------------------------------------------------------
// Lagged streaming: sweep level t produces row k-2t at step k (two rows behind level t-1), so
// every level reads only rows finished in earlier steps and the T*C updates of a step are
// independent (no intra-step dependency chain).  Level t keeps a 3-row ring; input rows and L rows
// are loaded PF steps ahead.  The step loop is unrolled by 6 (lcm of the ring period 3 and the
// load-buffer period PF+1) so every register ring index is a compile-time constant.
//
// L rows live in a per-wave LDS ring of R = 2T+1 rows (row r in slot r % R): each L row is loaded
// from memory once and read T times from LDS.
//
// Two arithmetic forms of the same update (bit-identical results):
//  * FAST (C == 2): the two columns of a lane are one v_pk_* operand pair, so the update costs
//    ~9 packed ops + 2 DPP moves + 2 pair assemblies per two pixels.  A packed op moves two lanes
//    of data at about the issue cost of a scalar op on gfx950 (tools/ubench/valu_rate.hip).  The
//    un-windowed mask is geometric: t = fma(d, H, b) with H = 0.5 on windowed pixels and 0 on
//    un-windowed ones (0 * finite = 0, b + 0 = b exactly).  H = Hcol(column) * Hrow(row) needs
//    the host's separable-coverage certificate (prepare_levels in pf_api.hip): a band pixel is
//    covered iff its row is in h0+1..h1-1 and its column in a fixed set that excludes column 0
//    (true of the reference's layouts: column 0 and the columns past the 359.9-degree cap are
//    uncovered).  L rows are sanitised (non-finite -> 0) as they enter the ring so that d stays
//    finite where H = 0.
//  * general: scalar ops, mask from the marker in L (cmp + cndmask per pixel), any coverage.
__device__ __forceinline__ f2 pk_add_clamp01(f2 a, f2 b)
{  // v_pk_add_f32 with the output clamp: both lanes clamped to [0, 1] (b' = clamp01(...))
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 clamp" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// a plain v_add_f32: keeps the backend from widening a lone add of two vector halves into a
// packed op plus a move
__device__ __forceinline__ float add_scalar(float a, float b)
{
    float r;
    asm("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float mul_scalar(float a, float b)
{
    float r;
    asm("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float sub_scalar(float a, float b)
{
    float r;
    asm("v_sub_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float add_clamp01(float a, float b)
{  // v_add_f32 with the output clamp (the scalar column of the C == 3 form)
    float r;
    asm("v_add_f32 %0, %1, %2 clamp" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
#ifndef PF_JFMAC_DPP
// 1: the E tap of a lane's last column is one v_fmac_f32_dpp (the neighbour lane's value read
// through DPP inside the FMA) instead of a v_mov_b32_dpp + v_fmac_f32: hipcc's DPP combiner folds
// a DPP move into a v_add_f32 but not into the tied-accumulator v_fmac_f32
#define PF_JFMAC_DPP 1
#endif
// acc + x[lane + 1] * q (lane 63: + 0 * q, bound_ctrl), one rounding: fma(x[lane+1], q, acc)
__device__ __forceinline__ float fmac_from_right(float acc, float x, float q)
{
#if PF_JFMAC_DPP
    asm("v_fmac_f32_dpp %0, %1, %2 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0"
        : "+v"(acc) : "v"(x), "v"(q));
    return acc;
#else
    return __builtin_fmaf(dpp_from_right(x), q, acc);
#endif
}
// fma(a, b, c) as a plain v_fma_f32 (same reason: two scalar FMAs on the halves of a pair would
// otherwise become a packed FMA after a pair assembly)
__device__ __forceinline__ float fma_scalar(float a, float b, float c)
{
    float r;
    asm("v_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

template <int C, int T, int SRC, bool OUT16, bool FAST>
struct JLag {
    static_assert(C % 2 == 0 || (C == 3 && FAST),
                  "column pairs: vector stores and the wrap logic assume even C (C == 3: the "
                  "packed form with per-column wraps and stores)");
    static_assert(!FAST || C == 2 || C == 3 || C == 4, "the packed form works on column pairs");
    static constexpr int PF = PF_JLAG_PF, NB = PF_JLAG_PF + 1;
    // ring of R >= 2T+1 rows, R a multiple of 6: the loop body is unrolled over the R/6 groups
    // of 6 steps so every ring slot is a compile-time constant (LDS immediate offsets, no SALU)
    static constexpr int R = (2 * T + 1 + 5) / 6 * 6, NG = R / 6;
    // The L ring in registers -- every slot index is a compile-time constant of the unrolled
    // step -- so no LDS store / load latency sits on a step's dependency chain (passes deeper
    // than PF_JLREG_T keep it in LDS: VGPR budget).
    // (C == 3 keeps it in LDS: its register ring would not fit 256 VGPRs beside the level rings;
    // 4 waves x 24 rows x 768 B = 72 KB per workgroup, two workgroups per CU)
    static constexpr bool LREG = C != 3 && T <= PF_JLREG_T;
    Row<C> Lr[LREG ? R : 1];  // LREG: ring slot s = Lr[s]
    Row<C> H[T][3];   // H[t][r % 3] = level t row r
    Row<C> In[NB];    // input row r lands in In[r % NB] (issued at step r + 1 - PF)
    Row<C> Lin[NB];   // L row r lands in Lin[r % NB] (issued at step r - PF), to LDS at step r
    float* lring;     // this wave's ring: R rows of 64*C floats
    int lane_c;       // lane * C (LDS column offset)
    float hcol[C];  // FAST: H of the lane's columns: 0.5 (covered column) or 0
    float vq;       // -1/4 in a VGPR (the folded-DPP FMA takes its second operand from a VGPR)
    const JacobiPass* P;
    int w, xs0, vlo, vhi, r0, r1, h0, h1;
    int kr0, kr1;  // r0 - T and r1 + T: the gating windows of sweep_packed
    int colbase;   // virtual column of lane 0 (wave-uniform)
    int lo;        // lane * C
    int rlo, rhi;  // rows loads are clamped to: the band [h0, h1].  A band pixel never reads a
                   // row outside it except as a neighbour of the un-windowed rows h0 / h1,
                   // whose update ignores its neighbours -- in the packed form through a zero
                   // factor, which needs the neighbours finite.  A halo lane's virtual columns
                   // past a row end still reach rows h0-1 / h1+1, which k_border keeps finite
    const float *src, *prev, *emap, *lnorm;
    float* dst;
    uint16_t* out;
    __amdgpu_buffer_rsrc_t orsrc;  // C == 3: the output plane (dst, or out with OUT16)

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
        } else if constexpr (C == 3) {  // 12-B load (4-B aligned)
            r.v = f3{rp[lo], rp[lo + 1], rp[lo + 2]};
        } else {
            float4 q = *reinterpret_cast<const float4*>(rp + lo);
            r.v[0] = q.x; r.v[1] = q.y; r.v[2] = q.z; r.v[3] = q.w;
        }
        return r;
    }

    __device__ __forceinline__ Row<C> load_input(int k) const
    {
        if constexpr (SRC == SRC_BUF) {
            return load_row(src, k);
        } else if constexpr (C == 3) {
            // a lane's three columns may straddle a row end (xs0 is any multiple of 3 shifted by
            // the halo): each column wraps on its own, as JLag's pairs do below
            Row<C> r;
#pragma unroll
            for (int j = 0; j < 3; j++) {
                int xr = xs0 + j, Y = k;
                if (xr < 0) { xr += w; Y -= 1; }
                else if (xr >= w) { xr -= w; Y += 1; }
                float v = 0.0f;
                if (Y >= 0 && Y < P->h) {
                    if constexpr (SRC == SRC_UPSAMPLE) {
                        v = prev[(long long)(Y >> 1) * (w >> 1) + (xr >> 1)];
                    } else if (Y >= P->h0 && Y <= P->h1) {  // level-0 seed (Depth.cpp:1442-1465)
                        v = emap[P->erow[Y + 1] + P->ecol[xr + 1]];
                    }
                }
                r.v[j] = v;
            }
            return r;
        } else {
            // Virtual column xs0 + j of row k is pixel (xr, Y) with |xs0 + j - xr| < w (the
            // halo is narrower than a row, jacobi_tcap), so the wrap is one compare, no division.
            // xs0 is even and C is even, so the pair (2m, 2m+1) never straddles a row end and
            // shares one source pixel of the half-resolution level.
            Row<C> r;
#pragma unroll
            for (int j = 0; j < C; j += 2) {
                int xr = xs0 + j, Y = k;
                if (xr < 0) { xr += w; Y -= 1; }
                else if (xr >= w) { xr -= w; Y += 1; }
                float v0 = 0.0f, v1 = 0.0f;
                if (Y >= 0 && Y < P->h) {
                    if constexpr (SRC == SRC_UPSAMPLE) {
                        v0 = v1 = prev[(long long)(Y >> 1) * (w >> 1) + (xr >> 1)];
                    } else if (Y >= P->h0 && Y <= P->h1) {  // level-0 seed (Depth.cpp:1442-1465)
                        const int ro = P->erow[Y + 1];
                        v0 = emap[ro + P->ecol[xr + 1]];
                        v1 = emap[ro + P->ecol[xr + 2]];
                    }
                }
                r.v[j] = v0;
                r.v[j + 1] = v1;
            }
            return r;
        }
    }

    static constexpr int slot(int ph, int a) { return ((ph - a) % 3 + 3) % 3; }

    // LDS ring slot of row k + d, with k = group base and GB = k mod R (compile-time)
    template <int GB, int D>
    __device__ __forceinline__ float* lslot() const
    {
        constexpr int s = ((GB + D) % R + R) % R;
        return lring + s * (64 * C) + lane_c;
    }
    template <int GB, int PH>
    __device__ __forceinline__ float* lslot_t(int t) const
    {  // t is a constant after unrolling; the modulo folds
        const int s = ((GB + PH - 2 * t) % R + R) % R;
        return lring + s * (64 * C) + lane_c;
    }
    __device__ __forceinline__ void lds_put(float* p, Row<C> r) const
    {
        if constexpr (FAST) {
#pragma unroll
            for (int j = 0; j < C; j++) r.v[j] = __builtin_isfinite(r.v[j]) ? r.v[j] : 0.0f;
        }
        if constexpr (C == 2) *reinterpret_cast<float2*>(p) = make_float2(r.v[0], r.v[1]);
        else if constexpr (C == 3) { p[0] = r.v[0]; p[1] = r.v[1]; p[2] = r.v[2]; }
        else *reinterpret_cast<float4*>(p) = make_float4(r.v[0], r.v[1], r.v[2], r.v[3]);
    }
    // the L ring: row k of the group (slot GB + PH) enters; level t reads row k - 2t
    template <int GB, int PH>
    __device__ __forceinline__ void ring_put(Row<C> r)
    {
        if constexpr (LREG) {
            if constexpr (FAST) {
#pragma unroll
                for (int j = 0; j < C; j++) r.v[j] = __builtin_isfinite(r.v[j]) ? r.v[j] : 0.0f;
            }
            Lr[((GB + PH) % R + R) % R] = r;
        } else {
            lds_put(lslot<GB, PH>(), r);
        }
    }
    template <int GB, int PH, int TT>
    __device__ __forceinline__ Row<C> ring_get() const
    {
        if constexpr (LREG) return Lr[((GB + PH - 2 * TT) % R + R) % R];
        else return lds_get(lslot_t<GB, PH>(TT));
    }
    __device__ __forceinline__ Row<C> lds_get(const float* p) const
    {
        Row<C> r;
        if constexpr (C == 2) {
            float2 q = *reinterpret_cast<const float2*>(p);
            r.v[0] = q.x; r.v[1] = q.y;
        } else if constexpr (C == 3) {
            r.v = f3{p[0], p[1], p[2]};
        } else {
            float4 q = *reinterpret_cast<const float4*>(p);
            r.v[0] = q.x; r.v[1] = q.y; r.v[2] = q.z; r.v[3] = q.w;
        }
        return r;
    }

    // Lv[t - TA] = L row of level t for t in [TA, TB] (compile-time t)
    template <int GB, int PH, int TA, int TB>
    __device__ __forceinline__ void ring_get_range(Row<C>* Lv) const
    {
        if constexpr (TA <= TB) {
            Lv[0] = ring_get<GB, PH, TA>();
            ring_get_range<GB, PH, TA + 1, TB>(Lv + 1);
        }
    }

    // general form: T*C scalar updates, stage-wise so consecutive VALU instructions belong to
    // different updates (hides the dependent-issue latency)
    template <int PH>
    __device__ __forceinline__ void sweep_general(const Row<C>* Lv, Row<C>* nw) const
    {
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
        // Lcur = (((W*q + N*q) + b) + S*q) + E*q with q = -1/4.  Every product by q (and by 0.5
        // below) is exact -- a power-of-two scaling -- so fl(W*q + N*q) = q*fl(W+N) and
        // fl(a + x*q) = fma(x, q, a): the fused form rounds exactly where the reference rounds.
        // (Exact unless an operand is below 2^-124, which depths in [0,1] never reach here.)
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
        // un-windowed pixel (L = marker): Lcur = L = 0, so the step is exactly +0.  Masked with
        // an AND so the compiler keeps this straight-line (no exec-mask branch).
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
                float tt = __builtin_fmaf(cur[t - 1][j], 0.5f, b);  // b + (L - Lcur)*0.5
                float v = tt * (1 - (float)1e-4) + b * (float)1e-4;
                // clamp01: b is never -0 or NaN here, so med3 equals the reference's compares
                nw[t - 1].v[j] = __builtin_amdgcn_fmed3f(v, 0.0f, 1.0f);
            }
    }

    // FAST form, C == 4: the lane's columns 0..3 are the pairs lo = (0, 1) and hi = (2, 3).  The
    // west pair of hi and the east pair of lo are the same (c1, c2), so per four pixels the
    // update costs 18 packed ops + 2 DPP moves + 3 pair assemblies (C == 2: 9 + 2 + 2 per two).
    template <int PH, int T0, int T1, bool ROWS>
    __device__ __forceinline__ void sweep_packed_group4(const Row<C>* Lv, Row<C>* nw, int k) const
    {
        constexpr int G = T1 - T0;
        const f2 q = {-0.25f, -0.25f};
        const f2 reg = {(float)1e-4, (float)1e-4};
        const f2 reg_ = {1 - (float)1e-4, 1 - (float)1e-4};
        float Wl[G], Er[G];
#pragma unroll
        for (int g = 0; g < G; g++) {
            constexpr int t0 = T0 + 1;
            Wl[g] = dpp_from_left(H[t0 + g - 1][slot(PH, 2 * (t0 + g))].v[3]);
            Er[g] = dpp_from_right(H[t0 + g - 1][slot(PH, 2 * (t0 + g))].v[0]);
        }
        f2 lo[G], hi[G];
        // Lcur = (((W*q + N*q) + b) + S*q) + E*q, q = -1/4, as in sweep_general
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int t = T0 + 1 + g;
            const f4 c = H[t - 1][slot(PH, 2 * t)].v, n = H[t - 1][slot(PH, 2 * t + 1)].v;
            lo[g] = f2{Wl[g], c[0]} + n.lo;
            hi[g] = f2{c[1], c[2]} + n.hi;
        }
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int t = T0 + 1 + g;
            const f4 c = H[t - 1][slot(PH, 2 * t)].v;
            lo[g] = __builtin_elementwise_fma(lo[g], q, c.lo);
            hi[g] = __builtin_elementwise_fma(hi[g], q, c.hi);
        }
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int t = T0 + 1 + g;
            const f4 sv = H[t - 1][slot(PH, 2 * t - 1)].v;
            lo[g] = __builtin_elementwise_fma(sv.lo, q, lo[g]);
            hi[g] = __builtin_elementwise_fma(sv.hi, q, hi[g]);
        }
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int t = T0 + 1 + g;
            const f4 c = H[t - 1][slot(PH, 2 * t)].v;
            lo[g] = __builtin_elementwise_fma(f2{c[1], c[2]}, q, lo[g]);
            hi[g] = __builtin_elementwise_fma(f2{c[3], Er[g]}, q, hi[g]);
        }
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int t = T0 + 1 + g;
            const f4 c = H[t - 1][slot(PH, 2 * t)].v;
            f2 hm0 = f2{hcol[0], hcol[1]}, hm1 = f2{hcol[2], hcol[3]};
            if constexpr (ROWS) {
                const int row = k - 2 * t;
                const float hr = (row == h0 || row == h1) ? 0.0f : 1.0f;
                hm0 = hm0 * hr;
                hm1 = hm1 * hr;
            }
            lo[g] = __builtin_elementwise_fma(Lv[g].v.lo - lo[g], hm0, c.lo);
            hi[g] = __builtin_elementwise_fma(Lv[g].v.hi - hi[g], hm1, c.hi);
        }
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int t = T0 + 1 + g;
            const f4 c = H[t - 1][slot(PH, 2 * t)].v;
            const f2 a = pk_add_clamp01(lo[g] * reg_, c.lo * reg);
            const f2 b = pk_add_clamp01(hi[g] * reg_, c.hi * reg);
            nw[t - 1].v = f4{a[0], a[1], b[0], b[1]};
        }
    }

    // FAST form, C == 3: columns 0, 1 are one packed pair (.xy), column 2 (.z) is scalar.  The
    // cross-lane taps are the W of column 0 (lane - 1's column 2, folded into a v_add_f32_dpp)
    // and the E of column 2 (lane + 1's column 0, a v_mov_b32_dpp); the rest is in-lane.  Per
    // three pixels: 7 packed + 12 scalar + 2 DPP ops, the per-pixel issue cost of C == 2 at 1.5x
    // the columns per strip (so the halo is a smaller share of a strip).
    template <int PH, int T0, int T1, bool ROWS>
    __device__ __forceinline__ void sweep_packed_group3(const Row<C>* Lv, Row<C>* nw, int k) const
    {
        constexpr int G = T1 - T0;
        const f2 q = {-0.25f, -0.25f};
        const f2 reg = {(float)1e-4, (float)1e-4};
        const f2 reg_ = {1 - (float)1e-4, 1 - (float)1e-4};
        f2 cur[G];
        float cz[G];
        // Lcur = (((W*q + N*q) + b) + S*q) + E*q, q = -1/4, as in sweep_general
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int t = T0 + 1 + g;
            const f3 c = H[t - 1][slot(PH, 2 * t)].v, n = H[t - 1][slot(PH, 2 * t + 1)].v;
            cur[g].x = dpp_from_left(c.z) + n.x;  // folds into v_add_f32_dpp
            cur[g].y = add_scalar(c.x, n.y);
            cz[g] = add_scalar(c.y, n.z);
        }
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int t = T0 + 1 + g;
            const f3 c = H[t - 1][slot(PH, 2 * t)].v;
            cur[g] = __builtin_elementwise_fma(cur[g], q, c.xy);
            cz[g] = fma_scalar(cz[g], vq, c.z);
        }
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int t = T0 + 1 + g;
            const f3 sv = H[t - 1][slot(PH, 2 * t - 1)].v;
            cur[g] = __builtin_elementwise_fma(sv.xy, q, cur[g]);
            cz[g] = fma_scalar(sv.z, vq, cz[g]);
        }
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int t = T0 + 1 + g;
            const f3 c = H[t - 1][slot(PH, 2 * t)].v;
            cur[g].x = fma_scalar(c.y, vq, cur[g].x);
            cur[g].y = fma_scalar(c.z, vq, cur[g].y);
            cz[g] = fmac_from_right(cz[g], c.x, vq);
        }
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int t = T0 + 1 + g;
            const f3 c = H[t - 1][slot(PH, 2 * t)].v;
            f2 hh = f2{hcol[0], hcol[1]};
            float hz = hcol[2];
            if constexpr (ROWS) {
                const int row = k - 2 * t;
                const float hr = (row == h0 || row == h1) ? 0.0f : 1.0f;
                hh = hh * hr;
                hz = mul_scalar(hz, hr);
            }
            cur[g] = __builtin_elementwise_fma(Lv[g].v.xy - cur[g], hh, c.xy);
            cz[g] = fma_scalar(sub_scalar(Lv[g].v.z, cz[g]), hz, c.z);
        }
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int t = T0 + 1 + g;
            const f3 c = H[t - 1][slot(PH, 2 * t)].v;
            const f2 a = pk_add_clamp01(cur[g] * reg_, c.xy * reg);
            const float z = add_clamp01(mul_scalar(cz[g], reg_.x), mul_scalar(c.z, reg.x));
            nw[t - 1].v = f3{a.x, a.y, z};
        }
    }

    // FAST form (C == 2): the same update on the lane's column pair, stage-wise over groups of
    // PF_JPK_GROUP levels (bounds the live temporaries, i.e. the VGPR count).  The terms that
    // cross lanes are scalar ops: W + N of column 0 is one v_add_f32_dpp (the DPP move folded
    // into the add) and the E terms are two scalar FMAs, the rest packed.  Measured issue costs
    // on MI355X (tools/ubench/dpp_rate.hip, >= 2 waves/SIMD): v_pk_* 4.7 cycles, v_add/v_fma 2.8,
    // any DPP op 4.4 -- so per level and column pair 7 packed + 1 folded DPP + 1 DPP move +
    // 3 scalar (~50 cycles) against 9 packed + 2 DPP moves + 2 pair assemblies (~57).
    template <int PH, int T0, int T1, bool ROWS>
    __device__ __forceinline__ void sweep_packed_group(const Row<C>* Lv, Row<C>* nw, int k) const
    {
        constexpr int G = T1 - T0;
        const f2 q = {-0.25f, -0.25f};
        const f2 reg = {(float)1e-4, (float)1e-4};
        const f2 reg_ = {1 - (float)1e-4, 1 - (float)1e-4};
        f2 cur[G];
        // Lcur = (((W*q + N*q) + b) + S*q) + E*q, q = -1/4, as in sweep_general
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int t = T0 + 1 + g;
            const f2 c = H[t - 1][slot(PH, 2 * t)].v, n = H[t - 1][slot(PH, 2 * t + 1)].v;
            cur[g].x = dpp_from_left(c.y) + n.x;  // folds into v_add_f32_dpp
            cur[g].y = add_scalar(c.x, n.y);
        }
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int t = T0 + 1 + g;
            cur[g] = __builtin_elementwise_fma(cur[g], q, H[t - 1][slot(PH, 2 * t)].v);
        }
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int t = T0 + 1 + g;
            cur[g] = __builtin_elementwise_fma(H[t - 1][slot(PH, 2 * t - 1)].v, q, cur[g]);
        }
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int t = T0 + 1 + g;
            const f2 c = H[t - 1][slot(PH, 2 * t)].v;
            cur[g].x = fma_scalar(c.y, vq, cur[g].x);
            cur[g].y = fmac_from_right(cur[g].y, c.x, vq);
        }
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int t = T0 + 1 + g;
            // rows h0 and h1 are un-windowed (the host certified the rest of the band); only
            // passes whose row window reaches them (ROWS) pay for the test
            f2 hh = f2{hcol[0], hcol[1]};
            if constexpr (ROWS) {
                const int row = k - 2 * t;
                const float hr = (row == h0 || row == h1) ? 0.0f : 1.0f;
                hh = hh * hr;
            }
            cur[g] = __builtin_elementwise_fma(Lv[g].v - cur[g], hh, H[t - 1][slot(PH, 2 * t)].v);
        }
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int t = T0 + 1 + g;
            nw[t - 1].v = pk_add_clamp01(cur[g] * reg_, H[t - 1][slot(PH, 2 * t)].v * reg);
        }
    }
    // Fill/drain gating.  Level t is only needed for rows [r0 - (T-t), r1 + (T-t)) of the chunk,
    // i.e. at steps k in [r0 - T + 3t, r1 + T + t); outside that window its row is never read by
    // a needed update (stencil closure), so a group of levels whose windows all miss step k is
    // skipped with one wave-uniform branch -- its ring slots then hold stale rows, read only by
    // unneeded updates.  At the default depths this drops 10-30% of the issued updates (the
    // lagged start fills T levels over 3T steps, the drain empties them over T).
    // levels LA..NA are computed this step (the rest are idle: NA < T in the chunk's fill,
    // LA > 1 in its drain, below)
    template <int PH, int GB, int T0, bool ROWS, int NA, int LA = 1>
    __device__ __forceinline__ void sweep_packed(Row<C>* nw, int k) const
    {
        constexpr int T1 = T0 + PF_JPK_GROUP < T ? T0 + PF_JPK_GROUP : T;
        // the groups run from the deepest level down: level t+1 reads the oldest row of level
        // t's ring before level t overwrites it, so the new row can take that row's registers
        // (all reads of a step are rows of earlier steps, so the order is free)
        if constexpr (T1 < T) sweep_packed<PH, GB, T1, ROWS, NA, LA>(nw, k);
        constexpr int TB = T1 < NA ? T1 : NA;
        constexpr int TA = T0 > LA - 1 ? T0 : LA - 1;  // levels TA+1 .. TB
        if constexpr (TA < TB)
#if PF_JGATE
        if (k - kr0 >= 3 * (T0 + 1) && k - kr1 < T1)
#endif
        {
            Row<C> Lv[TB - TA];
            ring_get_range<GB, PH, TA + 1, TB>(Lv);
            if constexpr (C == 4) sweep_packed_group4<PH, TA, TB, ROWS>(Lv, nw, k);
            else if constexpr (C == 3) sweep_packed_group3<PH, TA, TB, ROWS>(Lv, nw, k);
            else sweep_packed_group<PH, TA, TB, ROWS>(Lv, nw, k);
        }
    }

    // Step k = (group base) + PH; GB = (group base - k0) mod R: ring slots count from the
    // chunk's first step, so they are compile-time constants without aligning k0.  NA < T only
    // in the fill (fill_from).
    template <int PH, bool ROWS, int GB, int NA = T, int LA = 1>
    __device__ __forceinline__ void step(int k)
    {
        // level-0 row k-1 (loaded last step) joins the ring
        H[0][slot(PH, 1)] = In[(PH + NB - 1) % NB];
        // L row k (landed in Lin last step) goes to its ring slot; fetch L row k+PF.  The slot
        // is reused by row k+R > k, after every level has read row k (last read at k + 2T).
        ring_put<GB, PH>(Lin[PH % NB]);
#if PF_JDBG_NOGLOBAL  // profiling only (wrong results): no global loads in the loop
        Lin[(PH + PF) % NB] = H[T - 1][slot(PH, 1)];
        In[(PH + PF - 1) % NB] = H[T - 2][slot(PH, 2)];
#else
        Lin[(PH + PF) % NB] = load_row(lnorm, k + PF);
        // input row k + PF - 1 for a later step
        In[(PH + PF - 1) % NB] = load_input(k + PF - 1);
#endif
        Row<C> nw[T];
        if constexpr (FAST) {
            sweep_packed<PH, GB, 0, ROWS, NA, LA>(nw, k);
        } else {
            static_assert(NA == T && LA == 1, "the general form has no fill / drain specialisation");
            Row<C> Lv[T];
            ring_get_range<GB, PH, 1, T>(Lv);
            sweep_general<PH>(Lv, nw);
        }
#pragma unroll
        for (int t = 1; t < T; t++)
            if (t >= LA && t <= NA) H[t][slot(PH, 2 * t)] = nw[t - 1];  // idle: keeps its rows
        if constexpr (NA < T) return;  // no stored row before every level runs (fill_from)
        const int j = k - 2 * T;  // final-level row finished this step
        if constexpr (C == 3) {
            // the strip edges cut lanes (the halo is not a multiple of 3): a store per column,
            // each column inside [vlo, vhi) or dropped by the buffer's range check
            if (j >= r0 && j < r1) {
                const uint32_t rowb = (uint32_t)(j * w + colbase + lo);  // pixel index
#pragma unroll
                for (int p = 0; p < 3; p++) {
                    const bool in = xs0 + p >= vlo && xs0 + p < vhi;
                    if constexpr (OUT16) {
                        const uint32_t qv = (uint32_t)(nw[T - 1].v[p] * 65535.0f);
                        __builtin_amdgcn_raw_buffer_store_b16((uint16_t)qv, orsrc,
                                                              in ? (int)(2 * (rowb + p)) : -16, 0, 0);
                    } else {
                        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(nw[T - 1].v[p]), orsrc,
                                                              in ? (int)(4 * (rowb + p)) : -16, 0, 0);
                    }
                }
            }
            return;
        }
        // xs0, vlo, vhi and C are even, so a lane's columns are all inside [vlo, vhi) or all
        // outside: one vector store per lane.
        if (j >= r0 && j < r1 && xs0 >= vlo && xs0 < vhi) {
            const long long rowb = (long long)j * w + colbase;
            if constexpr (OUT16) {
                // quantise (Depth.cpp:1721-1736); v is already in [0,1], truncating cast
                uint32_t qv[C];
#pragma unroll
                for (int p = 0; p < C; p++) qv[p] = (uint32_t)(nw[T - 1].v[p] * 65535.0f);
                if constexpr (C == 2) {
                    *reinterpret_cast<uint32_t*>(out + rowb + lo) = qv[0] | (qv[1] << 16);
                } else {
                    *reinterpret_cast<uint2*>(out + rowb + lo) =
                        make_uint2(qv[0] | (qv[1] << 16), qv[2] | (qv[3] << 16));
                }
            } else {
                if constexpr (C == 2 && PF_JNT) {
                    typedef float f2v __attribute__((ext_vector_type(2)));
                    __builtin_nontemporal_store(f2v{nw[T - 1].v[0], nw[T - 1].v[1]},
                                                reinterpret_cast<f2v*>(dst + rowb + lo));
                } else if constexpr (C == 2)
                    *reinterpret_cast<float2*>(dst + rowb + lo) = make_float2(nw[T - 1].v[0], nw[T - 1].v[1]);
                else
                    *reinterpret_cast<float4*>(dst + rowb + lo) =
                        make_float4(nw[T - 1].v[0], nw[T - 1].v[1], nw[T - 1].v[2], nw[T - 1].v[3]);
            }
        }
    }

    // one group of 6 steps starting at k, k mod R == 6G
    template <bool ROWS, int G>
    __device__ __forceinline__ void group(int k)
    {
        step<0, ROWS, 6 * G>(k);
        step<1, ROWS, 6 * G>(k + 1);
        step<2, ROWS, 6 * G>(k + 2);
        step<3, ROWS, 6 * G>(k + 3);
        step<4, ROWS, 6 * G>(k + 4);
        step<5, ROWS, 6 * G>(k + 5);
    }
    // groups G..NG-1 of the unrolled ring period; returns false once k reaches kend
    template <bool ROWS, int G>
    __device__ __forceinline__ bool groups_from(int& k, int kend)
    {
        group<ROWS, G>(k);
        k += 6;
        if (k >= kend) return false;
        if constexpr (G + 1 < NG) return groups_from<ROWS, G + 1>(k, kend);
        else return true;
    }
    // The chunk's fill.  The stored rows [r0, r1) of level T read level t's rows
    // [r0 - (T - t), r1 + (T - t)) and nothing else; level t produces row k - 2t at step k, so
    // its first needed row comes at step r0 - T + 3t = k0 + 1 + 3t.  Before that (s = k - k0 <
    // 1 + 3t) level t feeds nothing that is stored.  The first NF groups therefore run as their
    // own unrolled steps with levels na(s) + 1 .. T compiled out; an idle level keeps its
    // zero-initialised rows, which only idle levels read (level t reads level t - 1 alone, which
    // is active from three steps earlier).  At T = 10: 175 of the ~2,100 level-steps of a
    // 183-row chunk.
    static constexpr int na(int s)
    {
        const int a = s >= 1 ? (s - 1) / 3 : 0;
        return a < T ? a : T;
    }
    static constexpr int NF_ALL = (3 * T + 1 + 5) / 6;  // groups with an idle level
    // hipcc's register allocation of the unrolled loop is erratic in the fill length: at T = 10,
    // 3 groups keep the step loop at 166-169 VGPRs (3 waves per SIMD) where 1 or 4 take 171-232;
    // at T = 8, 4 groups keep 140-143 where 3 take 188 (checked in the ISA)
    static constexpr int NF_AUTO = T == 8 ? 4 : 3;
    static constexpr int NF_SEL = PF_JFILL < 0 ? NF_AUTO : PF_JFILL;
    static constexpr int NF = !FAST ? 0 : (NF_SEL < NF_ALL ? NF_SEL : NF_ALL);
    template <bool ROWS, int F>
    __device__ __forceinline__ bool fill_from(int& k, int kend)
    {
        if constexpr (F < NF) {
            constexpr int GB = 6 * (F % NG);
            step<0, ROWS, GB, na(6 * F + 0)>(k);
            step<1, ROWS, GB, na(6 * F + 1)>(k + 1);
            step<2, ROWS, GB, na(6 * F + 2)>(k + 2);
            step<3, ROWS, GB, na(6 * F + 3)>(k + 3);
            step<4, ROWS, GB, na(6 * F + 4)>(k + 4);
            step<5, ROWS, GB, na(6 * F + 5)>(k + 5);
            k += 6;
            if (k >= kend) return false;
            return fill_from<ROWS, F + 1>(k, kend);
        } else {
            return true;
        }
    }
    // The chunk's drain, likewise: level t is last needed at step kend - 1 - (T - t), so in the
    // last T steps the shallow levels go idle one by one.  The last ND groups run as their own
    // steps with levels 1 .. la(p) - 1 compiled out, p = the step within those groups.  The
    // chunk's step count kend - k0 is not a multiple of 6: the groups end o = 0..5 steps past
    // kend, and la() assumes o = 0, the largest active set (a few idle level-steps remain when
    // o > 0; nothing needed is skipped).  The drain starts at a run-time ring group, hence one
    // copy per group of the ring period (drain_switch).
    static constexpr int ND_ALL = (T + 5) / 6;  // groups with an idle level (o = 0)
    static constexpr int ND = !(PF_JDRAIN && FAST) ? 0 : (PF_JDRAIN < ND_ALL ? PF_JDRAIN : ND_ALL);
    static constexpr int la(int p)
    {
        const int a = T - 6 * ND + p + 1;
        return a < 1 ? 1 : a;
    }
    template <bool ROWS, int G0, int I>
    __device__ __forceinline__ void drain_from(int& k)
    {
        if constexpr (I < ND) {
            constexpr int GB = 6 * ((G0 + I) % NG);
            step<0, ROWS, GB, T, la(6 * I + 0)>(k);
            step<1, ROWS, GB, T, la(6 * I + 1)>(k + 1);
            step<2, ROWS, GB, T, la(6 * I + 2)>(k + 2);
            step<3, ROWS, GB, T, la(6 * I + 3)>(k + 3);
            step<4, ROWS, GB, T, la(6 * I + 4)>(k + 4);
            step<5, ROWS, GB, T, la(6 * I + 5)>(k + 5);
            k += 6;
            drain_from<ROWS, G0, I + 1>(k);
        }
    }
    // the drain code is written for ring group 0: the L ring (registers) is rotated so that the
    // drain's first group sits at slot 0 (a register permutation once per chunk), instead of one
    // copy of the drain per ring group (which took the T = 10 pass from 166 to 214 VGPRs)
    template <int SH>
    __device__ __forceinline__ void ring_rotate()
    {
        Row<C> t[R];
#pragma unroll
        for (int x = 0; x < R; x++) t[x] = Lr[(x + SH) % R];
#pragma unroll
        for (int x = 0; x < R; x++) Lr[x] = t[x];
    }
    template <int G>
    __device__ __forceinline__ void ring_to_zero(int g)
    {
#if PF_JDRAIN_BIN
        // by binary parts of g: a rotation by 6 groups' worth of slots per set bit
        if constexpr (G == 1) {
            if (g & 1) ring_rotate<6>();
            if constexpr (NG > 2) { if (g & 2) ring_rotate<12 % R>(); }
        }
#else
        if constexpr (G < NG) {
            if (g == G) ring_rotate<6 * G>();
            else ring_to_zero<G + 1>(g);
        }
#endif
    }
    template <bool ROWS, int G>
    __device__ __forceinline__ void drain_switch(int g, int& k)
    {
        if constexpr (LREG && PF_JDRAIN_ROT) {
            if constexpr (NG > 1) ring_to_zero<1>(g);
            drain_from<ROWS, 0, 0>(k);
        } else if constexpr (G < NG) {
            if (g == G) drain_from<ROWS, G, 0>(k);
            else drain_switch<ROWS, G + 1>(g, k);
        }
    }
    // the step loop from the chunk's first step k0 (ring group 0): the fill, whole groups up to
    // the drain (or to the end, for a chunk too short for both), the drain
    template <bool ROWS>
    __device__ __forceinline__ void run(int k0, int kend)
    {
        int k = k0;
        const int gt = (kend - k0 + 5) / 6;  // groups of the chunk
        const bool dr = ND > 0 && gt >= NF + ND;
        if (!fill_from<ROWS, 0>(k, kend)) return;
        const int kd = dr ? k0 + 6 * (gt - ND) : kend;
        if (k < kd) {
            bool more = true;
            if constexpr (NF % NG != 0) more = groups_from<ROWS, NF % NG>(k, kd);
            while (more) more = groups_from<ROWS, 0>(k, kd);
        }
        if (dr) drain_switch<ROWS, 0>(__builtin_amdgcn_readfirstlane((gt - ND) % NG), k);
    }
};

template <int C, int T, int SRC, bool OUT16, bool FAST>
// C == 3: two waves per SIMD (its LDS ring allows two 4-wave workgroups per CU anyway)
__global__ void __launch_bounds__(256, FAST ? (C == 3 ? 2 : PF_JLAG_WAVES_FAST) : PF_JLAG_WAVES)
k_jlag(JacobiPass P)
{
    using S_t = JLag<C, T, SRC, OUT16, FAST>;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int job = blockIdx.x * 4 + wave;
    if (job >= P.nstrips * P.nchunks) return;  // wave-uniform
    const int b = blockIdx.y;
    const int strip = job % P.nstrips, chunk = job / P.nstrips;
    S_t S;
    S.P = &P;
    S.w = P.w;
    S.h0 = P.h0;
    S.h1 = P.h1;
    S.colbase = strip * P.V - P.Tp;
    S.lo = lane * C;
    S.vq = -0.25f;
    asm volatile("" : "+v"(S.vq));
    S.rlo = P.h0;
    S.rhi = P.h1;
    S.xs0 = strip * P.V - P.Tp + lane * C;
    S.vlo = strip * P.V;
    S.vhi = min(S.vlo + P.V, P.w);
    S.r0 = P.row_lo + chunk * P.rows_per_chunk;
    S.r1 = min(S.r0 + P.rows_per_chunk, P.row_hi);
    S.kr0 = S.r0 - T;
    S.kr1 = S.r1 + T;
    S.src = P.src + b * P.sstride;
    S.prev = P.prev + b * P.pstride;
    S.emap = P.emap + b * P.estride;
    S.lnorm = P.lnorm + b * P.lstride;
    S.dst = P.dst + b * P.dstride;
    S.out = P.out + b * P.ostride;
    // H of the lane's two columns.  Column 0 is un-windowed (certified), so the only halo cell
    // that can reach a stored pixel is virtual column w (pixel (0, Y+1), the east tap of column
    // w-1 -- the seam quirk), whose H is 0; other halo cells get 0 too (never read).
#pragma unroll
    for (int j = 0; j < C; j++) S.hcol[j] = 0.0f;
    if constexpr (FAST && C == 3) {
#pragma unroll
        for (int j = 0; j < 3; j++)
            if (S.xs0 + j >= 0 && S.xs0 + j < P.w) S.hcol[j] = P.hcol[S.xs0 + j];
        // range-checked stores: offsets past the plane are dropped (a -16 offset wraps past it)
        const uint32_t pbytes = (uint32_t)((long long)P.w * P.h * (OUT16 ? 2 : 4));
        S.orsrc = __builtin_amdgcn_make_buffer_rsrc(OUT16 ? (void*)S.out : (void*)S.dst, 0,
                                                    (int)pbytes, 0x00020000);
    } else if constexpr (FAST) {
        // xs0 and w are multiples of C, so the lane's C columns are all inside or all outside
        if (S.xs0 >= 0 && S.xs0 < P.w)
#pragma unroll
            for (int j = 0; j < C; j++) S.hcol[j] = P.hcol[S.xs0 + j];
    }
#pragma unroll
    for (int t = 0; t < T; t++)
#pragma unroll
        for (int q = 0; q < 3; q++)
#pragma unroll
            for (int j = 0; j < C; j++) S.H[t][q].v[j] = 0.0f;
#pragma unroll
    for (int q = 0; q < S_t::NB; q++)
#pragma unroll
        for (int j = 0; j < C; j++) { S.In[q].v[j] = 0.0f; S.Lin[q].v[j] = 0.0f; }
    constexpr int R = S_t::R;
    if constexpr (S_t::LREG) {
#pragma unroll
        for (int q = 0; q < R; q++)
#pragma unroll
            for (int j = 0; j < C; j++) S.Lr[q].v[j] = 0.0f;
        S.lring = nullptr;
    } else {
        __shared__ float lds_l[4 * R * 64 * C];  // per-wave private rings, no barriers needed
        S.lring = lds_l + wave * (R * 64 * C);
    }
    S.lane_c = lane * C;
    // steps k0 .. kend: level 0 needs rows from r0 - T, the last output row r1-1 finishes at
    // step r1 - 1 + 2T.  Ring slots count from k0 (JLag::step), so k0 needs no alignment.
    const int k0 = S.r0 - T - 1;
    const int kend = S.r1 + 2 * T;
    // prime the rows the first steps consume before their in-loop loads land (the rest are
    // loaded PF steps ahead inside step()).  The ring slots of rows before k0 stay unwritten:
    // they only feed halo/stale cells, like the zero-initialised level rows.  Row k0 + r sits
    // in buffer r (buffers count from k0, like the ring slots).
#pragma unroll
    for (int r = 0; r + 1 < S_t::PF; r++) S.In[r] = S.load_input(k0 + r);
#pragma unroll
    for (int r = 0; r < S_t::PF; r++) S.Lin[r] = S.load_row(S.lnorm, k0 + r);
    // rows computed by some level of this pass: k - 2t for k in [k0, kend + 5], t in [1, T]
    const int wlo = k0 - 2 * T, whi = kend + 3;
    const bool rows = (S.h0 >= wlo && S.h0 <= whi) || (S.h1 >= wlo && S.h1 <= whi);
    if (!FAST || rows) S.template run<true>(k0, kend);
    else S.template run<false>(k0, kend);
}

// ---------------------------------------------------------------------------------------------
// Pipelined passes: the T = S*TS sweep levels of one strip-chunk are split over the S waves of a
// workgroup.  Wave (stage) s owns levels s*TS+1 .. (s+1)*TS and runs the lagged stream of JLag
// over them; the input of its first level is its predecessor's last level, whose new row the
// predecessor leaves in a double-buffered LDS slot every step (one workgroup barrier per step).
// Against JLag at the same T: S times the waves per strip-chunk at 1/S of the register rings, so
// the small levels fill the chip with fewer row chunks (less vertical halo) and every level gets
// more waves per SIMD to hide the load/LDS latency behind.  Same arithmetic, same order: every
// pixel's value is bit-identical to JLag's (and the reference's).
static constexpr int md(int a, int m) { return ((a % m) + m) % m; }

template <int TS, int S, int SI, int SRC, bool OUT16>
struct JPipe {
    static constexpr int C = 2;
    static constexpr int T = TS * S;
    static constexpr int TB = SI * TS + 1, TE = TB + TS - 1;  // own levels
    static constexpr int PF = PF_JLAG_PF, NB = PF_JLAG_PF + 1;
    static constexpr int R = (2 * TS + 1 + 5) / 6 * 6;  // L ring rows (multiple of 6)
    static constexpr int NG = R / 6;
    static constexpr int G = PF_JPK_GROUP;
    Row<C> H[TS][3];  // H[l][row % 3]: level TB-1+l (l = 0: the input level of this stage)
    Row<C> In[NB];    // stage 0: level-0 input row r in In[r % NB]
    Row<C> Lin[NB];   // L row r in Lin[r % NB], put into the LDS ring PF steps after its load
    float* lring;     // this stage's ring: R rows of 64*C floats (row r in slot r % R)
    const float* xin; // stage > 0: the predecessor's exchange slots [2][64*C]
    float* xout;      // stage < S-1: this stage's exchange slots
    int lane_c;
    float hcol[C];
    float vq;  // -1/4 in a VGPR, as JLag::vq
    const JacobiPass* P;
    int w, xs0, vlo, vhi, r0, r1, h0, h1, colbase, lo, rlo, rhi;
    const float *src, *prev, *emap, *lnorm;
    float* dst;
    uint16_t* out;

    __device__ __forceinline__ Row<C> load_row(const float* base_ptr, int k) const
    {
        Row<C> r;
        int kc = k < rlo ? rlo : (k > rhi ? rhi : k);
        const float2 q = *reinterpret_cast<const float2*>(base_ptr + ((long long)kc * w + colbase) + lo);
        r.v[0] = q.x; r.v[1] = q.y;
        return r;
    }
    __device__ __forceinline__ Row<C> load_input(int k) const
    {  // as JLag::load_input
        if constexpr (SRC == SRC_BUF) {
            return load_row(src, k);
        } else {
            Row<C> r;
            int xr = xs0, Y = k;
            if (xr < 0) { xr += w; Y -= 1; }
            else if (xr >= w) { xr -= w; Y += 1; }
            float v0 = 0.0f, v1 = 0.0f;
            if (Y >= 0 && Y < P->h) {
                if constexpr (SRC == SRC_UPSAMPLE) {
                    v0 = v1 = prev[(long long)(Y >> 1) * (w >> 1) + (xr >> 1)];
                } else if (Y >= P->h0 && Y <= P->h1) {
                    const int ro = P->erow[Y + 1];
                    v0 = emap[ro + P->ecol[xr + 1]];
                    v1 = emap[ro + P->ecol[xr + 2]];
                }
            }
            r.v[0] = v0;
            r.v[1] = v1;
            return r;
        }
    }
    __device__ __forceinline__ void lds_put(float* p, Row<C> r) const
    {  // L rows sanitised as they enter the ring (the packed form's H = 0 trick, JLag)
        r.v[0] = __builtin_isfinite(r.v[0]) ? r.v[0] : 0.0f;
        r.v[1] = __builtin_isfinite(r.v[1]) ? r.v[1] : 0.0f;
        *reinterpret_cast<float2*>(p) = make_float2(r.v[0], r.v[1]);
    }
    __device__ __forceinline__ Row<C> lds_get(const float* p) const
    {
        Row<C> r;
        const float2 q = *reinterpret_cast<const float2*>(p);
        r.v[0] = q.x; r.v[1] = q.y;
        return r;
    }

    // own levels T0 < t <= T1 (global indices) of step k (phase PH), packed form of JLag
    template <int PH, int T0, int T1, bool ROWS>
    __device__ __forceinline__ void sweep_group(const Row<C>* Lv, Row<C>* nw, int k) const
    {
        constexpr int NGR = T1 - T0;
        const f2 q = {-0.25f, -0.25f};
        const f2 reg = {(float)1e-4, (float)1e-4};
        const f2 reg_ = {1 - (float)1e-4, 1 - (float)1e-4};
        f2 cur[NGR];
#pragma unroll
        for (int g = 0; g < NGR; g++) {
            const int t = T0 + 1 + g, l = t - TB;  // reads ring H[l] = level t-1
            const f2 c = H[l][md(PH - 2 * t, 3)].v, n = H[l][md(PH - 2 * t - 1, 3)].v;
            cur[g].x = dpp_from_left(c.y) + n.x;
            cur[g].y = add_scalar(c.x, n.y);
        }
#pragma unroll
        for (int g = 0; g < NGR; g++) {
            const int t = T0 + 1 + g, l = t - TB;
            cur[g] = __builtin_elementwise_fma(cur[g], q, H[l][md(PH - 2 * t, 3)].v);
        }
#pragma unroll
        for (int g = 0; g < NGR; g++) {
            const int t = T0 + 1 + g, l = t - TB;
            cur[g] = __builtin_elementwise_fma(H[l][md(PH - 2 * t + 1, 3)].v, q, cur[g]);
        }
#pragma unroll
        for (int g = 0; g < NGR; g++) {
            const int t = T0 + 1 + g, l = t - TB;
            const f2 c = H[l][md(PH - 2 * t, 3)].v;
            cur[g].x = fma_scalar(c.y, vq, cur[g].x);
            cur[g].y = fmac_from_right(cur[g].y, c.x, vq);
        }
#pragma unroll
        for (int g = 0; g < NGR; g++) {
            const int t = T0 + 1 + g, l = t - TB;
            f2 hh = f2{hcol[0], hcol[1]};
            if constexpr (ROWS) {
                const int row = k - 2 * t;
                const float hr = (row == h0 || row == h1) ? 0.0f : 1.0f;
                hh = hh * hr;
            }
            cur[g] = __builtin_elementwise_fma(Lv[t - TB].v - cur[g], hh, H[l][md(PH - 2 * t, 3)].v);
        }
#pragma unroll
        for (int g = 0; g < NGR; g++) {
            const int t = T0 + 1 + g, l = t - TB;
            nw[t - TB].v = pk_add_clamp01(cur[g] * reg_, H[l][md(PH - 2 * t, 3)].v * reg);
        }
    }
    // own levels T0 < t <= min(T1, NA): levels past NA are idle in the fill (JLag::fill_from)
    template <int PH, int T0, bool ROWS, int NA>
    __device__ __forceinline__ void sweep(const Row<C>* Lv, Row<C>* nw, int k) const
    {
        constexpr int T1 = T0 + G < TE ? T0 + G : TE;
        constexpr int TB_ = T1 < NA ? T1 : NA;
        if constexpr (T0 < TB_) sweep_group<PH, T0, TB_, ROWS>(Lv, nw, k);
        if constexpr (T1 < TE) sweep<PH, T1, ROWS, NA>(Lv, nw, k);
    }

    // step k = (group base) + PH, GB = (group base - k0) mod R (ring slots count from the
    // chunk's first step, as in JLag); levels past NA idle (the fill)
    template <int PH, bool ROWS, int GB, int NA = T>
    __device__ __forceinline__ void step(int k)
    {
        // the input level's row k - 2TB + 1 joins ring H[0]
        if constexpr (SI == 0) {
            H[0][md(PH - 1, 3)] = In[md(PH - 1, NB)];
        } else {
            H[0][md(PH - 2 * TB + 1, 3)] = lds_get(xin + md(PH - 1, 2) * (64 * C) + lane_c);
        }
        // L row q = k - 2TB + 2 enters the ring; rows k - 2t (t = TB..TE) are read from it
        constexpr int QO = -2 * TB + 2;
        lds_put(lring + md(GB + PH + QO, R) * (64 * C) + lane_c, Lin[md(PH + QO, NB)]);
        Row<C> Lv[TS];
#pragma unroll
        for (int t = TB; t <= TE; t++) Lv[t - TB] = lds_get(lring + md(GB + PH - 2 * t, R) * (64 * C) + lane_c);
        Lin[md(PH + QO + PF, NB)] = load_row(lnorm, k + QO + PF);
        if constexpr (SI == 0) In[md(PH + PF - 1, NB)] = load_input(k + PF - 1);
        Row<C> nw[TS];
        sweep<PH, TB - 1, ROWS, NA>(Lv, nw, k);
#pragma unroll
        for (int t = TB; t < TE; t++)
            if (t <= NA) H[t - TB + 1][md(PH - 2 * t, 3)] = nw[t - TB];
        if constexpr (SI < S - 1) {
            if constexpr (TE <= NA)  // else the next stage's first level is idle too
                *reinterpret_cast<float2*>(xout + md(PH, 2) * (64 * C) + lane_c) =
                    make_float2(nw[TS - 1].v[0], nw[TS - 1].v[1]);
        } else if constexpr (NA == T) {
            const int j = k - 2 * T;  // final-level row finished this step
            if (j >= r0 && j < r1 && xs0 >= vlo && xs0 < vhi) {
                const long long rowb = (long long)j * w + colbase;
                if constexpr (OUT16) {
                    const uint32_t q0 = (uint32_t)(nw[TS - 1].v[0] * 65535.0f);
                    const uint32_t q1 = (uint32_t)(nw[TS - 1].v[1] * 65535.0f);
                    *reinterpret_cast<uint32_t*>(out + rowb + lo) = q0 | (q1 << 16);
                } else {
                    *reinterpret_cast<float2*>(dst + rowb + lo) =
                        make_float2(nw[TS - 1].v[0], nw[TS - 1].v[1]);
                }
            }
        }
        __syncthreads();  // the exchange row of this step is visible to the next stage
    }

    template <bool ROWS, int GI>
    __device__ __forceinline__ void group(int k)
    {
        step<0, ROWS, 6 * GI>(k);
        step<1, ROWS, 6 * GI>(k + 1);
        step<2, ROWS, 6 * GI>(k + 2);
        step<3, ROWS, 6 * GI>(k + 3);
        step<4, ROWS, 6 * GI>(k + 4);
        step<5, ROWS, 6 * GI>(k + 5);
    }
    template <bool ROWS, int GI>
    __device__ __forceinline__ bool groups_from(int& k, int kend)
    {
        group<ROWS, GI>(k);
        k += 6;
        if (k >= kend) return false;
        if constexpr (GI + 1 < NG) return groups_from<ROWS, GI + 1>(k, kend);
        else return true;
    }
    // the fill as JLag::fill_from: level t idle for steps s = k - k0 < 1 + 3t (every stage runs
    // the same steps, so the barriers still pair up)
    static constexpr int na(int s)
    {
        const int a = s >= 1 ? (s - 1) / 3 : 0;
        return a < T ? a : T;
    }
    static constexpr int NF_ALL = (3 * T + 1 + 5) / 6;
    static constexpr int NF_SEL = PF_JFILL < 0 ? PF_JPIPE_FILL : PF_JFILL;
    static constexpr int NF = NF_SEL < NF_ALL ? NF_SEL : NF_ALL;
    template <bool ROWS, int F>
    __device__ __forceinline__ bool fill_from(int& k, int kend)
    {
        if constexpr (F < NF) {
            constexpr int GB = 6 * (F % NG);
            step<0, ROWS, GB, na(6 * F + 0)>(k);
            step<1, ROWS, GB, na(6 * F + 1)>(k + 1);
            step<2, ROWS, GB, na(6 * F + 2)>(k + 2);
            step<3, ROWS, GB, na(6 * F + 3)>(k + 3);
            step<4, ROWS, GB, na(6 * F + 4)>(k + 4);
            step<5, ROWS, GB, na(6 * F + 5)>(k + 5);
            k += 6;
            if (k >= kend) return false;
            return fill_from<ROWS, F + 1>(k, kend);
        } else {
            return true;
        }
    }
    template <bool ROWS>
    __device__ __forceinline__ void run(int k0, int kend)
    {
        int k = k0;
        bool more = fill_from<ROWS, 0>(k, kend);
        if constexpr (NF % NG != 0) {
            if (more) more = groups_from<ROWS, NF % NG>(k, kend);
        }
        while (more) more = groups_from<ROWS, 0>(k, kend);
    }
};

template <int TS, int S, int SI, int SRC, bool OUT16>
__device__ __forceinline__ void jpipe_stage(const JacobiPass& P, int lane, int b, int strip,
                                            int chunk, float* lring, float* xchg)
{
    using S_t = JPipe<TS, S, SI, SRC, OUT16>;
    constexpr int T = S_t::T, C = 2;
    S_t St;
    St.P = &P;
    St.w = P.w;
    St.h0 = P.h0;
    St.h1 = P.h1;
    St.colbase = strip * P.V - P.Tp;
    St.lo = lane * C;
    St.lane_c = lane * C;
    St.vq = -0.25f;
    asm volatile("" : "+v"(St.vq));
    St.rlo = P.h0;  // as JLag::rlo
    St.rhi = P.h1;
    St.xs0 = strip * P.V - P.Tp + lane * C;
    St.vlo = strip * P.V;
    St.vhi = min(St.vlo + P.V, P.w);
    St.r0 = P.row_lo + chunk * P.rows_per_chunk;
    St.r1 = min(St.r0 + P.rows_per_chunk, P.row_hi);
    St.src = P.src + b * P.sstride;
    St.prev = P.prev + b * P.pstride;
    St.emap = P.emap + b * P.estride;
    St.lnorm = P.lnorm + b * P.lstride;
    St.dst = P.dst + b * P.dstride;
    St.out = P.out + b * P.ostride;
    St.lring = lring + SI * (S_t::R * 64 * C);
    St.xin = SI > 0 ? xchg + (SI - 1) * (2 * 64 * C) : nullptr;
    St.xout = SI < S - 1 ? xchg + SI * (2 * 64 * C) : nullptr;
    St.hcol[0] = St.hcol[1] = 0.0f;
    if (St.xs0 >= 0 && St.xs0 < P.w) { St.hcol[0] = P.hcol[St.xs0]; St.hcol[1] = P.hcol[St.xs0 + 1]; }
#pragma unroll
    for (int l = 0; l < TS; l++)
#pragma unroll
        for (int q = 0; q < 3; q++) St.H[l][q].v = f2{0.0f, 0.0f};
#pragma unroll
    for (int q = 0; q < S_t::NB; q++) { St.In[q].v = f2{0.0f, 0.0f}; St.Lin[q].v = f2{0.0f, 0.0f}; }
    const int k0 = St.r0 - T - 1;  // ring slots count from k0: no alignment (JLag)
    const int kend = St.r1 + 2 * T;
    constexpr int QO = -2 * S_t::TB + 2;
    if constexpr (SI == 0) {
#pragma unroll
        for (int r = 0; r + 1 < S_t::PF; r++) St.In[md(r, S_t::NB)] = St.load_input(k0 + r);
    }
#pragma unroll
    for (int r = 0; r < S_t::PF; r++) St.Lin[md(QO + r, S_t::NB)] = St.load_row(St.lnorm, k0 + QO + r);
    const int wlo = k0 - 2 * T, whi = kend + 3;
    const bool rows = (St.h0 >= wlo && St.h0 <= whi) || (St.h1 >= wlo && St.h1 <= whi);
    // rows is uniform over the workgroup (it depends on the chunk only), so every stage takes the
    // same branch and runs the same number of steps (= barriers)
    if (rows) St.template run<true>(k0, kend);
    else St.template run<false>(k0, kend);
}

template <int TS, int S, int SRC, bool OUT16>
__global__ void __launch_bounds__(64 * S) k_jpipe(JacobiPass P)
{
    constexpr int C = 2, R = JPipe<TS, S, 0, SRC, OUT16>::R;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int job = blockIdx.x;
    if (job >= P.nstrips * P.nchunks) return;  // uniform over the workgroup
    const int b = blockIdx.y;
    const int strip = job % P.nstrips, chunk = job / P.nstrips;
    __shared__ float lring[S * R * 64 * C];
    __shared__ float xchg[(S > 1 ? S - 1 : 1) * 2 * 64 * C];
    // the exchange slots are read one step before they are first written (those rows only
    // feed halo cells); zero them so the stale cells are finite and deterministic
    for (int i = threadIdx.x; i < (S > 1 ? S - 1 : 1) * 2 * 64 * C; i += 64 * S) xchg[i] = 0.0f;
    __syncthreads();
    if (wave == 0) jpipe_stage<TS, S, 0, SRC, OUT16>(P, lane, b, strip, chunk, lring, xchg);
    if constexpr (S > 1) { if (wave == 1) jpipe_stage<TS, S, (S > 1 ? 1 : 0), SRC, OUT16>(P, lane, b, strip, chunk, lring, xchg); }
    if constexpr (S > 2) { if (wave == 2) jpipe_stage<TS, S, (S > 2 ? 2 : 0), SRC, OUT16>(P, lane, b, strip, chunk, lring, xchg); }
    if constexpr (S > 3) { if (wave == 3) jpipe_stage<TS, S, (S > 3 ? 3 : 0), SRC, OUT16>(P, lane, b, strip, chunk, lring, xchg); }
}

#if !defined(PF_JPART) || PF_JPART == 0
// Out-of-band rows of a level: 0 (level 0, Depth.cpp:1449-1452) or the nearest upsample of the
// previous level (Depth.cpp:1467-1485); stored to both ping-pong buffers, or quantised into the
// u16 output on the last level (where the ping-pong buffers get only the rows h0-1 and h1+1).
__global__ void __launch_bounds__(256) k_border(const float* __restrict__ prev, long long pstride,
                                                LevelDims L, float* __restrict__ a,
                                                float* __restrict__ bb, long long stride,
                                                uint16_t* __restrict__ out, long long ostride)
{
    // one panorama's level plane is < 2^31 pixels (the host checks out_w * out_h), so the
    // pixel arithmetic is 32-bit: no 64-bit division in the index split
    const int top = L.h0 * L.w;
    const int bot = (L.h - 1 - L.h1) * L.w;
    const int i = (int)blockIdx.x * 256 + (int)threadIdx.x;
    if (i >= top + bot) return;
    const int b = blockIdx.y;
    const int y = i < top ? i / L.w : L.h1 + 1 + (i - top) / L.w;
    const int x = i < top ? i - y * L.w : (i - top) - (y - L.h1 - 1) * L.w;
    const int o = y * L.w + x;
    float v = 0.0f;
    if (prev) v = prev[b * pstride + (y / 2) * (L.w / 2) + x / 2];
    if (out) {
        float q = v;
        if (q < 0) q = 0;
        if (q > 1) q = 1;
        out[b * ostride + o] = (uint16_t)(q * 65535.0f);
        // the rows next to the band: a pass's loads clamp rows to [h0, h1], but a halo lane's
        // virtual columns past either row end still reach rows h0-1 / h1+1 (the neighbours of
        // the un-windowed rows, whose zero factor needs them finite; JLag::rlo)
        if (a && (y == L.h0 - 1 || y == L.h1 + 1)) {
            a[b * stride + o] = v;
            bb[b * stride + o] = v;
        }
    } else {
        a[b * stride + o] = v;
        bb[b * stride + o] = v;
    }
}

// The same for widths divisible by 4: a thread owns 4 consecutive pixels of a row (one float2
// load of the half-resolution level, 16-B float / 8-B u16 stores).  The per-pixel scalar form
// stored 2 B per lane on the last level (0.09 ms per C3 step at level 2, ~1.2 TB/s).
__global__ void __launch_bounds__(256) k_border4(const float* __restrict__ prev, long long pstride,
                                                 LevelDims L, float* __restrict__ a,
                                                 float* __restrict__ bb, long long stride,
                                                 uint16_t* __restrict__ out, long long ostride)
{
    const int top = L.h0 * L.w;
    const int bot = (L.h - 1 - L.h1) * L.w;
    const int i = 4 * ((int)blockIdx.x * 256 + (int)threadIdx.x);
    if (i >= top + bot) return;
    const int b = blockIdx.y;
    const int y = i < top ? i / L.w : L.h1 + 1 + (i - top) / L.w;
    const int x = i < top ? i - y * L.w : (i - top) - (y - L.h1 - 1) * L.w;
    const int o = y * L.w + x;
    float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (prev) {  // x is a multiple of 4: the pair x/2, x/2+1 is one aligned float2
        const float2 q = *reinterpret_cast<const float2*>(prev + b * pstride + (y / 2) * (L.w / 2) + x / 2);
        v = make_float4(q.x, q.x, q.y, q.y);
    }
    if (out) {
        const float e[4] = {v.x, v.y, v.z, v.w};
        uint32_t u[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            float q = e[k];
            if (q < 0) q = 0;
            if (q > 1) q = 1;
            u[k] = (uint32_t)(uint16_t)(q * 65535.0f);
        }
        *reinterpret_cast<uint2*>(out + b * ostride + o) = make_uint2(u[0] | (u[1] << 16), u[2] | (u[3] << 16));
        if (a && (y == L.h0 - 1 || y == L.h1 + 1)) {  // see k_border
            *reinterpret_cast<float4*>(a + b * stride + o) = v;
            *reinterpret_cast<float4*>(bb + b * stride + o) = v;
        }
    } else {
        *reinterpret_cast<float4*>(a + b * stride + o) = v;
        *reinterpret_cast<float4*>(bb + b * stride + o) = v;
    }
}

#endif

// ---------------------------------------------------------------------------------------------
// The lagged passes of one sweep depth T are built in their own translation unit (the Makefile
// compiles this file once per T with -DPF_JPART=T, and once with PF_JPART=0 for the rest), so the
// 70-odd k_jlag instantiations compile in parallel.
#define PF_JCAT2(a, b) a##b
#define PF_JCAT(a, b) PF_JCAT2(a, b)
#define PF_JDECL(T)                                                                            \
    void PF_JCAT(jlag_launch_t, T)(hipStream_t s, const JacobiPass& P, int C, int batch,      \
                                   bool fast);                                               \
    int PF_JCAT(jlag_waves_t, T)(int C, bool fast);
PF_JDECL(1) PF_JDECL(2) PF_JDECL(4) PF_JDECL(5) PF_JDECL(8) PF_JDECL(10)

#if defined(PF_JPART) && PF_JPART > 0
template <int C, int T, int SRC, bool OUT16, bool FAST>
static void launch_pass_cts(hipStream_t s, const JacobiPass& P, int batch)
{
    long long jobs = (long long)P.nstrips * P.nchunks;
    dim3 grid((unsigned)((jobs + 3) / 4), batch);
    hipLaunchKernelGGL((k_jlag<C, T, SRC, OUT16, FAST>), grid, dim3(256), 0, s, P);
}

template <int C, int T, bool FAST>
static void launch_pass_ct(hipStream_t s, const JacobiPass& P, int batch)
{
    if (P.out_mode) {
        if (P.src_mode == SRC_BUF) launch_pass_cts<C, T, SRC_BUF, true, FAST>(s, P, batch);
        else if (P.src_mode == SRC_UPSAMPLE) launch_pass_cts<C, T, SRC_UPSAMPLE, true, FAST>(s, P, batch);
        else launch_pass_cts<C, T, SRC_SEED, true, FAST>(s, P, batch);
    } else {
        if (P.src_mode == SRC_BUF) launch_pass_cts<C, T, SRC_BUF, false, FAST>(s, P, batch);
        else if (P.src_mode == SRC_UPSAMPLE) launch_pass_cts<C, T, SRC_UPSAMPLE, false, FAST>(s, P, batch);
        else launch_pass_cts<C, T, SRC_SEED, false, FAST>(s, P, batch);
    }
}

template <int C, int T, bool FAST>
static int waves_per_cu_t()
{
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &nb, reinterpret_cast<const void*>(k_jlag<C, T, SRC_BUF, false, FAST>), 256, 0) != hipSuccess)
        nb = 1;
    return nb * 4;
}

// C == 4: packed form in PF_JACOBI_C4P builds, general form in PF_JACOBI_C4 builds (both off by
// default: measured slower than C == 2 on MI355X; they double the build time).
void PF_JCAT(jlag_launch_t, PF_JPART)(hipStream_t s, const JacobiPass& P, int C, int batch, bool fast)
{
    constexpr int T = PF_JPART;
    if (C == 4) {
#if PF_JACOBI_C4
        if (!fast) { launch_pass_ct<4, T, false>(s, P, batch); return; }
#endif
#if PF_JACOBI_C4P
        if (fast) { launch_pass_ct<4, T, true>(s, P, batch); return; }
#endif
        return;  // unreachable: the host checks jstream_supported_C first
    }
#if PF_JACOBI_C3
    if (C == 3) {  // packed form only (jstream_supported_C)
        if (fast) launch_pass_ct<3, T, true>(s, P, batch);
        return;
    }
#endif
    if (fast) launch_pass_ct<2, T, true>(s, P, batch);
    else launch_pass_ct<2, T, false>(s, P, batch);
}

int PF_JCAT(jlag_waves_t, PF_JPART)(int C, bool fast)
{
    constexpr int T = PF_JPART;
    if (C == 4) {
#if PF_JACOBI_C4
        if (!fast) return waves_per_cu_t<4, T, false>();
#endif
#if PF_JACOBI_C4P
        if (fast) return waves_per_cu_t<4, T, true>();
#endif
        return 4;
    }
#if PF_JACOBI_C3
    if (C == 3) return fast ? waves_per_cu_t<3, T, true>() : 4;
#endif
    return fast ? waves_per_cu_t<2, T, true>() : waves_per_cu_t<2, T, false>();
}
#else  // PF_JPART == 0: dispatch, the pipelined engine, the border kernel

bool jstream_supported_T(int T) { return T == 1 || T == 2 || T == 4 || T == 5 || T == 8 || T == 10; }

static int waves_per_cu_c(int C, int T, bool fast)
{
    switch (T) {
        case 1: return jlag_waves_t1(C, fast);
        case 2: return jlag_waves_t2(C, fast);
        case 4: return jlag_waves_t4(C, fast);
        case 5: return jlag_waves_t5(C, fast);
        case 8: return jlag_waves_t8(C, fast);
        default: return jlag_waves_t10(C, fast);
    }
}

// Resident waves per CU of the pass kernel at depth T (used to size the grid to whole rounds).
int jstream_waves_per_cu(int C, int T, bool fast)
{
    static int cache[3][2][11] = {{{0}}};
    if (T < 1 || T > 10 || !jstream_supported_T(T)) return 4;
    int& c = cache[C == 4 ? 1 : (C == 3 ? 2 : 0)][fast ? 1 : 0][T];
    if (!c) c = waves_per_cu_c(C == 4 ? 4 : (C == 3 ? 3 : 2), T, fast);
    return c;
}

bool jstream_supported_C(int C, bool fast)
{
    if (C == 2) return true;
    if (C == 3) return fast && PF_JACOBI_C3 != 0;
    if (C != 4) return false;
    return fast ? PF_JACOBI_C4P != 0 : PF_JACOBI_C4 != 0;
}

void launch_jstream(hipStream_t s, const JacobiPass& P, int C, int T, int batch, bool fast)
{
    switch (T) {
        case 1: jlag_launch_t1(s, P, C, batch, fast); break;
        case 2: jlag_launch_t2(s, P, C, batch, fast); break;
        case 4: jlag_launch_t4(s, P, C, batch, fast); break;
        case 5: jlag_launch_t5(s, P, C, batch, fast); break;
        case 8: jlag_launch_t8(s, P, C, batch, fast); break;
        default: jlag_launch_t10(s, P, C, batch, fast); break;
    }
}

// Pipelined passes (k_jpipe): T = S * TS.
template <int TS, int S>
static void launch_pipe_ts(hipStream_t s, const JacobiPass& P, int batch)
{
    dim3 grid((unsigned)(P.nstrips * P.nchunks), batch);
    if (P.out_mode) {
        if (P.src_mode == SRC_BUF) hipLaunchKernelGGL((k_jpipe<TS, S, SRC_BUF, true>), grid, dim3(64 * S), 0, s, P);
        else if (P.src_mode == SRC_UPSAMPLE) hipLaunchKernelGGL((k_jpipe<TS, S, SRC_UPSAMPLE, true>), grid, dim3(64 * S), 0, s, P);
        else hipLaunchKernelGGL((k_jpipe<TS, S, SRC_SEED, true>), grid, dim3(64 * S), 0, s, P);
    } else {
        if (P.src_mode == SRC_BUF) hipLaunchKernelGGL((k_jpipe<TS, S, SRC_BUF, false>), grid, dim3(64 * S), 0, s, P);
        else if (P.src_mode == SRC_UPSAMPLE) hipLaunchKernelGGL((k_jpipe<TS, S, SRC_UPSAMPLE, false>), grid, dim3(64 * S), 0, s, P);
        else hipLaunchKernelGGL((k_jpipe<TS, S, SRC_SEED, false>), grid, dim3(64 * S), 0, s, P);
    }
}

// (S, TS) pairs the pipelined engine is built for; T = S * TS
bool jpipe_supported(int S, int TS) { return S == 2 && (TS == 5 || TS == 4); }

void launch_jpipe(hipStream_t s, const JacobiPass& P, int S, int TS, int batch)
{
    if (S == 2 && TS == 5) launch_pipe_ts<5, 2>(s, P, batch);
    else if (S == 2 && TS == 4) launch_pipe_ts<4, 2>(s, P, batch);
}

template <int TS, int S>
static int pipe_waves_per_cu_t()
{
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &nb, reinterpret_cast<const void*>(k_jpipe<TS, S, SRC_BUF, false>), 64 * S, 0) != hipSuccess)
        nb = 1;
    return nb * S;
}

int jpipe_waves_per_cu(int S, int TS)
{
    static int cache[2] = {0, 0};
    const int i = TS == 5 ? 0 : 1;
    if (!cache[i]) cache[i] = TS == 5 ? pipe_waves_per_cu_t<5, 2>() : pipe_waves_per_cu_t<4, 2>();
    (void)S;
    return cache[i];
}

void launch_border(hipStream_t s, const float* prev, long long pstride, LevelDims L, float* a,
                   float* b, long long stride, uint16_t* out, long long ostride, int batch)
{
    long long n = (long long)(L.h0 + (L.h - 1 - L.h1)) * L.w;
    if (n <= 0) return;
    // the vector form needs 4 | w (then the plane strides are multiples of 4 too: aligned stores)
    if (L.w % 4 == 0 && stride % 4 == 0 && ostride % 4 == 0 && pstride % 2 == 0) {
        dim3 grid((unsigned)((n / 4 + 255) / 256), batch);
        hipLaunchKernelGGL(k_border4, grid, dim3(256), 0, s, prev, pstride, L, a, b, stride, out,
                           ostride);
        return;
    }
    dim3 grid((unsigned)((n + 255) / 256), batch);
    hipLaunchKernelGGL(k_border, grid, dim3(256), 0, s, prev, pstride, L, a, b, stride, out,
                       ostride);
}

#endif  // PF_JPART

}  // namespace pf
