// pf_jres.hip -- resident damped Jacobi for the coarse fusion level: ONE launch runs all of the
// level's sweeps (Depth.cpp:1649-1718; 200 at level 0).
//
// Why: the level-0 band of a C3 panorama is 512 x 185 pixels.  The streaming engine
// (pf_jacobi.hip) covers it with ~2 waves per SIMD and pays 40 launches, each with its 3T-1
// fill/drain steps per row chunk and its load latency (0.92-0.99 ms per 64 panoramas, 0.11 of
// the VALU roof).  Here the level stays on chip for all its sweeps:
//
//  * A workgroup (16 waves) owns a block of band rows of one panorama: `core` rows plus K halo
//    rows on each side, 16*RS rows in all, at CPL = w/64 columns per lane -- a wave holds RS
//    whole rows (its lanes side by side across the row), so every horizontal neighbour is in the
//    lane's own registers except one per row end, which crosses one lane by DPP.  The levels
//    b and L live in VGPRs for the whole launch (L is read from HBM once, not once per pass).
//  * Vertical neighbours across waves go through LDS: after every sweep each wave writes its
//    first and last row (double-buffered by sweep parity, so one workgroup barrier per sweep).
//  * Blocks of one panorama exchange K rows with their neighbours every K sweeps (a "round"):
//    after k sweeps of a round the rows within k of a block edge are stale, so after K sweeps
//    exactly the core is current, and the neighbours' cores refresh the halos.  The hand-off is
//    the write-through form of MI355X_MICROARCH.md (inter-workgroup visibility): sc1 row stores,
//    every storing wave's vmcnt(0), a workgroup barrier, one sc1 flag store; the consumer polls
//    the flag with one lane's sc1 load, joins a barrier, then reads the rows with sc1 loads.
//  * Deadlock freedom without co-residency: a workgroup takes its (panorama, block) from a
//    ticket counter when it STARTS, so the blocks holding tickets are running, groups are filled
//    in ticket order, and at most one group of a launch is incomplete at any time; every other
//    running group finishes on its own.  A launch needs only `nb` workgroups resident at once
//    (checked on the host), however many other kernels share the chip.  Spins are bounded: a
//    timeout counts into an error word instead of hanging the GPU, and the host turns a non-zero
//    count into PF_ETIMEOUT for the fusion (pf_synchronize, the next pf_fuse / pf_merge).
//
// Arithmetic: the packed form of pf_jacobi.hip (JLag::sweep_packed_group), bit-identical to the
// reference's fp32 operand order: Lcur = ((((W*q) + N*q) + C) + S*q) + E*q with q = -1/4 (every
// product by q is exact, so the adds fold into FMAs that round where the reference rounds),
// t = b + (L - Lcur)*H, b' = clamp01(t*(1-1e-4) + b*1e-4), H = 0.5 on windowed pixels and 0 on
// un-windowed ones (the host's separable-coverage certificate; column 0 is never windowed, so the
// west tap of column 0 is never needed).  The east tap of column w-1 is pixel (0, Y+1): the
// reference's linear buffer[yy*width + xx] addressing.
#include "pf_internal.hpp"

namespace pf {

namespace {

typedef float f2 __attribute__((ext_vector_type(2)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float dpp_shr(float v)
{  // lane i <- lane i-1 (wave_shr:1), lane 0 <- 0
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xF, 0xF, true));
}
__device__ __forceinline__ float dpp_rol(float v)
{  // lane i <- lane (i+1) mod 64 (wave_rol:1)
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x134, 0xF, 0xF, false));
}
// acc + x[(lane + 1) mod 64] * q in one v_fmac_f32_dpp (wave_rol:1), one rounding: the E tap of
// a lane's last column (hipcc folds a DPP move into v_add_f32, not into the tied v_fmac_f32).
// x is a select computed just before (the seam lane's operand), and the hazard recognizer does
// not see into inline asm: the two wait states a DPP read of a fresh VGPR needs are the s_nop
// (tools/dpp_hazards.py, tests/test_dpp_hazards.py)
__device__ __forceinline__ float fmac_rol(float acc, float x, float q)
{
    asm("s_nop 1\n\tv_fmac_f32_dpp %0, %1, %2 wave_rol:1 row_mask:0xf bank_mask:0xf"
        : "+v"(acc) : "v"(x), "v"(q));
    return acc;
}
__device__ __forceinline__ f2 pk_add_clamp01(f2 a, f2 b)
{
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 clamp" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float add_scalar(float a, float b)
{
    float r;
    asm("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float fma_scalar(float a, float b, float c)
{
    float r;
    asm("v_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

#ifndef PF_JRES_LDSFLAG
#define PF_JRES_LDSFLAG 0  // barrier-free sweeps + per-row hand-off flags (measured: same time as barriers)
#endif
#ifndef PF_JRES_EARLY_EDGE
// 1: a wave's new last row goes to LDS before its row 0 is computed (the store overlaps row 0's
// arithmetic).  Round 6, three alternating serial rounds on one MI355X: 506-528 us against
// 508-523 us per C3 launch: no change.  Off.
#define PF_JRES_EARLY_EDGE 0
#endif
#ifndef PF_JRES_GRANULE
#define PF_JRES_GRANULE 0  // hand-off by data-tagged granules (measured 2x slower: 32-KB edges)
#endif

// sc1 (write-through / L2-bypassing) buffer accesses for the inter-workgroup row hand-off
constexpr int kSC1 = 16;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

}  // namespace

// A bounded wait gave up: count it on the device (pf_jres_errors) and raise the host's flag
// (coherent pinned memory; the host reports PF_ETIMEOUT).  Only on the failure path.
__device__ __forceinline__ void jres_timeout(const JresArgs& A)
{
    __hip_atomic_fetch_add(A.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (A.err_host) __hip_atomic_store(A.err_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int CPL, int RS, int NWV, int SRC, bool OUT16>
struct JRes {
    static constexpr int NP = CPL / 2;  // column pairs per lane
    static constexpr int NW = NWV;      // waves per workgroup
    f2 b[RS][NP];   // the level, rows wv*RS + r of the block's region
    f2 L[RS][NP];   // targets (sanitised: non-finite -> 0)
    f2 hc[NP];      // H of the lane's columns
    float vq;       // -1/4 in a VGPR
    int lane, wv;

    // new values of row R (in place) from N = the old row above and S = the row below (old);
    // on return N holds row R's old value (the next row's N).  EDGE: H = 0.
    template <int R, bool EDGE>
    __device__ __forceinline__ void row(f2* N, const f2* S)
    {
        const f2 q = {-0.25f, -0.25f};
        const f2 reg = {(float)1e-4, (float)1e-4};
        const f2 reg_ = {1 - (float)1e-4, 1 - (float)1e-4};
        f2* c = b[R];
        // east tap of the lane's last column: the next lane's first column of this row; for
        // lane 63 (column w-1) lane 0's first column of the row below -- pixel (0, Y+1)
        const float xr = lane == 0 ? S[0].x : c[0].x;
        f2 cur[NP];
#pragma unroll
        for (int k = 0; k < NP; k++) {
            // W + N (the W*q + N*q of the reference, scaled by q below)
            const float wx = k == 0 ? dpp_shr(c[NP - 1].y) : c[k - 1].y;
            cur[k].x = (k == 0) ? (wx + N[k].x) : add_scalar(wx, N[k].x);
            cur[k].y = add_scalar(c[k].x, N[k].y);
        }
#pragma unroll
        for (int k = 0; k < NP; k++) cur[k] = __builtin_elementwise_fma(cur[k], q, c[k]);
#pragma unroll
        for (int k = 0; k < NP; k++) cur[k] = __builtin_elementwise_fma(S[k], q, cur[k]);
#pragma unroll
        for (int k = 0; k < NP; k++) {
            cur[k].x = fma_scalar(c[k].y, vq, cur[k].x);
            if (k == NP - 1) cur[k].y = fmac_rol(cur[k].y, xr, vq);  // E from the next lane
            else cur[k].y = fma_scalar(c[k + 1].x, vq, cur[k].y);
        }
#pragma unroll
        for (int k = 0; k < NP; k++) {
            N[k] = c[k];
            if constexpr (EDGE) {
                // un-windowed row (h0 or h1): t = b exactly
                c[k] = pk_add_clamp01(c[k] * reg_, c[k] * reg);
            } else {
                const f2 t = __builtin_elementwise_fma(L[R][k] - cur[k], hc[k], c[k]);
                c[k] = pk_add_clamp01(t * reg_, c[k] * reg);
            }
        }
    }

    // one sweep over the wave's rows.  The rows that need the neighbour waves' edge rows (row 0:
    // the row above, from LDS; row RS-1: the row below) go last, so the LDS reads issued at the
    // start of the sweep land while rows 1..RS-2 are computed: rows 1..RS-1 top to bottom (n =
    // old row 0, then each row's old value for the next), then row 0 with S = old row 1 (kept).
    // HAS_EDGE: this wave holds row h0 or h1 (bit r of em), which only two waves of a panorama
    // do, so the others run the branch-free body.
    template <int R, bool HAS_EDGE>
    __device__ __forceinline__ void rows_mid(f2* n, const f2* dn, uint32_t em)
    {
        if constexpr (R < RS) {
            const f2* S = R + 1 < RS ? b[R + 1 < RS ? R + 1 : 0] : dn;
            if (HAS_EDGE && (em & (1u << R))) row<R, true>(n, S);
            else row<R, false>(n, S);
            rows_mid<R + 1, HAS_EDGE>(n, dn, em);
        }
    }
    // bot_out (JRES_EARLY_EDGE): the LDS slot of this wave's new last row, stored as soon as
    // that row is done, so the store overlaps row 0's arithmetic instead of joining the stores
    // every wave issues just before the sweep's barrier
    template <bool HAS_EDGE>
    __device__ __forceinline__ void sweep(const f2* up_lds, const f2* dn_lds, uint32_t em,
                                          f2* bot_out = nullptr)
    {
        f2 up[NP], dn[NP], s1[NP], n[NP];
#pragma unroll
        for (int k = 0; k < NP; k++) {
            up[k] = up_lds ? up_lds[64 * k] : f2{0.0f, 0.0f};
            dn[k] = dn_lds ? dn_lds[64 * k] : f2{0.0f, 0.0f};
            s1[k] = b[RS > 1 ? 1 : 0][k];
            n[k] = b[0][k];
        }
        if constexpr (RS > 1) rows_mid<1, HAS_EDGE>(n, dn, em);
        if (RS > 1 && bot_out)
#pragma unroll
            for (int k = 0; k < NP; k++) bot_out[64 * k] = b[RS - 1][k];
        if (HAS_EDGE && (em & 1u)) row<0, true>(up, RS > 1 ? s1 : dn);
        else row<0, false>(up, RS > 1 ? s1 : dn);
    }
};

template <int CPL, int RS, int NWV, int SRC, bool OUT16>
__global__ void __launch_bounds__(64 * NWV) k_jres(JresArgs A)
{
    using S_t = JRes<CPL, RS, NWV, SRC, OUT16>;
    constexpr int NP = S_t::NP, NW = S_t::NW;
    // [sweep parity][0 top / 1 bottom][wave][column pair k][lane]: a lane's pair k of a wave's
    // first / last row; lane-minor, so the 8-B accesses of a wave are conflict-free
    __shared__ f2 lds_edge[2][2][NW][NP][64];
    __shared__ uint32_t lds_ticket;
    const int tid = threadIdx.x;
    S_t S;
    S.lane = tid & 63;
    S.wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    S.vq = -0.25f;
    asm volatile("" : "+v"(S.vq));
    const int lane = S.lane, wv = S.wv;
    if (tid == 0) lds_ticket = __hip_atomic_fetch_add(A.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const uint32_t t = __builtin_amdgcn_readfirstlane(lds_ticket - A.tbase);
    const int p = (int)(t / (uint32_t)A.nb), j = (int)(t % (uint32_t)A.nb);
    const int w = A.w;
    const int c0 = A.h0 + j * A.core;
    const int c1 = min(c0 + A.core, A.h1 + 1);
    const int K = A.K;
    const int rs = j == 0 ? A.h0 : c0 - K;                       // region's first row
    const int re = j == A.nb - 1 ? A.h1 + 1 : min(c1 + K, A.h1 + 1);  // one past its last row
    const int x0 = lane * CPL;
    const int qc0 = c0 - rs, qc1 = c1 - rs;  // the core in region rows

    // ---- initial state of the region, targets, H
    {
        const float* lp = A.lnorm + p * A.lstride;
#pragma unroll
        for (int k = 0; k < NP; k++) {
            S.hc[k].x = A.hcol[x0 + 2 * k];
            S.hc[k].y = A.hcol[x0 + 2 * k + 1];
        }
#pragma unroll
        for (int r = 0; r < RS; r++) {
            const int Y = rs + wv * RS + r;
            const bool live = Y < re;
#pragma unroll
            for (int k = 0; k < NP; k++) {
                float v0 = 0.0f, v1 = 0.0f, l0 = 0.0f, l1 = 0.0f;
                if (live) {
                    const int x = x0 + 2 * k;
                    if constexpr (SRC == 2) {  // level-0 seed (Depth.cpp:1442-1465)
                        const float* ep = A.emap + p * A.estride + A.erow[Y + 1];
                        v0 = ep[A.ecol[x + 1]];
                        v1 = ep[A.ecol[x + 2]];
                    } else if constexpr (SRC == 1) {  // nearest upsample (Depth.cpp:1467-1485)
                        v0 = v1 = A.prev[p * A.pstride + (long long)(Y >> 1) * (w >> 1) + (x >> 1)];
                    } else {
                        const float2 q = *reinterpret_cast<const float2*>(A.src + p * A.sstride + (long long)Y * w + x);
                        v0 = q.x;
                        v1 = q.y;
                    }
                    const float2 lq = *reinterpret_cast<const float2*>(lp + (long long)Y * w + x);
                    l0 = __builtin_isfinite(lq.x) ? lq.x : 0.0f;
                    l1 = __builtin_isfinite(lq.y) ? lq.y : 0.0f;
                }
                S.b[r][k] = f2{v0, v1};
                S.L[r][k] = f2{l0, l1};
            }
        }
    }
    // rows h0 / h1 of this wave: un-windowed (their update ignores the neighbours)
    uint32_t em = 0;
#pragma unroll
    for (int r = 0; r < RS; r++) {
        const int Y = rs + wv * RS + r;
        if (Y == A.h0 || Y == A.h1) em |= 1u << r;
    }
    em = __builtin_amdgcn_readfirstlane(em);

    const auto put_edges = [&](int pb) {
#pragma unroll
        for (int k = 0; k < NP; k++) {
            lds_edge[pb][0][wv][k][lane] = S.b[0][k];
            lds_edge[pb][1][wv][k][lane] = S.b[RS - 1][k];
        }
    };

    const long long xplane = (long long)K * w;  // floats of one published edge
    float* const xb = A.xbuf;
#if PF_JRES_LDSFLAG
    // Barrier-free sweeps: wave w starts sweep s+1 once its neighbour waves have published their
    // edge rows of state s (an LDS flag per wave), so a wave runs at most one sweep ahead of its
    // neighbours and, while the halo waves wait for a hand-off, the waves further in keep
    // sweeping (a wave d waves from the halo can run d sweeps ahead).  Edge rows of state s sit in
    // buffer s & 1: wave w overwrites buffer s & 1 only after its neighbours published state s+1,
    // i.e. after they read state s-1 from it.  The hand-off is per row: each published row
    // carries its own flag (one sc1 store after the storing wave's vmcnt(0)); a halo wave polls
    // the flags of its own rows only.  No workgroup barrier after the start.
    __shared__ int eflag[NW];
    auto publish_edges = [&](int st) {
        put_edges(st & 1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) *reinterpret_cast<volatile int*>(&eflag[wv]) = st;
    };
    auto wait_edges = [&](int nbw, int st) {
        int spins = 0;
        while (*reinterpret_cast<volatile int*>(&eflag[nbw]) < st) {
            __builtin_amdgcn_s_sleep(0);
            if (++spins > (1 << 26)) {
                if (lane == 0) jres_timeout(A);
                break;
            }
        }
        asm volatile("" ::: "memory");  // the edge reads below stay after the flag read
    };
    // halo rows of this wave (refreshed from the neighbour blocks after every round), as bits
    uint32_t halo = 0;
#pragma unroll
    for (int r = 0; r < RS; r++) {
        const int Y = rs + wv * RS + r;
        if ((j > 0 && Y >= c0 - K && Y < c0) || (j < A.nb - 1 && Y >= c1 && Y < re)) halo |= 1u << r;
    }
    halo = __builtin_amdgcn_readfirstlane(halo);
    uint32_t* const gflag = A.flags;  // [batch][nb][2 edge][K] per published row
    publish_edges(0);
    __syncthreads();  // every wave's state-0 edges and flag in place
    int s = 0, round = 0;
    while (true) {
        const int n = min(K, A.iters - s);
        for (int i = 0; i < n; i++) {
            if (wv > 0) wait_edges(wv - 1, s);
            if (wv < NW - 1) wait_edges(wv + 1, s);
            const int cb = s & 1;
            const f2* up = wv > 0 ? &lds_edge[cb][1][wv > 0 ? wv - 1 : 0][0][lane] : nullptr;
            const f2* dn = wv < NW - 1 ? &lds_edge[cb][0][wv < NW - 1 ? wv + 1 : 0][0][lane] : nullptr;
            const int reach = n - 1 - i;
            const bool skip = (j > 0 && wv * RS + RS - 1 < qc0 - reach) ||
                              (j < A.nb - 1 && wv * RS >= qc1 + reach);
            if (!(A.dbg & 4) && !skip) {
                if (em) S.template sweep<true>(up, dn, em);
                else S.template sweep<false>(up, dn, em);
            }
            s++;
            // a halo wave publishes its end-of-round edges after the hand-off refreshed its rows
            if (!(i == n - 1 && halo && s < A.iters)) publish_edges(s);
        }
        round++;
        if (s >= A.iters) break;
        if (A.dbg & 1) {
            if (halo) publish_edges(s);
            continue;
        }
        int xl = x0;
        asm volatile("" : "+v"(xl));
        const int par = round & 1;
        const uint32_t want = A.fbase + (uint32_t)round;
        // publish: this wave's core rows that a neighbour block needs (sc1 stores, drained, then
        // one sc1 flag per row)
        {
            float* mine = xb + ((long long)(p * A.nb + j) * 2 + par) * 2 * xplane;
            const auto mr = rsrc(mine, (uint32_t)(sizeof(float) * xplane * 2));
            uint32_t pubm = 0;  // bit 2r+e: row r published in edge set e
#pragma unroll
            for (int r = 0; r < RS; r++) {
                const int Y = rs + wv * RS + r;
#pragma unroll
                for (int e = 0; e < 2; e++) {
                    const bool pub = e == 0 ? (j > 0 && Y >= c0 && Y < c0 + K)
                                            : (j < A.nb - 1 && Y >= c1 - K && Y < c1);
                    if (!pub) continue;  // wave-uniform
                    pubm |= 1u << (2 * r + e);
                    const int yo = e == 0 ? Y - c0 : Y - (c1 - K);
                    const int off = (int)(sizeof(float) * (e * xplane + (long long)yo * w + xl));
#pragma unroll
                    for (int k = 0; k < NP; k += 2) {
                        u4v v;
                        v[0] = __float_as_uint(S.b[r][k].x);
                        v[1] = __float_as_uint(S.b[r][k].y);
                        v[2] = __float_as_uint(S.b[r][k + 1].x);
                        v[3] = __float_as_uint(S.b[r][k + 1].y);
                        __builtin_amdgcn_raw_buffer_store_b128(v, mr, off + 8 * k, 0, kSC1);
                    }
                }
            }
            if (pubm) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                // lane 2r+e flags row r of edge set e
                if (lane < 2 * RS && ((pubm >> lane) & 1u)) {
                    const int r = lane >> 1, e = lane & 1;
                    const int Y = rs + wv * RS + r;
                    const int yo = e == 0 ? Y - c0 : Y - (c1 - K);
                    __hip_atomic_store(&gflag[((long long)(p * A.nb + j) * 2 + e) * K + yo], want,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
        if (halo) {
            // poll the flags of this wave's halo rows (lane r: row r), then load them
            int spins = 0;
            while (true) {
                bool ok = true;
                if (lane < RS && ((halo >> lane) & 1u)) {
                    const int Y = rs + wv * RS + lane;
                    const bool top = j > 0 && Y < c0;
                    const int sj = top ? j - 1 : j + 1, e = top ? 1 : 0;
                    const int yo = top ? Y - (c0 - K) : Y - c1;
                    const uint32_t f = __hip_atomic_load(&gflag[((long long)(p * A.nb + sj) * 2 + e) * K + yo],
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok = (int)(f - want) >= 0;
                }
                if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1 << A.spin_log2)) {
                    if (lane == 0) jres_timeout(A);
                    break;
                }
            }
#pragma unroll
            for (int r = 0; r < RS; r++) {
                if (!((halo >> r) & 1u)) continue;  // wave-uniform
                const int Y = rs + wv * RS + r;
                const bool top = j > 0 && Y < c0;
                const int sj = top ? j - 1 : j + 1, e = top ? 1 : 0;
                const int yo = top ? Y - (c0 - K) : Y - c1;
                const float* theirs = xb + ((long long)(p * A.nb + sj) * 2 + par) * 2 * xplane;
                const auto tr = rsrc(theirs, (uint32_t)(sizeof(float) * xplane * 2));
                const int off = (int)(sizeof(float) * (e * xplane + (long long)yo * w + xl));
#pragma unroll
                for (int k = 0; k < NP; k += 2) {
                    const u4v v = __builtin_amdgcn_raw_buffer_load_b128(tr, off + 8 * k, 0, kSC1);
                    S.b[r][k] = f2{__uint_as_float(v[0]), __uint_as_float(v[1])};
                    S.b[r][k + 1] = f2{__uint_as_float(v[2]), __uint_as_float(v[3])};
                }
            }
            publish_edges(s);
        }
    }
#else
    int s = 0, round = 0;
    while (true) {
        const int n = min(K, A.iters - s);
        put_edges(0);
        __syncthreads();
        for (int i = 0; i < n; i++) {
            const int cb = i & 1;
            const f2* up = wv > 0 ? &lds_edge[cb][1][wv > 0 ? wv - 1 : 0][0][lane] : nullptr;
            const f2* dn = wv < NW - 1 ? &lds_edge[cb][0][wv < NW - 1 ? wv + 1 : 0][0][lane] : nullptr;
            // Dependency cone: sweep i of the round only needs the rows within n-1-i of the core;
            // a wave whose rows all lie outside it skips the sweep (its rows feed only rows that
            // are no longer needed, and the hand-off refreshes them before the next round).
            const int reach = n - 1 - i;
            const bool skip = (j > 0 && wv * RS + RS - 1 < qc0 - reach) ||
                              (j < A.nb - 1 && wv * RS >= qc1 + reach);
            if (!(A.dbg & 4) && !skip) {
#if PF_JRES_EARLY_EDGE
                f2* bot = RS > 1 && !(A.dbg & 8) ? &lds_edge[cb ^ 1][1][wv][0][lane] : nullptr;
#else
                f2* bot = nullptr;
#endif
                if (em) S.template sweep<true>(up, dn, em, bot);
                else S.template sweep<false>(up, dn, em, bot);
                if (!(A.dbg & 8)) {
                    if (bot) {  // the last row went out inside the sweep
#pragma unroll
                        for (int k = 0; k < NP; k++) lds_edge[cb ^ 1][0][wv][k][lane] = S.b[0][k];
                    } else {
                        put_edges(cb ^ 1);
                    }
                    __syncthreads();
                }
            } else if (!(A.dbg & 8)) {
                put_edges(cb ^ 1);
                __syncthreads();
            }
        }
        s += n;
        round++;
        if (s >= A.iters) break;
        if (A.dbg & 1) continue;

        // ---- hand-off: publish the core's first / last K rows, take the neighbours'
        // (the lane offset is re-materialised here so that the per-row offsets below are not
        // hoisted out of the round loop, where they would sit in VGPRs through the sweeps)
        int xl = x0;
        asm volatile("" : "+v"(xl));
        const int par = round & 1;
        const uint32_t want = A.fbase + (uint32_t)round;
#if PF_JRES_GRANULE
        // Data-tagged granules (MI355X_MICROARCH.md, handoff-1to1): every float travels as one
        // 8-B {value, round tag} granule, stored write-through (sc1) with no wait and no flag;
        // the consumer waves re-read their rows (sc1) until every tag is this round's.  Parity
        // slots: a block overwrites slot (round & 1) only after taking its neighbours' rows of
        // the round in between, which they publish after reading this slot.
        uint32_t* const gb = reinterpret_cast<uint32_t*>(xb);
        const long long gplane = 2 * xplane;  // uint32 words of one published edge
        const uint32_t gbytes = (uint32_t)(sizeof(uint32_t) * gplane * 2);
        const auto mr = rsrc(gb + ((long long)(p * A.nb + j) * 2 + par) * 2 * gplane, gbytes);
#pragma unroll
        for (int r = 0; r < RS; r++) {
            const int Y = rs + wv * RS + r;
#pragma unroll
            for (int e = 0; e < 2; e++) {  // a row can be in both published sets when core < 2K
                const bool pub = e == 0 ? (j > 0 && Y >= c0 && Y < c0 + K)
                                        : (j < A.nb - 1 && Y >= c1 - K && Y < c1);
                if (!pub) continue;  // wave-uniform
                const int yo = e == 0 ? Y - c0 : Y - (c1 - K);
                const int off = (int)(sizeof(uint32_t) * (e * gplane + 2 * ((long long)yo * w + xl)));
#pragma unroll
                for (int k = 0; k < NP; k++) {
                    const u4v v = {__float_as_uint(S.b[r][k].x), want, __float_as_uint(S.b[r][k].y), want};
                    __builtin_amdgcn_raw_buffer_store_b128(v, mr, off + 16 * k, 0, kSC1);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < RS; r++) {
            const int Y = rs + wv * RS + r;
            int src_j = -1, e = 0, yo = 0;
            if (j > 0 && Y >= c0 - K && Y < c0) { src_j = j - 1; e = 1; yo = Y - (c0 - K); }
            else if (j < A.nb - 1 && Y >= c1 && Y < re) { src_j = j + 1; e = 0; yo = Y - c1; }
            if (src_j >= 0) {  // wave-uniform
                const auto tr = rsrc(gb + ((long long)(p * A.nb + src_j) * 2 + par) * 2 * gplane, gbytes);
                const int off = (int)(sizeof(uint32_t) * (e * gplane + 2 * ((long long)yo * w + xl)));
                int spins = 0;
                while (true) {
                    bool ok = true;
#pragma unroll
                    for (int k = 0; k < NP; k++) {
                        const u4v v = __builtin_amdgcn_raw_buffer_load_b128(tr, off + 16 * k, 0, kSC1);
                        S.b[r][k] = f2{__uint_as_float(v[0]), __uint_as_float(v[2])};
                        ok = ok && v[1] == want && v[3] == want;
                    }
                    if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;  // every lane's granules current
                    __builtin_amdgcn_s_sleep(1);
                    if (++spins > (1 << (A.spin_log2 - 2))) {  // bounded: counted, never hangs
                        if (lane == 0) jres_timeout(A);
                        break;
                    }
                }
            }
        }
#else
        float* mine = xb + ((long long)(p * A.nb + j) * 2 + par) * 2 * xplane;
        const auto mr = rsrc(mine, (uint32_t)(sizeof(float) * xplane * 2));
#pragma unroll
        for (int r = 0; r < RS; r++) {
            const int Y = rs + wv * RS + r;
            // a row can be in both published sets when core < 2K
#pragma unroll
            for (int e = 0; e < 2; e++) {
                const bool pub = e == 0 ? (j > 0 && Y >= c0 && Y < c0 + K)
                                        : (j < A.nb - 1 && Y >= c1 - K && Y < c1);
                if (!pub) continue;  // wave-uniform
                const int yo = e == 0 ? Y - c0 : Y - (c1 - K);
                const int off = (int)(sizeof(float) * (e * xplane + (long long)yo * w + xl));
#pragma unroll
                for (int k = 0; k < NP; k += 2) {
                    u4v v;
                    v[0] = __float_as_uint(S.b[r][k].x);
                    v[1] = __float_as_uint(S.b[r][k].y);
                    v[2] = __float_as_uint(S.b[r][k + 1].x);
                    v[3] = __float_as_uint(S.b[r][k + 1].y);
                    __builtin_amdgcn_raw_buffer_store_b128(v, mr, off + 8 * k, 0, kSC1);
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (!((A.dbg & 16) && j == 0))  // the fault hook withholds block 0's flag
                __hip_atomic_store(&A.flags[p * A.nb + j], want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // wait for the neighbours' rows of this round (bounded: a timeout is counted, never hangs)
            for (int nbj = j - 1; nbj <= j + 1; nbj += 2) {
                if (nbj < 0 || nbj >= A.nb) continue;
                uint32_t* f = &A.flags[p * A.nb + nbj];
                int spins = 0;
                while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - want) < 0) {
                    __builtin_amdgcn_s_sleep(2);
                    if (++spins > (1 << A.spin_log2)) {
                        jres_timeout(A);
                        break;
                    }
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < RS; r++) {
            const int Y = rs + wv * RS + r;
            int src_j = -1, e = 0, yo = 0;
            if (j > 0 && Y >= c0 - K && Y < c0) { src_j = j - 1; e = 1; yo = Y - (c0 - K); }
            else if (j < A.nb - 1 && Y >= c1 && Y < re) { src_j = j + 1; e = 0; yo = Y - c1; }
            if (src_j >= 0) {  // wave-uniform
                const float* theirs = xb + ((long long)(p * A.nb + src_j) * 2 + par) * 2 * xplane;
                const auto tr = rsrc(theirs, (uint32_t)(sizeof(float) * xplane * 2));
                const int off = (int)(sizeof(float) * (e * xplane + (long long)yo * w + xl));
#pragma unroll
                for (int k = 0; k < NP; k += 2) {
                    const u4v v = __builtin_amdgcn_raw_buffer_load_b128(tr, off + 8 * k, 0, kSC1);
                    S.b[r][k] = f2{__uint_as_float(v[0]), __uint_as_float(v[1])};
                    S.b[r][k + 1] = f2{__uint_as_float(v[2]), __uint_as_float(v[3])};
                }
            }
        }
#endif
    }

#endif

    // ---- the core rows of the finished level
#pragma unroll
    for (int r = 0; r < RS; r++) {
        const int Y = rs + wv * RS + r;
        if (Y < c0 || Y >= c1) continue;  // wave-uniform
        const long long o = (long long)Y * w + x0;
        if constexpr (OUT16) {
            uint16_t* op = A.out + p * A.ostride + o;
#pragma unroll
            for (int k = 0; k < NP; k++) {
                // quantise (Depth.cpp:1721-1736); b is already in [0, 1], truncating cast
                const uint32_t q0 = (uint32_t)(S.b[r][k].x * 65535.0f);
                const uint32_t q1 = (uint32_t)(S.b[r][k].y * 65535.0f);
                *reinterpret_cast<uint32_t*>(op + 2 * k) = q0 | (q1 << 16);
            }
        } else {
            float* dp = A.dst + p * A.dstride + o;
#pragma unroll
            for (int k = 0; k < NP; k += 2)
                *reinterpret_cast<float4*>(dp + 2 * k) =
                    make_float4(S.b[r][k].x, S.b[r][k].y, S.b[r][k + 1].x, S.b[r][k + 1].y);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Host side.
template <int CPL, int RS, int NWV, int SRC, bool OUT16>
static void launch_t(hipStream_t s, const JresArgs& A, int grid)
{
    hipLaunchKernelGGL((k_jres<CPL, RS, NWV, SRC, OUT16>), dim3(grid), dim3(64 * NWV), 0, s, A);
}
template <int CPL, int RS, int NWV>
static void launch_cr(hipStream_t s, const JresArgs& A, int grid, int src_mode, bool out16)
{
    if (out16) {
        if (src_mode == 2) launch_t<CPL, RS, NWV, 2, true>(s, A, grid);
        else if (src_mode == 1) launch_t<CPL, RS, NWV, 1, true>(s, A, grid);
        else launch_t<CPL, RS, NWV, 0, true>(s, A, grid);
    } else {
        if (src_mode == 2) launch_t<CPL, RS, NWV, 2, false>(s, A, grid);
        else if (src_mode == 1) launch_t<CPL, RS, NWV, 1, false>(s, A, grid);
        else launch_t<CPL, RS, NWV, 0, false>(s, A, grid);
    }
}

// Workgroup shape: PF_JRES_WAVES waves over a 64-row region -- 16 waves of 4 rows (default: one
// workgroup per CU at <= 128 VGPRs) or 8 waves of 8 rows (two waves per SIMD at <= 256 VGPRs,
// leaving a sixth of the register file to co-resident kernels).  Measured in the pipelined C3
// step on MI355X (profiles/r03 logs; recipe: tools/gpu_round.sh ab, three alternating rounds): 13.64-13.97k panoramas/s for 16
// waves, 13.66-13.76k for 8, 12.89-13.02k for the streaming passes.
#ifndef PF_JRES_WAVES
#define PF_JRES_WAVES 16
#endif
static constexpr int kJW = PF_JRES_WAVES;
int jres_words_per_value() { return PF_JRES_GRANULE ? 2 : 1; }
// hand-off flag words per row block: one per published row (LDS-flag form) or one per block
int jres_flags_per_block(int K) { return PF_JRES_LDSFLAG ? 2 * K : 1; }
static constexpr int kRS512 = 64 / kJW, kRS256 = 128 / kJW;

// 1024-wide levels (round 5, off): 16 columns per lane, 8 waves of 4 rows (a 32-row region; the
// LDS edge rows of 16 waves would need 256 KB, 8 waves need 128 KB: one workgroup per CU, two
// waves per SIMD at 236 VGPRs, no spills).  Measured slower than the streaming passes: C5's one
// call 2.42 ms against 2.16 (its 1024-wide level 0 at batch 1), and C3's batch-64 level 1
// (PF_JRES1024_ANY=1) 14.2k against 16.7k panoramas/s (profiles/r05/jres1024.txt).
#ifndef PF_JRES_1024
#define PF_JRES_1024 0
#endif
static constexpr int kJW1024 = 8, kRS1024 = 4;

// Half-height regions (round 5): the same workgroup with half the rows per wave (512 wide: 2
// rows, a 32-row region).  A sweep then costs each wave half the updates, which is what a
// launch whose blocks are all resident at once waits for (one panorama: C2's level 0 is 200
// sequential sweeps); a full batch wants the taller region (fewer redundant halo rows per core
// row).  jres_plan weighs both.
#ifndef PF_JRES_HALF
#define PF_JRES_HALF 1
#endif

// region rows of the resident kernel's workgroup at this width (0: not supported)
int jres_region_rows(int w, bool half)
{
    if (half) return (PF_JRES_HALF && w == 512) ? 32 : 0;
    if (w == 512) return 64;
    if (w == 256) return 128;
    if (w == 1024 && PF_JRES_1024) return kJW1024 * kRS1024;
    return 0;
}
int jres_threads() { return 64 * kJW; }

void launch_jres(hipStream_t s, const JresArgs& A)
{
    const int grid = A.nb * A.batch;
#if PF_JRES_HALF
    if (A.w == 512 && A.half) launch_cr<8, kRS512 / 2, kJW>(s, A, grid, A.src_mode, A.out != nullptr);
    else
#endif
    if (A.w == 512) launch_cr<8, kRS512, kJW>(s, A, grid, A.src_mode, A.out != nullptr);
    else if (A.w == 256) launch_cr<4, kRS256, kJW>(s, A, grid, A.src_mode, A.out != nullptr);
#if PF_JRES_1024
    else if (A.w == 1024)
        launch_cr<16, kRS1024, kJW1024>(s, A, grid, A.src_mode, A.out != nullptr);
#endif
}

// resident blocks per CU of the instantiation that launches at this width (half: the half-height
// 512-wide region, whose register and LDS use may differ from the full one's)
int jres_blocks_per_cu(int w, bool half)
{
    int nb = 0;
    const void* f = reinterpret_cast<const void*>(k_jres<8, kRS512, kJW, 0, false>);
    int threads = 64 * kJW;
#if PF_JRES_HALF
    if (w == 512 && half) f = reinterpret_cast<const void*>(k_jres<8, kRS512 / 2, kJW, 0, false>);
#else
    (void)half;
#endif
    if (w == 256) f = reinterpret_cast<const void*>(k_jres<4, kRS256, kJW, 0, false>);
#if PF_JRES_1024
    if (w == 1024) {
        f = reinterpret_cast<const void*>(k_jres<16, kRS1024, kJW1024, 0, false>);
        threads = 64 * kJW1024;
    }
#endif
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f, threads, 0) != hipSuccess) nb = 0;
    return nb;
}

}  // namespace pf
