// pfaai_rows_pl.hpp -- k_rows_pl: the software-pipelined genome-major row
// kernel (the default K-S+J of the fused path).
//
// What it computes is exactly k_rows (pfaai_kernels.hpp): for output row A
// and every protein p in ascending order, the intersection counts
// c(p, A, B) = |{t : A, B both in run (t, p)}| -- the run-lengths of the
// reference's sorted E (ds_helper.hpp:270-357, psort.hpp:27-53) -- and
// S += c / (T[p][A] + T[p][B] - c), N += 1 over c > 0
// (algorithm_impl.hpp:240-275), then AJI = S / N (algorithm_impl.hpp:318).
//
// Why a new kernel: per protein, k_rows walks a chain of dependent global
// loads (G list -> run table -> member ids -> LDS atomics -> barrier -> T ->
// divide) and nothing else is in flight meanwhile; measured on MI355X it is
// latency-serialised, not bandwidth- or LDS-bound.  Here the chain is cut
// into five stages that run for five different proteins in the same
// iteration, with ONE workgroup barrier per protein:
//
//   iteration i:  S1(i+3) load the row genome's G list for protein i+3
//                 S2(i+2) load the run-table entries of protein i+2's list
//                 S3(i+1) cut protein i+1's runs into 16-member line tasks
//                         (wave scan + one LDS atomic per wave, no barrier)
//                 S4(i)   member-id loads + ds_add_u32 into counter row i&1
//                 S5(i-1) normalise counter row (i-1)&1 into S, N; clear it
//                 barrier
//
// Member-id loads of S4 are issued first, the prefetches of S1/S2 and the
// T words of protein i after them (gfx9 vmcnt retires loads in order, so
// waiting for the member ids never waits for a prefetch), and S3 + S5 run
// while the member ids are in flight.  Two counter rows (u16 pairs) double
// buffer S4 against S5.  Runs too long for line tasks, and tasks beyond the
// LDS task capacity, are flagged in a per-protein bitmask and walked by the
// whole workgroup in S4 -- slower, never wrong.
//
// Preconditions (checked on the host, pfaai_hip.hip pick_rows_kernel):
// genome-major input, every (genome, protein) G list <= 1024 entries,
// ncw <= KW*1024 counter words per chunk.
#pragma once
#include <type_traits>

#include "pfaai_counts.hpp"  // buffer-load helpers

namespace pfaai {

constexpr int kPlTaskCap = 4096;   // u16 line tasks per protein stage
constexpr int kPlMaxLines = 63;    // runs with more lines go to the whole-workgroup walk
constexpr uint16_t kPlNoTask = 0xFFFFu;
#ifndef PFAAI_PL_WAVES
#define PFAAI_PL_WAVES 4  // waves per SIMD: one 1024-thread workgroup per CU (~85 VGPRs)
#endif

// Inclusive wave64 prefix sum with DPP row shifts and row broadcasts (no LDS).
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

// 16-B blk entry -> member range [lo, hi) and line count after pruning to
// the column window [wlo, whi) with the run's line splitters (k_blk).
__device__ __forceinline__ uint32_t pl_prune(uint4 r4, int32_t wlo, int32_t whi, uint2& r) {
    r = make_uint2(r4.x, r4.y);
    if (r.y - r.x <= 1u) return 0u;  // a run of one member is A alone: no partner
    const uint32_t first = r.x & ~(uint32_t)(kGroup - 1);
    uint32_t nl = (r.y - first + kGroup - 1) / kGroup;
    if (nl > 1u) {
        const uint64_t sp = (uint64_t)r4.z | ((uint64_t)r4.w << 32);
        uint32_t l0 = 0, l1 = nl;
#pragma unroll
        for (uint32_t i = 1; i <= (uint32_t)kSplitters; ++i) {
            const int32_t f = (int32_t)((sp >> (kSplitBits * (i - 1))) & kSplitNone);
            if (i < nl) {
                if (f <= wlo) l0 = i;               // lines < i hold ids < f <= wlo
                if (f >= whi && l1 > i) l1 = i;     // lines >= i hold ids >= f >= whi
            }
        }
        if (l1 <= l0) return 0u;
        if (l0) r.x = first + l0 * kGroup;
        if (l1 < nl) r.y = first + l1 * kGroup;
        nl = l1 - l0;
    }
    return nl;
}

template <int MODE>
__device__ __forceinline__ void pl_scatter(const Dev& d, int32_t a, int32_t b, uint32_t* acc, int32_t cc0,
                                           int32_t wlo, int32_t whi, uint32_t& ev, uint32_t flags = 0u) {
    if (b < wlo || b >= whi) return;  // also drops b = -1 (no member)
    if (MODE == 1 && !(b != a && (!d.is_q[b] || b > a))) return;  // isValidPair, ds_impl.hpp:270-273
    const uint32_t o = (uint32_t)(b - cc0);
    if (!(flags & 0x200u)) atomicAdd(&acc[o >> 1], 1u << ((o & 1u) << 4));  // 0x200: diagnostics, no atomics
    ++ev;
}

// Branch-free E triple: every lane issues its ds_add_u32; a lane without a
// valid member adds 0 to a counter word of its own (lane-private address, so
// no same-address serialisation).  Exec-mask branches cost more than the
// LDS op they would skip (SQ_INSTS_SALU/BRANCH dominated the branchy form).
template <int MODE>
__device__ __forceinline__ void bf_scatter(const Dev& d, int32_t a, int32_t b, bool ok, uint32_t* acc, int32_t cc0,
                                           int32_t wlo, int32_t whi, uint32_t& ev) {
    ok = ok && b >= wlo && b < whi;
    if (MODE == 1) ok = ok && b != a && (!d.is_q[ok ? b : a] || b > a);  // isValidPair, ds_impl.hpp:270-273
    const uint32_t o = ok ? (uint32_t)(b - cc0) : (uint32_t)(threadIdx.x & 63) << 1;
    atomicAdd(&acc[o >> 1], (uint32_t)ok << ((o & 1u) << 4));
    ev += ok;
}

// c / d for integers 1 <= c <= d < 2^24, bit-identical to IEEE division:
// the same reciprocal, Newton steps and final residual correction that the
// compiler expands '/' into (v_rcp_f64, 2 x fma refinement, mul, fma
// residual, fma correction), minus v_div_scale / v_div_fmas / v_div_fixup,
// which are the identity for operands this far from the exponent limits
// (no scaling needed, no inf/nan/zero/denormal cases).  Exhaustively
// checked against '/' on the GPU (tests/test_gpu_div.py).
__device__ __forceinline__ double exact_div_small(double c, double dd) {
    double y = __builtin_amdgcn_rcp(dd);
    double e = __builtin_fma(-dd, y, 1.0);
    y = __builtin_fma(y, e, y);
    e = __builtin_fma(-dd, y, 1.0);
    y = __builtin_fma(y, e, y);
    const double q = c * y;
    const double r = __builtin_fma(-dd, q, c);
    return __builtin_fma(r, y, q);
}

// Member loads of the line tasks k0 + u*64 (u < U) of this lane's
// 16-lane group: task ids and run ranges are read from LDS in batches of 4
// (all reads of a batch in flight together), then every lane issues its
// loads unconditionally (an out-of-range offset where it has no member, so
// no exec-mask branches).  Bit u of the returned mask: b[u] is a member.
template <int U>
__device__ __forceinline__ uint32_t pl_issue(rsrc_t fg, const uint16_t* tk, const uint2* rt, int k0, int rem,
                                             int gl, int32_t* b) {
    uint32_t ok_mask = 0u;
#pragma unroll
    for (int h = 0; h < U; h += 4) {
        uint32_t t[4];
        uint2 rr[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) t[j] = tk[min(k0 + (h + j) * kNumGroups, kPlTaskCap - 1)];
#pragma unroll
        for (int j = 0; j < 4; ++j) rr[j] = rt[t[j] & 1023u];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t m = (rr[j].x & ~(uint32_t)(kGroup - 1)) + (t[j] >> 10) * kGroup + (uint32_t)gl;
            const bool ok = (h + j) * kNumGroups < rem && t[j] != kPlNoTask && m >= rr[j].x && m < rr[j].y;
            ok_mask |= (uint32_t)ok << (h + j);
            b[h + j] = (int32_t)bld_u32(fg, ok ? m * 4u : 0xFFFFFFF0u, 0u);
        }
    }
    return ok_mask;
}

// 4-lane-group form: a lane loads 4 consecutive members (16 B) of its
// group's line task k0 + u*256, so one wave instruction covers 16 lines.
// Bits 4u..4u+3 of the returned mask: b[u].{x,y,z,w} are members.
template <int U>
__device__ __forceinline__ uint32_t pl_issue4(rsrc_t fg, const uint16_t* tk, const uint2* rt, int k0, int rem,
                                              int gl4, uint4* b) {
    constexpr int NG = kRowThreads / 4;
    uint32_t ok_mask = 0u;
    uint32_t t[U];
    uint2 rr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) t[u] = tk[min(k0 + u * NG, kPlTaskCap - 1)];
#pragma unroll
    for (int u = 0; u < U; ++u) rr[u] = rt[t[u] & 1023u];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t m0 = (rr[u].x & ~(uint32_t)(kGroup - 1)) + (t[u] >> 10) * kGroup + 4u * (uint32_t)gl4;
        const bool task = u * NG < rem && t[u] != kPlNoTask;
        uint32_t ok4 = 0u;
#pragma unroll
        for (int j = 0; j < 4; ++j) ok4 |= (uint32_t)(task && m0 + j >= rr[u].x && m0 + j < rr[u].y) << j;
        ok_mask |= ok4 << (4 * u);
        b[u] = bld_u128(fg, ok4 ? m0 * 4u : 0xFFFFFFF0u, 0u);
    }
    return ok_mask;
}

// Diagnostics (flags 0x1000): per-stage clock accumulation, written by wave
// 0 of each workgroup into s_out as 8 doubles per workgroup.
#define PL_TICK(slot)                                   \
    if (prof) {                                         \
        const uint64_t t_ = clock64();             \
        tacc[slot] += t_ - tlast;                       \
        tlast = t_;                                     \
    }

template <int MODE, int KW, int U, int GL = kGroup, bool DEEP = false, bool BAL = false, bool BF = false>
__global__ __launch_bounds__(kRowThreads, PFAAI_PL_WAVES) void k_rows_pl(
    Dev d, int64_t row_begin, int32_t chunk_cols, uint32_t flags, const unsigned long long* __restrict__ first_key,
    double* __restrict__ aji, double* __restrict__ s_out, int32_t* __restrict__ n_out,
    unsigned long long* __restrict__ n_events) {
    constexpr int W = KW * kRowThreads;        // counter words per row
    extern __shared__ uint32_t pl_smem[];      // acc[2][W], goff[P + 1]
    __shared__ uint2 rt[2][kRowThreads];       // runs of a protein stage: member range [lo, hi)
    __shared__ uint16_t tk[2][kPlTaskCap];     // line tasks: run slot | line << 10
    __shared__ uint32_t wmask[3][kRowThreads / 32];  // whole-workgroup runs, by protein % 3
    __shared__ uint32_t ntask[3], nwhole[3];   // by protein % 3

    const int tid = threadIdx.x, lane = tid & 63;
    const int grp = tid / GL, gl = tid % GL;
    constexpr int NG = kRowThreads / GL;  // lane groups
    const int64_t rl = xcd_row(blockIdx.x, gridDim.x);
    const int32_t a = d.row_genome[row_begin + rl];
    int32_t clo, chi;
    row_cols<MODE>(d, a, clo, chi);
    // chunks start at even columns so a counter word / T word holds columns (2w, 2w+1)
    const int32_t cc0 = (clo & ~1) + (int32_t)blockIdx.y * chunk_cols;
    const int32_t wlo = max(cc0, clo), whi = min(chi, cc0 + chunk_cols);
    if (wlo >= whi) return;  // uniform
    const int32_t ncw = (whi - cc0 + 1) >> 1;
    const bool compat = flags & 1u;
    const int P = d.n_prot;
    uint32_t* acc = pl_smem;
    uint32_t* goff = pl_smem + 2 * W;

    const int64_t g0 = d.G_off[(int64_t)a * P];
    for (int p = tid; p <= P; p += kRowThreads) goff[p] = (uint32_t)(d.G_off[(int64_t)a * P + p] - g0);
    for (int w = tid; w < 2 * W; w += kRowThreads) acc[w] = 0u;
    if (tid < 3) { ntask[tid] = 0u; nwhole[tid] = 0u; }
    if (tid < 3 * (kRowThreads / 32)) (&wmask[0][0])[tid] = 0u;
    const int32_t tca = compat ? d.tcol_row[a] : a;  // T column of genomeA (row Q quirk only in compat)
    const uint16_t* T16 = compat ? d.T16c : d.T16;
    const int64_t t16w = d.t16_cols >> 1;            // u32 words per protein row of T16
    double S[2 * KW];
    uint32_t N[KW];
#pragma unroll
    for (int k = 0; k < KW; ++k) { S[2 * k] = 0.0; S[2 * k + 1] = 0.0; N[k] = 0u; }
    uint32_t ev = 0;
    const bool prof = flags & 0x1000u;
    uint64_t tacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t tlast = prof ? clock64() : 0;
    __syncthreads();

    const rsrc_t r_fg = mk_rsrc(d.Fg, (uint64_t)d.n_f * 4u);
    // LDS-sourced values that are uniform go through readfirstlane so buffer
    // resources and scalar offsets stay in SGPRs (no waterfall loops)
    auto uni = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); };
    const rsrc_t r_g = mk_rsrc(d.G_tet + g0, (uint64_t)uni(goff[P]) * 4u);
    const rsrc_t r_blk = mk_rsrc(d.blk, (uint64_t)P * kNTetramers * 16u);
    const rsrc_t r_t16 = mk_rsrc(T16, (uint64_t)P * d.t16_cols * 2u);
    // S1: G list entry tid of protein p (a tetramer id; meaningful for tid < n(p))
    // S2: run-table entry of that tetramer in protein p ({0,0,..} past the list)
    // Both return the raw load: nothing may touch a prefetched value before
    // its consumer, or the compiler waits for it on the spot.
    auto glen = [&](int p) -> uint32_t { return p < P ? uni(goff[p + 1]) - uni(goff[p]) : 0u; };
    // BAL: G entry e of a protein goes to wave e % 16, lane e / 16, so every
    // wave cuts about 1/16 of the runs (instead of the first few waves all)
    const uint32_t ent = BAL ? (uint32_t)((tid & 63) * (kRowThreads / 64) + (tid >> 6)) : (uint32_t)tid;
    auto s1 = [&](int p) -> int32_t {
        const uint32_t o = p < P ? uni(goff[p]) : 0u;
        return (int32_t)bld_u32(r_g, ent < glen(p) ? ent * 4u : 0xFFFFFFF0u, o * 4u);
    };
    auto s2 = [&](int p, int32_t t) -> uint4 {
        const bool ok = ent < glen(p);
        return bld_u128(r_blk, ok ? (uint32_t)t * 16u : 0xFFFFFFF0u, (uint32_t)min(p, P - 1) * (kNTetramers * 16u));
    };
    // S3: line tasks of protein q from this thread's run (slot tid)
    auto s3 = [&](int q, uint4 r4) {
        const int st = q & 1, cs = q % 3;
        uint2 r;
        const uint32_t nl = pl_prune(r4, wlo, whi, r);
        rt[st][ent] = r;
        bool whole = nl > (uint32_t)kPlMaxLines;
        const uint32_t v = whole ? 0u : nl;
        const uint32_t inc = wave_incl_scan_dpp(v);
        const uint32_t tot = (uint32_t)__shfl((int)inc, 63, 64);
        uint32_t base = 0;
        if (tot) {  // wave-uniform
            if (lane == 63) base = atomicAdd(&ntask[cs], tot);
            base = (uint32_t)__shfl((int)base, 63, 64);
        }
        if (v) {
            const uint32_t e0 = base + inc - v;
            if (base + inc <= (uint32_t)kPlTaskCap) {
                if constexpr (BAL) {
#pragma unroll
                    for (uint32_t j = 0; j < 4; ++j)
                        if (j < v) tk[st][e0 + j] = (uint16_t)(ent | (j << 10));
#pragma unroll 1
                    for (uint32_t j = 4; j < v; ++j) tk[st][e0 + j] = (uint16_t)(ent | (j << 10));
                } else {
#pragma unroll 1
                    for (uint32_t j = 0; j < v; ++j) tk[st][e0 + j] = (uint16_t)(ent | (j << 10));
                }
            } else {  // over capacity: the whole workgroup walks this run
                for (uint32_t j = e0; j < (uint32_t)kPlTaskCap; ++j) tk[st][j] = kPlNoTask;
                whole = true;
            }
        }
        const unsigned long long wb = __ballot(whole);
        if (wb) {
            if (whole) atomicOr(&wmask[cs][ent >> 5], 1u << (ent & 31));
            if (lane == 0) atomicAdd(&nwhole[cs], (uint32_t)__popcll(wb));
        }
    };

    // prologue: runs of protein 0 cut into tasks; blk of protein 1; G of protein 2
    // DEEP: G lists loaded 2 iterations before their run-table lookups, the
    // run-table entries 2 iterations before their tasks are cut, T words one
    // iteration before their normalisation (register rings).
    {
        int32_t gt, gtB = -1;
        uint4 r4, r4B = make_uint4(0u, 0u, 0u, 0u);
        uint32_t twp[KW];  // DEEP: T words of protein i-1
        int32_t tap = 0;
#pragma unroll
        for (int k = 0; k < KW; ++k) twp[k] = 0u;
        if constexpr (DEEP) {
            const int32_t g0_ = s1(0), g1_ = s1(1), g2_ = s1(2);
            const uint4 r0_ = s2(0, g0_);
            r4 = s2(1, g1_);   // protein i+1 on loop entry
            r4B = s2(2, g2_);  // protein i+2
            gt = s1(3);        // protein i+3
            gtB = s1(4);       // protein i+4
            s3(0, r0_);
        } else {
            gt = s1(0);
            r4 = s2(0, gt);
            gt = s1(1);
            s3(0, r4);
            r4 = s2(1, gt);   // protein i+1 on loop entry
            gt = s1(2);       // protein i+2 on loop entry
        }
        __syncthreads();

#pragma unroll 1
        for (int i = 0; i <= P; ++i) {
            const int st = i & 1, cs = i % 3;
            uint32_t* acc_i = acc + st * W;
            const bool has_i = i < P && uni(goff[i + 1]) > uni(goff[i]);
            const bool has_p = i >= 1 && uni(goff[i]) > uni(goff[i - 1]);
            // T words of protein i-1 (normalised below, after the member loads are in flight)
            uint32_t tw[KW];
            const int pt = DEEP ? min(i, P - 1) : (i >= 1 ? i - 1 : 0);  // DEEP: protein i, used next iteration
            const uint32_t tso = (uint32_t)((int64_t)pt * t16w + (cc0 >> 1)) * 4u;
#pragma unroll
            for (int k = 0; k < KW; ++k)
                tw[k] = bld_u32(r_t16, (uint32_t)tid * 4u, tso + (uint32_t)k * (kRowThreads * 4u));
            const int32_t ta = d.T[(int64_t)pt * d.t_cols + tca];
            PL_TICK(0)
            // S4 (issue): first round of member loads of protein i
            const int nt = (has_i && !(flags & 0x400u)) ? min((int)uni(ntask[cs]), kPlTaskCap) : 0;  // 0x400: diagnostics, no member loads
            using BT = typename std::conditional<GL == 4, uint4, int32_t>::type;
            BT b[U];
            uint32_t okm;
            if constexpr (GL == 4) okm = pl_issue4<U>(r_fg, tk[st], rt[st], grp, nt - grp, gl, b);
            else okm = pl_issue<U>(r_fg, tk[st], rt[st], grp, nt - grp, gl, b);
            PL_TICK(1)
            // prefetches S2, S1 (after the member loads: vmcnt retires in order)
            const uint4 r4n = DEEP ? s2(i + 3, gt) : s2(i + 2, gt);
            const int32_t gtn = DEEP ? s1(i + 5) : s1(i + 3);
            PL_TICK(2)
            // S5: normalise protein i-1
            if (has_p && (flags & 0x100u)) {  // diagnostics: clear only
                uint32_t* acc_p = acc + (st ^ 1) * W;
#pragma unroll
                for (int k = 0; k < KW; ++k) {
                    const int32_t w = tid + k * kRowThreads;
                    if (w < ncw) acc_p[w] = 0u;
                }
            } else if (has_p && BF) {
                uint32_t* acc_p = acc + (st ^ 1) * W;
                const int32_t tap_ = DEEP ? tap : ta;
#pragma unroll
                for (int k = 0; k < KW; ++k) {
                    if (k * kRowThreads + (tid & ~63) < ncw) {  // wave-uniform: the wave's words exist
                        const int32_t w = tid + k * kRowThreads;
                        const uint32_t v = acc_p[w];
                        acc_p[w] = 0u;
                        const uint32_t t2 = DEEP ? twp[k] : tw[k];
                        const int32_t c0 = (int32_t)(v & 0xFFFFu), c1 = (int32_t)(v >> 16);
                        const int32_t d0 = max(tap_ + (int32_t)(t2 & 0xFFFFu) - c0, 1);
                        const int32_t d1 = max(tap_ + (int32_t)(t2 >> 16) - c1, 1);
                        // c = 0 adds +0.0: S is unchanged bit for bit
                        S[2 * k] += exact_div_small((double)c0, (double)d0);
                        S[2 * k + 1] += exact_div_small((double)c1, (double)d1);
                        N[k] += (uint32_t)(c0 != 0) + ((uint32_t)(c1 != 0) << 16);
                    }
                }
            } else if (has_p) {
                uint32_t* acc_p = acc + (st ^ 1) * W;
#pragma unroll
                for (int k = 0; k < KW; ++k) {
                    const int32_t w = tid + k * kRowThreads;
                    if (w < ncw) {
                        const uint32_t v = acc_p[w];
                        if (v) {
                            acc_p[w] = 0u;
                            const int32_t c0 = (int32_t)(v & 0xFFFFu), c1 = (int32_t)(v >> 16);
                            if (c0) {
                                S[2 * k] += (double)c0 / (double)((DEEP ? tap : ta) + (int32_t)((DEEP ? twp[k] : tw[k]) & 0xFFFFu) - c0);
                                N[k] += 1u;
                            }
                            if (c1) {
                                S[2 * k + 1] += (double)c1 / (double)((DEEP ? tap : ta) + (int32_t)((DEEP ? twp[k] : tw[k]) >> 16) - c1);
                                N[k] += 1u << 16;
                            }
                        }
                    }
                }
            }
            PL_TICK(3)
            // S4 (complete): atomics, further rounds, whole-workgroup runs
            if (has_i) {
                auto scat = [&]() {
                    if constexpr (GL == 4 && BF) {
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            const uint32_t m = okm >> (4 * u);
                            bf_scatter<MODE>(d, a, (int32_t)b[u].x, m & 1u, acc_i, cc0, wlo, whi, ev);
                            bf_scatter<MODE>(d, a, (int32_t)b[u].y, m & 2u, acc_i, cc0, wlo, whi, ev);
                            bf_scatter<MODE>(d, a, (int32_t)b[u].z, m & 4u, acc_i, cc0, wlo, whi, ev);
                            bf_scatter<MODE>(d, a, (int32_t)b[u].w, m & 8u, acc_i, cc0, wlo, whi, ev);
                        }
                    } else if constexpr (GL == 4) {
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            const uint32_t m = okm >> (4 * u);
                            pl_scatter<MODE>(d, a, (m & 1u) ? (int32_t)b[u].x : -1, acc_i, cc0, wlo, whi, ev, flags);
                            pl_scatter<MODE>(d, a, (m & 2u) ? (int32_t)b[u].y : -1, acc_i, cc0, wlo, whi, ev, flags);
                            pl_scatter<MODE>(d, a, (m & 4u) ? (int32_t)b[u].z : -1, acc_i, cc0, wlo, whi, ev, flags);
                            pl_scatter<MODE>(d, a, (m & 8u) ? (int32_t)b[u].w : -1, acc_i, cc0, wlo, whi, ev, flags);
                        }
                    } else {
#pragma unroll
                        for (int u = 0; u < U; ++u)
                            pl_scatter<MODE>(d, a, (okm >> u) & 1u ? b[u] : -1, acc_i, cc0, wlo, whi, ev, flags);
                    }
                };
                scat();
                for (int k0 = grp + U * NG; k0 < nt; k0 += U * NG) {
                    if constexpr (GL == 4) okm = pl_issue4<U>(r_fg, tk[st], rt[st], k0, nt - k0, gl, b);
                    else okm = pl_issue<U>(r_fg, tk[st], rt[st], k0, nt - k0, gl, b);
                    scat();
                }
                if (uni(nwhole[cs])) {
                    for (int wd = 0; wd < kRowThreads / 32; ++wd) {
                        uint32_t m = uni(wmask[cs][wd]);
                        while (m) {
                            const int s = __builtin_ctz(m);
                            m &= m - 1u;
                            const uint32_t rx = uni(rt[st][wd * 32 + s].x), ry = uni(rt[st][wd * 32 + s].y);
                            for (uint32_t mm = rx + tid; mm < ry; mm += kRowThreads)
                                pl_scatter<MODE>(d, a, (int32_t)bld_u32(r_fg, mm * 4u, 0u), acc_i, cc0, wlo, whi, ev);
                        }
                    }
                }
            }
            PL_TICK(4)
            // S3: tasks of protein i+1 (last: the member ids and T words are dead here)
            if (i + 1 < P && !(flags & 0x800u)) s3(i + 1, r4);  // 0x800: diagnostics, no tasks
            if constexpr (DEEP) {
                r4 = r4B;
                r4B = r4n;
                gt = gtB;
                gtB = gtn;
#pragma unroll
                for (int k = 0; k < KW; ++k) twp[k] = tw[k];
                tap = ta;
            } else {
                r4 = r4n;
                gt = gtn;
            }
            // recycle the protein-(i+2) counter set (last read by S4(i-1))
            if (tid < 32) wmask[(i + 2) % 3][tid] = 0u;
            if (tid == 32) { ntask[(i + 2) % 3] = 0u; nwhole[(i + 2) % 3] = 0u; }
            PL_TICK(5)
            __syncthreads();
            PL_TICK(6)
        }
    }

    if (prof) {
        if (tid == 0) {
            double* o = reinterpret_cast<double*>(s_out) + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 8;
            for (int k = 0; k < 7; ++k) o[k] = (double)tacc[k];
            o[7] = (double)P;
        }
        return;
    }
    // |E| of this row chunk
    ev = wave_sum_u32(ev);
    if (lane == 0 && ev) atomicAdd(n_events, (unsigned long long)ev);

    // epilogue: JAC S/N and AJI at the reference's JAC index
#pragma unroll
    for (int k = 0; k < KW; ++k) {
        const int32_t w = tid + k * kRowThreads;
        if (w >= ncw) continue;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int32_t b = cc0 + 2 * w + h;
            if (b < wlo || b >= whi || !col_valid<MODE>(d, a, b)) continue;
            const int64_t idx = pair_index<MODE>(d, a, b, compat);
            double s = S[2 * k + h];
            int32_t n = (int32_t)((N[k] >> (16 * h)) & 0xFFFFu);
            if (n == 0 && compat) {
                // extents stay 0/0 -> J of E[0]'s protein, N = 1
                const unsigned long long key = *first_key;
                const int32_t p0 = key == ~0ull ? 0 : (int32_t)(key & ((1ull << 21) - 1));
                const int32_t* Tp = d.T + (int64_t)p0 * d.t_cols;
                s = 0.0 + 1.0 / (double)(Tp[tca] + Tp[d.tcol_col[b]] - 1);
                n = 1;
            }
            if (aji) aji[idx] = n ? s / (double)n : 0.0;
            if (s_out) s_out[idx] = s;
            if (n_out) n_out[idx] = n;
        }
    }
}

}  // namespace pfaai
