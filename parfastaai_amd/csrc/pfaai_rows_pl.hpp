// pfaai_rows_pl.hpp -- k_rows_pl: the default row kernel (genome-major input).
//
// What it computes is exactly k_rows (pfaai_kernels.hpp): for output row A
// and every protein p in ascending order, the intersection counts
// c(p, A, B) = |{t : A, B both in run (t, p)}| -- the run-lengths of the
// reference's sorted E (ds_helper.hpp:270-357, psort.hpp:27-53) -- and
// S += c / (T[p][A] + T[p][B] - c), N += 1 over c > 0
// (algorithm_impl.hpp:240-275), then AJI = S / N (algorithm_impl.hpp:318).
//
// Per protein, a one-row workgroup walks a chain of dependent loads (G list
// -> run table -> member ids -> LDS atomics -> barrier -> T -> divide).  The
// chain is cut into stages that work on different proteins in the same
// iteration, with ONE workgroup barrier per protein:
//
//   iteration i:  T(i-1)  T16 words of protein i-1 (for S5)
//                 S4a(i)  issue the member-id loads of protein i's line tasks
//                 S3(i+1) cut protein i+1's runs into 16-member line tasks
//                         (wave scan + one LDS atomic per wave, no barrier)
//                 S2(i+2) issue the run-table lookups of protein i+2
//                 S1(i+3) issue the G-list load of protein i+3
//                 S5(i-1) normalise counter row (i-1)&1 into S, N; clear it
//                 S4b(i)  ds_add_u32 the members into counter row i&1, then
//                         further task rounds (two tasks per 4-lane group in
//                         flight) and whole-workgroup runs
//                 barrier
//
// gfx9 retires vector loads in order (vmcnt), so the loads are issued in
// the order they are consumed: T (S5), members (S4b), then the prefetches --
// waiting for T never waits for the members, waiting for the members never
// waits for the prefetches (T first and two tasks in flight: 12.7 -> 12.0 ms
// at 10k).  |E| is summed from the counter rows in S5 rather than per member.
// A line task is 16 members = 64 B; a 4-lane group takes one task and each
// lane loads 4 members with one 16-B buffer load (a wave instruction covers
// 16 lines), which measured 13 % faster than 16-lane groups of 4-B loads.
// Two counter rows (packed u16 pairs) double-buffer S4 against S5.  Runs too
// long for line tasks, and tasks beyond the LDS capacity, are flagged in a
// per-protein bitmask and walked by the whole workgroup -- slower, never
// wrong.
//
// NT threads per workgroup and WPE waves per SIMD: the default is NT = 1024
// with WPE = 8, i.e. <= 64 VGPRs (no spills in the WK 3 forms) so that two
// workgroups share a CU and one's barrier waits overlap the other's work
// (12.2 ms at 10k vs 15.6 ms at one per CU); NT = 512 is the alternative
// form (twice the counter words per thread).
//
// Preconditions (checked on the host, pfaai_hip.hip): genome-major input,
// every (genome, protein) G list <= kPlEntries entries, ncw <= KW*NT
// counter words per chunk, T < 2^16.
#pragma once
#include <type_traits>

#include "pfaai_util.hpp"

namespace pfaai {

constexpr int kPlEntries = 1024;   // G entries per (genome, protein) (host-checked)
constexpr int kPlTaskCap = 4096;   // u16 line tasks per protein stage: run slot | line << 10
constexpr int kPlMaxLines = 63;    // runs with more lines go to the whole-workgroup walk
constexpr uint16_t kPlNoTask = 0xFFFFu;

// E triple (p, A, b): +1 into the u16 counter of column b.  |E| is counted
// from the counter rows in S5, not here (one VALU op less per member).
template <int MODE>
__device__ __forceinline__ void pl_add(const Dev& d, int32_t a, int32_t b, uint32_t* acc, int32_t cc0, int32_t wlo,
                                       int32_t whi) {
    if ((uint32_t)(b - wlo) >= (uint32_t)(whi - wlo)) return;  // also drops b = -1 (no member)
    if (MODE == 1 && !(b != a && (!d.is_q[b] || b > a))) return;  // isValidPair, ds_impl.hpp:270-273
    if (MODE == kModeFull && b == a) return;
    const uint32_t o = (uint32_t)(b - cc0);
    atomicAdd(&acc[o >> 1], 1u << ((o & 1u) << 4));
}

// Member loads of line task k of this lane's 4-lane group: 4 members (16 B)
// of the task's 64-B line, issued unconditionally (an out-of-range offset
// where the lane has none).  Bit j of the result: member j of b is valid.
// BIGF (|F| >= 2^30, where a 32-bit byte offset into F wraps -- buffer
// offsets, strided index included, are 32-bit on gfx9): a 64-bit global load
// instead; a lane without members re-reads F[0..3] (its ok bits are clear).
template <int TC = kPlTaskCap, bool BIGF = false>
__device__ __forceinline__ uint32_t pl_issue(rsrc_t fg, const int32_t* __restrict__ Fg, const uint16_t* tk,
                                             const uint2* rt, int k, int nt, int gl, uint4& b) {
    const uint32_t t = tk[min(k, TC - 1)];
    const uint2 rr = rt[t & 1023u];
    const uint32_t m0 = (rr.x & ~(uint32_t)(kGroup - 1)) + (t >> 10) * kGroup + 4u * (uint32_t)gl;
    const bool task = k < nt && t != kPlNoTask;
    uint32_t ok = 0u;
#pragma unroll
    for (int j = 0; j < 4; ++j) ok |= (uint32_t)(task && m0 + j >= rr.x && m0 + j < rr.y) << j;
    if constexpr (BIGF)
        b = *reinterpret_cast<const uint4*>(Fg + (ok ? m0 : 0u));
    else
        b = bld_u128(fg, ok ? m0 * 4u : kOOB, 0u);
    return ok;
}

template <int MODE>
__device__ __forceinline__ void pl_scatter4(const Dev& d, int32_t a, uint4 b, uint32_t ok, uint32_t* acc, int32_t cc0,
                                            int32_t wlo, int32_t whi) {
    pl_add<MODE>(d, a, (ok & 1u) ? (int32_t)b.x : -1, acc, cc0, wlo, whi);
    pl_add<MODE>(d, a, (ok & 2u) ? (int32_t)b.y : -1, acc, cc0, wlo, whi);
    pl_add<MODE>(d, a, (ok & 4u) ? (int32_t)b.z : -1, acc, cc0, wlo, whi);
    pl_add<MODE>(d, a, (ok & 8u) ? (int32_t)b.w : -1, acc, cc0, wlo, whi);
}

// The same three steps with fewer VALU operations (the kernel is VALU-bound:
// ~85 % of a SIMD's issue cycles at 10k, rocprofv3 SQ_INSTS_VALU):
//  * pl_issue_m: the task's valid members form the contiguous range
//    [lo, hi) of the lane's 4 (run bounds minus the lane's first member
//    index), so the 4-bit mask is one bit-field (v_med3 clamps + v_bfm)
//    instead of eight compares;
//  * pl_add_m: chunks start at even columns, so counter word (b - cc0) / 2
//    is accb[b >> 1] with accb = acc - cc0 / 2, and the member's mask bit
//    joins the window test in one predicate.
template <int TC = kPlTaskCap, bool BIGF = false>
__device__ __forceinline__ uint32_t pl_issue_m(rsrc_t fg, const int32_t* __restrict__ Fg, const uint16_t* tk,
                                               const uint2* rt, int k, int nt, uint32_t gl4, uint4& b) {
    const uint32_t t = tk[min(k, TC - 1)];
    const uint2 rr = rt[t & 1023u];
    const uint32_t m0 = (rr.x & ~(uint32_t)(kGroup - 1)) + ((t >> 6) & ~15u) + gl4;  // + (t >> 10) * 16
    const int32_t l0 = min(max((int32_t)(rr.x - m0), 0), 4);
    const int32_t h0 = min(max((int32_t)(rr.y - m0), l0), 4);
    uint32_t mask = ((1u << (uint32_t)(h0 - l0)) - 1u) << (uint32_t)l0;
    if (!(k < nt && t != kPlNoTask)) mask = 0u;
    if constexpr (BIGF)
        b = *reinterpret_cast<const uint4*>(Fg + (mask ? m0 : 0u));
    else
        b = bld_u128(fg, mask ? m0 * 4u : kOOB, 0u);
    return mask;
}

// WK: the window test a member needs -- 0: wlo <= b < whi; 1: wlo <= b (the
// window reaches the last id, e.g. an all-vs-all row in one chunk); 2: none
// (the window is every id, e.g. a full row); 3: none (the members after A in
// a run, all-vs-all with G_pos, see pl_issue_m2).
template <int MODE, int WK>
__device__ __forceinline__ void pl_add_m(const Dev& d, int32_t a, int32_t b, bool valid, uint32_t* accb, int32_t wlo,
                                         uint32_t wspan) {
    bool ok = valid;
    if constexpr (WK == 0) ok = ok && (uint32_t)(b - wlo) < wspan;
    if constexpr (WK == 1) ok = ok && b >= wlo;
    if (MODE == 1) ok = ok && b != a && (!d.is_q[b] || b > a);  // isValidPair, ds_impl.hpp:270-273
    if (MODE == kModeFull) ok = ok && b != a;
    if (ok) {
        // counter word b >> 1: a v_lshrrev the compiler cannot fold back into
        // (b << 1) & ~3, so the address is one v_lshl_add (4 VALU per member
        // instead of 5)
        uint32_t wi;
        asm("v_lshrrev_b32 %0, 1, %1" : "=v"(wi) : "v"(b));
        atomicAdd(&accb[wi], 1u << (((uint32_t)b & 1u) << 4));
    }
}

// Branch-free WK 3 member adds (VAR bit 256, A/B): an invalid slot adds 0
// to a lane-private word of the counter row (acc[lane], no bank conflict, no
// change) instead of an exec-masked branch per slot (3 SALU + a branch).
__device__ __forceinline__ void pl_add_bf(uint32_t b, bool valid, uint32_t* accb, uint32_t lane_wi) {
    uint32_t wi;
    asm("v_lshrrev_b32 %0, 1, %1" : "=v"(wi) : "v"(b));
    const uint32_t inc = valid ? 1u << ((b & 1u) << 4) : 0u;
    __hip_atomic_fetch_add(&accb[valid ? wi : lane_wi], inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void pl_scatter4_bf(uint4 b, uint32_t m, uint32_t* accb, uint32_t lane_wi) {
    pl_add_bf(b.x, m & 1u, accb, lane_wi);
    pl_add_bf(b.y, m & 2u, accb, lane_wi);
    pl_add_bf(b.z, m & 4u, accb, lane_wi);
    pl_add_bf(b.w, m & 8u, accb, lane_wi);
}

template <int MODE, int WK>
__device__ __forceinline__ void pl_scatter4_m(const Dev& d, int32_t a, uint4 b, uint32_t m, uint32_t* accb,
                                              int32_t wlo, uint32_t wspan) {
    pl_add_m<MODE, WK>(d, a, (int32_t)b.x, m & 1u, accb, wlo, wspan);
    pl_add_m<MODE, WK>(d, a, (int32_t)b.y, m & 2u, accb, wlo, wspan);
    pl_add_m<MODE, WK>(d, a, (int32_t)b.z, m & 4u, accb, wlo, wspan);
    pl_add_m<MODE, WK>(d, a, (int32_t)b.w, m & 8u, accb, wlo, wspan);
}

// Two-lane groups (the k_rows_pl default): a lane takes half a line task, 8
// members by two 16-B loads, so a protein's tasks fill half as many wave
// rounds and the per-task issue work is shared by 8 members instead of 4.
// A8 (WK 3, all-vs-all rows in one chunk, G_pos loaded): a run's members
// after the row genome A are exactly its partners b > A (runs are sorted by
// genome), so the tasks are 16-member spans of [G_pos + 1, run end) from an
// 8-aligned start, and the members need no window test -- instead of the
// run's 16-aligned lines pruned only at line granularity by the splitters
// (SYN 10k: 50 % of the loaded member slots were events).  8-member tasks,
// one per lane, overflow the 2048-entry task list for low rows (up to 4 200
// per protein at 10k: 13.3 ms vs 9.8).
template <int TC = kPlTaskCap, bool BIGF = false, bool A8 = false>
__device__ __forceinline__ uint32_t pl_issue_m2(rsrc_t fg, const int32_t* __restrict__ Fg, const uint16_t* tk,
                                                const uint2* rt, int k, int nt, uint32_t gl8, uint4& b, uint4& bh) {
    const uint32_t t = tk[min(k, TC - 1)];
    const uint2 rr = rt[t & 1023u];
    const uint32_t m0 = (rr.x & ~(uint32_t)(A8 ? 7 : kGroup - 1)) + ((t >> 6) & ~15u) + gl8;
    const int32_t l0 = min(max((int32_t)(rr.x - m0), 0), 8);
    const int32_t h0 = min(max((int32_t)(rr.y - m0), l0), 8);
    uint32_t mask = ((1u << (uint32_t)(h0 - l0)) - 1u) << (uint32_t)l0;
    if (!(k < nt && t != kPlNoTask)) mask = 0u;
    if constexpr (BIGF) {
        b = *reinterpret_cast<const uint4*>(Fg + ((mask & 15u) ? m0 : 0u));
        bh = *reinterpret_cast<const uint4*>(Fg + ((mask >> 4) ? m0 + 4u : 0u));
    } else {
        b = bld_u128(fg, (mask & 15u) ? m0 * 4u : kOOB, 0u);
        bh = bld_u128(fg, (mask >> 4) ? m0 * 4u + 16u : kOOB, 0u);
    }
    return mask;
}

// CLK (diagnostics, PFAAI_PL_CLK): every wave of the first kClkBlocks
// workgroups sums the shader-clock time of each stage of the protein loop
// into clk[(block * (NT / 64) + wave) * 8 + stage] (pfaai_debug_clocks,
// tools/gpu/stage_clocks.py).
constexpr int kClkBlocks = 256;

// NK: where the per-column counts N live.  0: u16 pairs in registers (KW
// VGPRs, any P); 1: u8 pairs in LDS (P <= 255; no VGPRs, half the task
// capacity, an LDS read-modify-write per word in S5); 2: u8 quads in
// registers (P <= 255; ceil(KW / 2) VGPRs, two VALU ops per word:
// N += pk_min(counter word, 1) shifted into place).
// S5F: S5 (normalise protein i-1) runs FIRST in iteration i, on T words
// loaded during iteration i-1.  At KW = 5 the 64-VGPR budget spills a few fp64
// accumulators; their reloads in S5 are scratch loads, and gfx9 waits for
// vector loads in order, so an S5 after the prefetches waited for the
// members and run-table entries just issued (s_waitcnt vmcnt(0)) -- first, it
// waits only for loads of the previous iteration, needed by now anyway.
// LA (lookahead, WK 3 with N in LDS only): the first round of a protein's
// member loads is issued at the end of the PREVIOUS iteration and stays in
// flight across the barrier, S5 and S3 -- the per-protein chain no longer
// waits for member lines once per protein.  Its tasks must then be cut two
// proteins ahead (S3(i+2), S2(i+3), S1(i+4)), so the task / run slots are
// three (q % 3) and the task counter sets four (q % 4).  It needs the 9
// VGPRs of the loads in flight across the barrier: the narrow launches (KW
// <= 2) have them within the 64-VGPR budget.
template <int MODE, int KW, int NT, int WPE = 4, bool CLK = false, int NK = 0, bool BIGF = false,
          bool S5F = true, bool BR = false, int VAR = 0, int WK = 0, bool LA = false>
__global__ __launch_bounds__(NT, WPE) void k_rows_pl(Dev d, int64_t row_begin, int32_t chunk_cols, int32_t abs_chunk,
                                                   uint32_t flags,
                                                   const unsigned long long* __restrict__ first_key,
                                                   double* __restrict__ aji, double* __restrict__ s_out,
                                                   int32_t* __restrict__ n_out,
                                                   unsigned long long* __restrict__ n_events,
                                                   unsigned long long* __restrict__ clk = nullptr) {
    constexpr int W = KW * NT;            // counter words per row chunk
    constexpr int EPT = kPlEntries / NT;  // G entries per thread
    constexpr int NG = NT / 4;            // 4-lane groups
    constexpr bool NL = NK == 1;
    constexpr int NN = NK == 0 ? KW : NK == 2 ? (KW + 1) / 2 : 1;  // N registers
    constexpr int TC = NL ? kPlTaskCap / 2 : kPlTaskCap;  // line tasks per stage
    static_assert(!LA || (WK == 3 && NK == 1 && S5F), "the lookahead form is WK 3 with N in LDS");
    constexpr int NSL = LA ? 3 : 2;                      // task / run slots (protein % NSL)
    constexpr int NCS = LA ? 4 : 3;                      // task counter sets (protein % NCS)
    extern __shared__ uint32_t pl_smem[];                // acc[2][W], goff[P + 1], (NL) n16[W]
    __shared__ uint2 rt[NSL][kPlEntries];                // runs of a protein stage: member range [lo, hi)
    __shared__ uint16_t tk[NSL][TC];                     // line tasks
    __shared__ uint32_t wmask[NCS][kPlEntries / 32];     // whole-workgroup runs, by protein % NCS
    __shared__ uint32_t ntask[NCS], nwhole[NCS];         // by protein % NCS

    const int tid = threadIdx.x, lane = tid & 63;
    const int grp = tid >> 2, gl = tid & 3;
    const int64_t rl = xcd_row(blockIdx.x, gridDim.x, d.xcd_chunk);
    const int32_t a = d.row_genome[row_begin + rl];
    int32_t clo, chi;
    row_cols<MODE>(d, a, clo, chi);
    // chunks start at even columns so a counter word / T word holds columns (2w, 2w+1);
    // abs_chunk >= 0: one absolute column window [abs_chunk * chunk_cols, +chunk_cols),
    // the one the run table was built for (k_blk<true>)
    const int32_t cc0 = abs_chunk >= 0 ? abs_chunk * chunk_cols : (clo & ~1) + (int32_t)blockIdx.y * chunk_cols;
    const int32_t wlo = max(cc0, clo), whi = min(chi, cc0 + chunk_cols);
    if (wlo >= whi) return;  // uniform
    const int32_t ncw = (whi - cc0 + 1) >> 1;
    const bool compat = flags & 1u;
    const uint32_t min_len = abs_chunk >= 0 ? 0u : 1u;  // window sub-runs: one member may be a partner
    const uint32_t prio = (flags >> 16) & 3u;
    const int P = d.n_prot;
    uint32_t* acc = pl_smem;
    uint32_t* goff = pl_smem + 2 * W;
    // NL: N of the thread's columns as u8 in LDS: NPK (default) u32
    // n32[tid + (k >> 1) * NT] holds word tid + k * NT's two columns, k even
    // in bytes (0, 2), k odd in bytes (1, 3), so S5 updates it by one packed
    // min (+ a shift) and a no-return LDS atomic at a constant offset instead
    // of a read, 7 VALU ops and a write (10.13 -> 9.77 ms at 10k); VAR bit
    // 1024 keeps the first form, u16 n16[w] = the u8 pair of word w (A/B)
    constexpr bool NPK = NL && (VAR & 1024) == 0;
    constexpr int NWORDS = !NL ? 0 : NPK ? (KW + 1) / 2 * NT : W / 2;
    uint16_t* n16 = reinterpret_cast<uint16_t*>(pl_smem + 2 * W + P + 1);
    uint32_t* n32 = pl_smem + 2 * W + P + 1;
    uint16_t* taL = reinterpret_cast<uint16_t*>(pl_smem + 2 * W + P + 1 + NWORDS);  // T[p][A], p < P

    const int64_t g0 = d.G_off[(int64_t)a * P];
    for (int p = tid; p <= P; p += NT) goff[p] = (uint32_t)(d.G_off[(int64_t)a * P + p] - g0);
    for (int w = tid; w < 2 * W; w += NT) acc[w] = 0u;
    if (NL)
        for (int w = tid; w < NWORDS; w += NT) n32[w] = 0u;
    if (tid < NCS) { ntask[tid] = 0u; nwhole[tid] = 0u; }
    for (int w = tid; w < NCS * (kPlEntries / 32); w += NT) (&wmask[0][0])[w] = 0u;
    const int32_t tca = compat ? d.tcol_row[a] : a;  // T column of genomeA (row Q quirk only in compat)
    for (int p = tid; p < P; p += NT) taL[p] = (uint16_t)d.T[(int64_t)p * d.t_cols + tca];
    const uint16_t* T16 = compat ? d.T16c : d.T16;
    const int64_t t16w = d.t16_cols >> 1;            // u32 words per protein row of T16
    double S[2 * KW];
    uint32_t N[NN];  // NK 0: u16 pair of word k in N[k]; NK 2: word k's pair at bits 8(k&1) + {0, 16} of N[k/2]
#pragma unroll
    for (int k = 0; k < KW; ++k) { S[2 * k] = 0.0; S[2 * k + 1] = 0.0; }
#pragma unroll
    for (int k = 0; k < NN; ++k) N[k] = 0u;
    uint32_t ev = 0;
    __syncthreads();

    // Fg carries 16 padding entries and the range covers them: a 16-B load
    // that crosses num_records reads all zeros, not just its tail
    const rsrc_t r_fg = mk_rsrc(d.Fg, (uint64_t)(d.n_f + 16) * 4u);
    const rsrc_t r_g = mk_rsrc(d.G_tet + g0, (uint64_t)uni_u32(goff[P]) * 4u);
    // the run table: 16-B entries (k_blk), or u32 run ends under WK 3 (k_blk_end)
    const rsrc_t r_blk = mk_rsrc(d.blk, (uint64_t)P * kNTetramers * 16u);  // < 4 GiB: P <= 1600 (host-checked); unused by WK 3
    const rsrc_t r_t16 = mk_rsrc(T16, (uint64_t)P * d.t16_cols * 2u);
    const rsrc_t r_t = mk_rsrc(d.T, (uint64_t)P * d.t_cols * 4u);
    // S1 / S2 return the raw loads: nothing may touch a prefetched value
    // before its consumer, or the compiler waits for it on the spot.
    auto glen = [&](int p) -> uint32_t { return p < P ? uni_u32(goff[p + 1]) - uni_u32(goff[p]) : 0u; };
    // a wave none of whose entries tid + j*NT is below the list length n has
    // nothing to do in S1-S3 for that protein (the typical list holds ~290 of
    // the 1024 entries: 11 of 16 waves are idle), so it skips them -- a
    // wave-uniform branch (10.17 -> 9.96 ms at 10k; VAR bit 64 restores the
    // unconditional form for A/B)
    constexpr bool kSkip = (VAR & 64) == 0;
    const uint32_t wbase0 = uni_u32((uint32_t)tid & ~63u);
    // WK 3: S1 loads each entry's G_pos and G_end (the end of its F run,
    // built at load) -- two coalesced loads, no tetramer id and no run-table
    // lookup; S2 only carries them on (gq -> gq2, gt -> r4.y); S3 cuts
    // [G_pos + 1, G_end) into 16-member tasks from an 8-aligned start
    // (pl_issue_m2<A8>)
    constexpr bool GP = WK == 3;
    const rsrc_t r_gp = mk_rsrc(GP ? d.G_pos + g0 : nullptr, GP ? (uint64_t)uni_u32(goff[P]) * 4u : 0u);
    const rsrc_t r_ge = mk_rsrc(GP ? d.G_end + g0 : nullptr, GP ? (uint64_t)uni_u32(goff[P]) * 4u : 0u);
    // WK 3: S1's loads are issued by every wave (out-of-range offsets read
    // 0): a load issued under the wave skip made the number of loads in
    // flight path-dependent, and the compiler then waited for everything
    // (vmcnt(0)) wherever an older load was consumed -- the member loads in
    // S4b waited for this iteration's G_pos / G_end loads (VAR bit 128 keeps
    // the skip, A/B)
    constexpr bool kSkipS1 = kSkip && !(GP && (VAR & 128) == 0);
    auto s1 = [&](int p, int32_t (&gt)[EPT], uint32_t (&gq)[EPT]) {  // G entries tid + j*NT of protein p (tetramer ids)
        const uint32_t o = p < P ? uni_u32(goff[p]) : 0u, n = glen(p);
        if constexpr (kSkipS1) {
            if (wbase0 >= n) return;
        }
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
            const uint32_t e = (uint32_t)(tid + j * NT);
            if constexpr (GP) {
                gq[j] = bld_u32(r_gp, e < n ? e * 4u : kOOB, o * 4u);
                gt[j] = (int32_t)bld_u32(r_ge, e < n ? e * 4u : kOOB, o * 4u);  // run end (0 past the list)
            } else {
                gt[j] = (int32_t)bld_u32(r_g, e < n ? e * 4u : kOOB, o * 4u);
            }
        }
    };
    auto s2 = [&](int p, const int32_t (&gt)[EPT], uint4 (&r4)[EPT], const uint32_t (&gq)[EPT], uint32_t (&gq2)[EPT]) {
        // run-table entries ({0..} past the list)
        const uint32_t n = glen(p);
        if constexpr (kSkip) {
            if (wbase0 >= n) return;
        }
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
            const uint32_t e = (uint32_t)(tid + j * NT);
            if constexpr (GP) {
                (void)e;
                gq2[j] = gq[j];
                r4[j].y = (uint32_t)gt[j];  // G_end (S1)
            } else {
                r4[j] = bld_u128(r_blk, e < n ? (uint32_t)gt[j] * 16u : kOOB,
                                 (uint32_t)min(p, P - 1) * (kNTetramers * 16u));
            }
        }
    };
    auto s3 = [&](int q, const uint4 (&r4)[EPT], const uint32_t (&gq2)[EPT]) {  // line tasks of protein q
        const int st = q % NSL, cs = q % NCS;
        if constexpr (kSkip) {
            if (wbase0 >= glen(q)) return;
        }
        uint32_t nl[EPT], v = 0;
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
            const int e = tid + j * NT;
            uint2 r;
            if constexpr (GP) {
                r = make_uint2(gq2[j] + 1u, r4[j].y);  // OOB entries: (1, 0), empty
                nl[j] = r.y > r.x ? (r.y - (r.x & ~7u) + 15u) >> 4 : 0u;
            } else {
                nl[j] = run_lines(r4[j], wlo, whi, r, min_len, !(MODE == 2 && abs_chunk >= 0));
            }
            rt[st][e] = r;
            if (nl[j] > (uint32_t)kPlMaxLines) {
                atomicOr(&wmask[cs][e >> 5], 1u << (e & 31));
                atomicAdd(&nwhole[cs], 1u);
                nl[j] = 0u;
            }
            v += nl[j];
        }
        // one LDS atomic per wave reserves the wave's tasks
        const uint32_t inc = wave_scan_dpp(v);
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        uint32_t base = 0;
        if (tot) {
            if (lane == 63) base = atomicAdd(&ntask[cs], tot);
            base = (uint32_t)__builtin_amdgcn_readlane((int)base, 63);
        }
        uint32_t e0 = base + inc - v;
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
            const uint32_t slot = (uint32_t)(tid + j * NT), n = nl[j];
            if (e0 + n <= (uint32_t)TC) {
#pragma unroll
                for (uint32_t l = 0; l < 4; ++l)
                    if (l < n) tk[st][e0 + l] = (uint16_t)(slot | (l << 10));
#pragma unroll 1
                for (uint32_t l = 4; l < n; ++l) tk[st][e0 + l] = (uint16_t)(slot | (l << 10));
            } else if (n) {  // over capacity: the whole workgroup walks this run
#pragma unroll 1
                for (uint32_t l = e0; l < (uint32_t)TC; ++l) tk[st][l] = kPlNoTask;
                atomicOr(&wmask[cs][slot >> 5], 1u << (slot & 31));
                atomicAdd(&nwhole[cs], 1u);
            }
            e0 += n;
        }
    };

    // prologue: tasks of protein 0; run-table entries of protein 1; G lists of protein 2
    // (LA: tasks of proteins 0 and 1, entries of 2, lists of 3)
    int32_t gt[EPT];
    uint4 r4[EPT];
    uint32_t gq[EPT], gq2[EPT];
#pragma unroll
    for (int j = 0; j < EPT; ++j) { r4[j] = make_uint4(0u, 0u, 0u, 0u); gq[j] = gq2[j] = 0u; }
    s1(0, gt, gq);
    s2(0, gt, r4, gq, gq2);
    s1(1, gt, gq);
    s3(0, r4, gq2);
    s2(1, gt, r4, gq, gq2);
    s1(2, gt, gq);
    if constexpr (LA) {
        if (1 < P) s3(1, r4, gq2);
        s2(2, gt, r4, gq, gq2);
        s1(3, gt, gq);
    }
    __syncthreads();

    unsigned long long ck[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long tprev = CLK ? clock64() : 0;
    auto stamp = [&](int j) {
        if constexpr (CLK) {
            const unsigned long long t = clock64();
            ck[j] += t - tprev;
            tprev = t;
        }
    };
    // S5 of protein i-1 on counter row (i-1)&1 with its T words (fp64,
    // ascending protein order per pair)
    // d >= c always holds with the true T columns; only QT under REF_COMPAT
    // (row Q: other genomes' T columns) can give d < c, d <= 0 -- that case
    // keeps per-column branches and the IEEE fallback.  Otherwise S5 is
    // branch-free per word: a zero counter divides 0 by max(d, 1) and adds an
    // exact +0.0 (S >= +0), N adds pk_min(word, 1); only waves with no column
    // in the chunk skip a word (a scalar branch, no exec-mask juggling).
    auto n_add = [&](int k, uint32_t v, int32_t w) {
        if constexpr (NK == 0) {
            N[k] += min(v & 0xFFFFu, 1u) | (min(v >> 16, 1u) << 16);
        } else if constexpr (NK == 2) {
            N[k >> 1] += (min(v & 0xFFFFu, 1u) | (min(v >> 16, 1u) << 16)) << (8 * (k & 1));
        } else {
            if constexpr (NPK) {
                const uint32_t x = pk_min1_u16(v);  // (min(c0, 1), min(c1, 1)) at bits 0, 16
                atomicAdd(&n32[tid + (k >> 1) * NT], (k & 1) ? x << 8 : x);
            } else if constexpr ((VAR & 4) != 0)  // first form (A/B)
                n16[w] = (uint16_t)(n16[w] + (uint32_t)((v & 0xFFFFu) != 0u) + ((uint32_t)((v >> 16) != 0u) << 8));
            else
                n16[w] = (uint16_t)(n16[w] + min(v & 0xFFFFu, 1u) + (min(v >> 16, 1u) << 8));
        }
    };
    auto s5 = [&](int i, const uint32_t (&tw)[KW], int32_t ta) {
        if (!(i >= 1 && glen(i - 1) > 0u)) return;
        uint32_t* acc_p = acc + ((i - 1) & 1) * W;
        const int32_t wbase = (int32_t)uni_u32((uint32_t)tid & ~63u);
        if (BR || (MODE == 2 && compat)) {  // BR: per-column branches everywhere (A/B)
            auto div = [&](int32_t c, int32_t dd) -> double {
                if constexpr ((VAR & 1) != 0) return (double)(c + dd);  // diagnostics: no division (wrong results)
                if (MODE == 2 && compat) return exact_div_any((double)c, (double)dd);
                return exact_div_small((double)c, (double)dd);
            };
#pragma unroll
            for (int k = 0; k < KW; ++k) {
                const int32_t w = tid + k * NT;
                // words past the row's last column stay 0: a wave whose words
                // are all past it stops (WK 3 only, where row widths vary
                // within a launch; in the other forms it costs 6 spilled VGPRs
                // -- 100k streamed 613 -> 689 ms; VAR bit 512: no skip, A/B);
                // read and clear by one ds_wrxchg_rtn_b32: no faster
                if (WK == 3 && (VAR & 512) == 0 && wbase + k * NT >= ncw) break;
                const uint32_t v = acc_p[w];
                if (v) {
                    acc_p[w] = 0u;
                    const int32_t c0 = (int32_t)(v & 0xFFFFu), c1 = (int32_t)(v >> 16);
                    ev += (uint32_t)(c0 + c1);
                    n_add(k, v, w);
                    const int32_t d0 = ta + (int32_t)(tw[k] & 0xFFFFu) - c0, d1 = ta + (int32_t)(tw[k] >> 16) - c1;
                    if (c0) S[2 * k] += div(c0, d0);
                    if (c1) S[2 * k + 1] += div(c1, d1);
                }
            }
            return;
        }
#pragma unroll
        for (int k = 0; k < KW; ++k) {
            if (wbase + k * NT >= ncw) break;  // wave-uniform: later words are further out
            const int32_t w = tid + k * NT;
            const uint32_t v = acc_p[w];
            acc_p[w] = 0u;
            const int32_t c0 = (int32_t)(v & 0xFFFFu), c1 = (int32_t)(v >> 16);
            ev += (uint32_t)(c0 + c1);
            n_add(k, v, w);
            const int32_t d0 = max(ta + (int32_t)(tw[k] & 0xFFFFu) - c0, 1);
            const int32_t d1 = max(ta + (int32_t)(tw[k] >> 16) - c1, 1);
            S[2 * k] += exact_div_small((double)c0, (double)d0);
            S[2 * k + 1] += exact_div_small((double)c1, (double)d1);
        }
    };
    uint32_t twc[KW];  // S5F: T words of the previous protein, carried across the barrier
#pragma unroll
    for (int k = 0; k < KW; ++k) twc[k] = 0u;
    int32_t tac = 0;
    // TL (default; VAR bit 32 restores the first form for A/B): the T words
    // are loaded after S4b instead of before S4a, so they are live across the
    // barrier only, not across the member rounds, and T[p][A] comes from an
    // LDS table filled once per row -- one spilled fp64 accumulator instead of
    // two, 10.37 -> 10.10 ms at 10k
    constexpr bool TL = S5F && (VAR & 32) == 0;
    // member path: two-lane groups (pl_issue_m2), 8 members per lane and task
    // (10.60 -> 10.47 ms, VALU instructions -5.8 % at 10k); VAR bit 8 keeps the
    // four-lane groups with two tasks in flight, VAR bit 2 the first form
    // (pl_issue / pl_scatter4), for A/B
    constexpr bool kLegacyM = (VAR & 2) != 0 && !GP;
    constexpr bool G2 = ((VAR & 8) == 0 && !kLegacyM) || GP;
    constexpr int NGX = G2 ? NT / 2 : NG;
    const int grpx = G2 ? tid >> 1 : grp;
    const uint32_t gl8 = 8u * (uint32_t)(tid & 1);
    const uint32_t gl4 = 4u * (uint32_t)gl, wspan = (uint32_t)(whi - wlo);
    int st_cur = 0;
    auto issue = [&](int k, int ntk, uint4& bb) -> uint32_t {
        if constexpr (kLegacyM) return pl_issue<TC, BIGF>(r_fg, d.Fg, tk[st_cur], rt[st_cur], k, ntk, gl, bb);
        return pl_issue_m<TC, BIGF>(r_fg, d.Fg, tk[st_cur], rt[st_cur], k, ntk, gl4, bb);
    };
    // WK: the window test of pl_add_m, chosen by the launcher for every row
    // of the launch (pfaai_launch.hpp)
    auto scatter = [&](uint32_t* acc_x, uint4 bb, uint32_t m) {
        if constexpr (kLegacyM) pl_scatter4<MODE>(d, a, bb, m, acc_x, cc0, wlo, whi);
        else pl_scatter4_m<MODE, WK>(d, a, bb, m, acc_x - (cc0 >> 1), wlo, wspan);
    };
    auto issue2 = [&](int k, int ntk, uint4& bb, uint4& bbh) -> uint32_t {
        return pl_issue_m2<TC, BIGF, GP>(r_fg, d.Fg, tk[st_cur], rt[st_cur], k, ntk, gl8, bb, bbh);
    };
    auto scatter8 = [&](uint32_t* acc_x, uint4 bb, uint4 bbh, uint32_t m) {
        if constexpr (WK == 3 && MODE == 0 && (VAR & 256) != 0) {
            const uint32_t lane_wi = (uint32_t)(cc0 >> 1) + (uint32_t)lane;  // accb[lane_wi] = acc_x[lane]
            pl_scatter4_bf(bb, m & 15u, acc_x - (cc0 >> 1), lane_wi);
            pl_scatter4_bf(bbh, m >> 4, acc_x - (cc0 >> 1), lane_wi);
        } else {
            pl_scatter4_m<MODE, WK>(d, a, bb, m & 15u, acc_x - (cc0 >> 1), wlo, wspan);
            pl_scatter4_m<MODE, WK>(d, a, bbh, m >> 4, acc_x - (cc0 >> 1), wlo, wspan);
        }
    };

    if constexpr (LA) {
        // first round of protein 0's member loads, in flight into iteration 0
        uint4 b, bh;
        st_cur = 0;
        uint32_t okm = issue2(grpx, glen(0) > 0u ? min((int)uni_u32(ntask[0]), TC) : 0, b, bh);
#pragma unroll 1
        for (int i = 0; i <= P; ++i) {
            uint32_t* acc_i = acc + (i & 1) * W;
            const bool has_i = i < P && glen(i) > 0u;
            s5(i, twc, i >= 1 ? (int32_t)uni_u32(taL[i - 1]) : 0);
            stamp(0);
            if (i + 2 < P) s3(i + 2, r4, gq2);
            stamp(1);
            s2(i + 3, gt, r4, gq, gq2);
            s1(i + 4, gt, gq);
            stamp(2);
            if (has_i) {
                const int cs = i % NCS;
                const int nt = min((int)uni_u32(ntask[cs]), TC);
                scatter8(acc_i, b, bh, okm);  // the first round, loaded during the previous iteration
                stamp(4);
                st_cur = i % NSL;
                for (int k = grpx + NGX; k < nt; k += NGX) {
                    okm = issue2(k, nt, b, bh);
                    scatter8(acc_i, b, bh, okm);
                }
                if (uni_u32(nwhole[cs])) {  // e.g. a tetramer shared by every genome
                    for (int wd = 0; wd < kPlEntries / 32; ++wd) {
                        uint32_t m = uni_u32(wmask[cs][wd]);
                        while (m) {
                            const int sb = __builtin_ctz(m);
                            m &= m - 1u;
                            const uint32_t rx = uni_u32(rt[st_cur][wd * 32 + sb].x), ry = uni_u32(rt[st_cur][wd * 32 + sb].y);
                            for (uint32_t mm = rx + tid; mm < ry; mm += NT)
                                pl_add<MODE>(d, a, d.Fg[mm], acc_i, cc0, wlo, whi);
                        }
                    }
                }
            }
            stamp(5);
            // T words of protein i for the next S5 (issued before the member
            // loads below: S5 waits for them, not for the members)
            {
                const int pt = min(i, P - 1);
                const uint32_t tso = (uint32_t)((int64_t)pt * t16w + (cc0 >> 1)) * 4u;
#pragma unroll
                for (int k = 0; k < KW; ++k) twc[k] = bld_u32(r_t16, (uint32_t)tid * 4u, tso + (uint32_t)k * (NT * 4u));
            }
            // the first round of protein i + 1 (its tasks were cut in iteration i - 1)
            {
                const int q = i + 1;
                const int ntq = (q < P && glen(q) > 0u) ? min((int)uni_u32(ntask[q % NCS]), TC) : 0;
                st_cur = q % NSL;
                okm = issue2(grpx, ntq, b, bh);
            }
            stamp(3);
            // recycle the counter set of protein i + 3 (last read in iteration i - 1)
            if (tid < kPlEntries / 32) wmask[(i + 3) % NCS][tid] = 0u;
            if (tid == 32) { ntask[(i + 3) % NCS] = 0u; nwhole[(i + 3) % NCS] = 0u; }
            __syncthreads();
            stamp(6);
        }
    } else {
#pragma unroll 1
    for (int i = 0; i <= P; ++i) {
        const int st = i & 1, cs = i % 3;
        st_cur = st;
        uint32_t* acc_i = acc + st * W;
        const bool has_i = i < P && glen(i) > 0u;
        if constexpr (S5F) {
            s5(i, twc, TL ? (i >= 1 ? (int32_t)uni_u32(taL[i - 1]) : 0) : tac);
            stamp(7);
        }
        // T words of the thread's columns and T[p][A] (S5F: of protein i, for
        // the next iteration; else of protein i-1, issued first so that S5
        // waits for nothing issued after them)
        const int pt = S5F ? min(i, P - 1) : (i >= 1 ? i - 1 : 0);
        if (prio & 1u) __builtin_amdgcn_s_setprio(2);  // loads issue ahead of other waves' S5 (flags bits 16-17)
        uint32_t tw[KW];
        int32_t ta = 0;
        const uint32_t tso = (uint32_t)((int64_t)pt * t16w + (cc0 >> 1)) * 4u;
        const uint32_t tao = (uint32_t)((int64_t)pt * d.t_cols + tca) * 4u;
        if constexpr (!TL) {
#pragma unroll
            for (int k = 0; k < KW; ++k) tw[k] = bld_u32(r_t16, (uint32_t)tid * 4u, tso + (uint32_t)k * (NT * 4u));
            ta = (int32_t)bld_u32(r_t, 0u, tao);
        }
        // S4a: first round of member loads of protein i (one task per 4-lane group)
        const int nt = has_i ? min((int)uni_u32(ntask[cs]), TC) : 0;
        uint4 b, bh;
        uint32_t okm = G2 ? issue2(grpx, nt, b, bh) : issue(grp, nt, b);
        stamp(0);
        // S3(i+1), then the prefetches S2(i+2), S1(i+3)
        if (i + 1 < P) s3(i + 1, r4, gq2);
        stamp(1);
        s2(i + 2, gt, r4, gq, gq2);
        s1(i + 3, gt, gq);
        stamp(2);
        if (prio) __builtin_amdgcn_s_setprio(0);
        // S5: normalise protein i-1
        if constexpr (!S5F) {
            s5(i, tw, ta);
        } else if constexpr (!TL) {
#pragma unroll
            for (int k = 0; k < KW; ++k) twc[k] = tw[k];
            tac = (int32_t)uni_u32((uint32_t)ta);  // uniform: an SGPR across the barrier
        }
        stamp(3);
        if (prio & 2u) __builtin_amdgcn_s_setprio(1);
        // S4b: atomics of the first round, further rounds (two tasks per
        // group in flight), whole-workgroup runs
        if (has_i) {
            if constexpr (G2) {
                scatter8(acc_i, b, bh, okm);
                stamp(4);
                for (int k = grpx + NGX; k < nt; k += NGX) {
                    okm = issue2(k, nt, b, bh);
                    scatter8(acc_i, b, bh, okm);
                }
            } else {
                scatter(acc_i, b, okm);
                stamp(4);
                int k = grp + NG;
                for (; k + NG < nt; k += 2 * NG) {
                    uint4 b2;
                    okm = issue(k, nt, b);
                    const uint32_t ok2 = issue(k + NG, nt, b2);
                    scatter(acc_i, b, okm);
                    scatter(acc_i, b2, ok2);
                }
                if (k < nt) {
                    okm = issue(k, nt, b);
                    scatter(acc_i, b, okm);
                }
            }
            if (uni_u32(nwhole[cs])) {  // e.g. a tetramer shared by every genome
                for (int wd = 0; wd < kPlEntries / 32; ++wd) {
                    uint32_t m = uni_u32(wmask[cs][wd]);
                    while (m) {
                        const int s = __builtin_ctz(m);
                        m &= m - 1u;
                        const uint32_t rx = uni_u32(rt[st][wd * 32 + s].x), ry = uni_u32(rt[st][wd * 32 + s].y);
                        for (uint32_t mm = rx + tid; mm < ry; mm += NT)
                            pl_add<MODE>(d, a, d.Fg[mm], acc_i, cc0, wlo, whi);
                    }
                }
            }
        }
        if constexpr (TL) {  // T words of protein i for the next S5, live only across the barrier
#pragma unroll
            for (int k = 0; k < KW; ++k) twc[k] = bld_u32(r_t16, (uint32_t)tid * 4u, tso + (uint32_t)k * (NT * 4u));
        }
        stamp(5);
        // recycle the protein-(i+2) counter set (last read by S4(i-1))
        if (tid < kPlEntries / 32) wmask[(i + 2) % 3][tid] = 0u;
        if (tid == 32) { ntask[(i + 2) % 3] = 0u; nwhole[(i + 2) % 3] = 0u; }
        __syncthreads();
        stamp(6);
    }
    }  // !LA
    if constexpr (CLK) {
        if (lane == 0 && blockIdx.x < kClkBlocks && blockIdx.y == 0)
            for (int j = 0; j < 8; ++j) clk[((int64_t)blockIdx.x * (NT / 64) + (tid >> 6)) * 8 + j] = ck[j];
    }

    // |E| of this row chunk (the sum of its counters over all proteins)
    ev = wave_sum_u32(ev);
    if (lane == 0 && ev) atomicAdd(n_events, (unsigned long long)ev);

    // epilogue: JAC S/N and AJI at the reference's JAC index
#pragma unroll
    for (int k = 0; k < KW; ++k) {
        const int32_t w = tid + k * NT;
        if (w >= ncw) continue;
        double sv[2];
        int32_t nv[2];
        bool ok[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int32_t b = cc0 + 2 * w + h;
            ok[h] = b >= wlo && b < whi && col_valid<MODE>(d, a, b);
            double s = S[2 * k + h];
            int32_t n = NPK ? (int32_t)((n32[tid + (k >> 1) * NT] >> (8 * (k & 1) + 16 * h)) & 0xFFu)
                        : NK == 1 ? (int32_t)((n16[w] >> (8 * h)) & 0xFFu)
                        : NK == 2 ? (int32_t)((N[(k >> 1) % NN] >> (8 * (k & 1) + 16 * h)) & 0xFFu)
                                  : (int32_t)((N[k % NN] >> (16 * h)) & 0xFFFFu);
            if (ok[h] && n == 0 && compat) {
                // extents stay 0/0 -> J of E[0]'s protein, N = 1
                const unsigned long long key = *first_key;
                const int32_t p0 = key == ~0ull ? 0 : (int32_t)(key & ((1ull << 21) - 1));
                const int32_t* Tp = d.T + (int64_t)p0 * d.t_cols;
                s = 0.0 + 1.0 / (double)(Tp[tca] + Tp[d.tcol_col[b]] - 1);
                n = 1;
            }
            sv[h] = s;
            nv[h] = n;
        }
        put_pair<MODE>(d, a, cc0 + 2 * w, ok, sv, nv, compat, aji, s_out, n_out);
    }
}

}  // namespace pfaai
