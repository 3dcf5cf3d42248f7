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
//   iteration i:  S5(i-1) normalise counter row (i-1)&1 into S, N with the T
//                         words loaded in iteration i-1; clear it
//                 S4a(i)  issue the member-id loads of protein i's line tasks
//                 S3(i+1) cut protein i+1's runs into 16-member line tasks
//                         (wave scan + one LDS atomic per wave, no barrier)
//                 S2(i+2) issue the run-table lookups of protein i+2
//                 S1(i+3) issue the G-list load of protein i+3
//                 S4b(i)  ds_add_u32 the members into counter row i&1, then
//                         further task rounds and whole-workgroup runs
//                 T(i)    T16 words of protein i (for the next S5)
//                 barrier
//
// gfx9 retires vector loads in order (vmcnt), so the loads are issued in
// the order they are consumed: members (S4b), then the prefetches, then T --
// waiting for the members never waits for the prefetches.  S5 runs first:
// it waits only for loads of the previous iteration.  |E| is summed from the
// counter rows in S5 rather than per member.  A line task is 16 members =
// 64 B, taken by a pair of lanes, 8 members each by two 16-B buffer loads.
// Two counter rows (packed u16 pairs) double-buffer S4 against S5.  Runs too
// long for line tasks, and tasks beyond the LDS capacity, are flagged in a
// per-protein bitmask and walked by the whole workgroup -- slower, never
// wrong.
//
// NT threads per workgroup and WPE waves per SIMD: the default is NT = 1024
// with WPE = 8, i.e. <= 64 VGPRs so that two workgroups share a CU and one's
// barrier waits overlap the other's work (12.2 ms at 10k vs 15.6 ms at one
// per CU); NT = 512 is the form of the narrow rows (four workgroups per CU).
//
// The rejected forms of earlier rounds (the lookahead member loads, 4-lane
// groups, branch-free member adds, early T loads, S5 last, k_rows_v2) are
// described with their measurements in DESIGN.md §3 and are no longer
// compiled; profiles/r02*-r04* hold their A/B records.
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
// k_rows_pl's scheduling switches in flags (set by pfaai_run from these
// defaults; PFAAI_PL_PRIO / _STAG / _REV override them in the diagnostics build):
// bits 16-17 wave priorities of the load-issue stages / scatter rounds,
// bits 18-20 the S5 entry order, bit 21 the further member rounds from the
// last lane pair down
constexpr int kPlPrio = 3;
constexpr int kPlStag = 2;
constexpr int kPlRev = 0;
// k_rows_pl's column selection (its abs_chunk argument) besides a fixed
// window index >= 0: per-row chunks, the row's diagonal window, or a grid
// of windows over blockIdx.y starting at window kWinGrid0 - abs_chunk
constexpr int32_t kWinRow = -1, kWinDiag = -2, kWinGrid0 = -3;

// E triple (p, A, b): +1 into the u16 counter of column b (the
// whole-workgroup walk of runs too long for line tasks).
template <int MODE>
__device__ __forceinline__ void pl_add(const Dev& d, int32_t a, int32_t b, uint32_t* acc, int32_t cc0, int32_t wlo,
                                       int32_t whi) {
    if ((uint32_t)(b - wlo) >= (uint32_t)(whi - wlo)) return;  // also drops b = -1 (no member)
    if (MODE == 1 && !(b != a && (!d.is_q[b] || b > a))) return;  // isValidPair, ds_impl.hpp:270-273
    if (MODE == kModeFull && b == a) return;
    const uint32_t o = (uint32_t)(b - cc0);
    atomicAdd(&acc[o >> 1], 1u << ((o & 1u) << 4));
}

// One member of a line task (chunks start at even columns, so counter word
// (b - cc0) / 2 is accb[b >> 1] with accb = acc - cc0 / 2).  WK: the window
// test a member needs -- 0: wlo <= b < whi; 1: wlo <= b (the window reaches
// the last id, e.g. an all-vs-all row in one chunk); 2: none (the window is
// every id, e.g. a full row); 3: none (the members after A in a run,
// all-vs-all with G_pos, see pl_issue_m2); 4: none (a column window's
// sub-run that holds only partners: all-vs-all windows past the row's
// first column, query-vs-target windows, whose tables stop at n_tgt).
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

template <int MODE, int WK>
__device__ __forceinline__ void pl_scatter4_m(const Dev& d, int32_t a, uint4 b, uint32_t m, uint32_t* accb,
                                              int32_t wlo, uint32_t wspan) {
    pl_add_m<MODE, WK>(d, a, (int32_t)b.x, m & 1u, accb, wlo, wspan);
    pl_add_m<MODE, WK>(d, a, (int32_t)b.y, m & 2u, accb, wlo, wspan);
    pl_add_m<MODE, WK>(d, a, (int32_t)b.z, m & 4u, accb, wlo, wspan);
    pl_add_m<MODE, WK>(d, a, (int32_t)b.w, m & 8u, accb, wlo, wspan);
}

// Member loads of line task k: a lane takes half of it, 8 members by two
// 16-B loads (issued unconditionally: an out-of-range offset where the lane
// has none).  The task's valid members are the contiguous range [lo, hi) of
// the lane's 8 (run bounds minus the lane's first member index), so the mask
// is one bit field (v_med3 clamps + a shift).  A8 (WK 3, all-vs-all rows in
// one chunk, G_pos loaded): a run's members after the row genome A are
// exactly its partners b > A (runs are sorted by genome), so the tasks are
// 16-member spans of [G_pos + 1, run end) from an 8-aligned start, and the
// members need no window test (SYN 10k: 50 % of the loaded member slots were
// events with the run's 16-aligned lines).  BIGF (|F| >= 2^30, where a 32-bit
// byte offset into F wraps -- buffer offsets, strided index included, are
// 32-bit on gfx9): 64-bit global loads instead; a lane without members
// re-reads F[0..7] (its mask bits are clear).
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

// T24 (WK 4, V bit 32): 24-member tasks from an 8-aligned start, 12 members
// per lane of the pair (gl12 = 12 * (tid & 1)) by three 16-B loads: task l of
// a run starts at member 24 l of its 8-aligned span; the mask has 12 bits.
template <int TC = kPlTaskCap, bool BIGF = false>
__device__ __forceinline__ uint32_t pl_issue_m3(rsrc_t fg, const int32_t* __restrict__ Fg, const uint16_t* tk,
                                                const uint2* rt, int k, int nt, uint32_t gl12, uint4& b, uint4& bh,
                                                uint4& bx) {
    const uint32_t t = tk[min(k, TC - 1)];
    const uint2 rr = rt[t & 1023u];
    const uint32_t m0 = (rr.x & ~7u) + (t >> 10) * 24u + gl12;
    const int32_t l0 = min(max((int32_t)(rr.x - m0), 0), 12);
    const int32_t h0 = min(max((int32_t)(rr.y - m0), l0), 12);
    uint32_t mask = ((1u << (uint32_t)(h0 - l0)) - 1u) << (uint32_t)l0;
    if (!(k < nt && t != kPlNoTask)) mask = 0u;
    if constexpr (BIGF) {
        // one 64-bit address for the three pieces (F[0..11] where the lane has
        // no task; a piece without members re-reads its task's lines, which
        // F's 16 padding entries keep in range)
        const uint4* pb = reinterpret_cast<const uint4*>(Fg + (mask ? m0 : 0u));
        b = pb[0];
        bh = pb[1];
        bx = pb[2];
    } else {
        b = bld_u128(fg, (mask & 15u) ? m0 * 4u : kOOB, 0u);
        bh = bld_u128(fg, (mask & 0xF0u) ? m0 * 4u + 16u : kOOB, 0u);
        bx = bld_u128(fg, (mask >> 8) ? m0 * 4u + 32u : kOOB, 0u);
    }
    return mask;
}

// c0 / d0 and c1 / d1 with one v_rcp_f64 (V bit 8): Y ~ 1 / (d0 d1) (the
// product is exact: d < 2^17), one Newton step, then y0 = d1 Y ~ 1 / d0 and
// y1 = d0 Y ~ 1 / d1 (relative error ~2^-44), and per column q = c y and the
// residual correction -- whose result is then within ~2^-88 of c / d,
// closer than any rounding boundary (>= 2^-54 / d away), i.e. IEEE c / d.
// Checked on the device by pfaai_debug_div_check's pair mode.  Needs d >= 1
// (S5 clamps a zero counter's d to 1).  One v_rcp_f64 (~17 cycles of issue)
// and a Newton step fewer per word for one more multiply.
__device__ __forceinline__ void exact_div_pair(int32_t c0, int32_t d0i, int32_t c1, int32_t d1i, double& s0, double& s1) {
    const double d0 = (double)d0i, d1 = (double)d1i, pd = d0 * d1;
    double y = __builtin_amdgcn_rcp(pd);
    y = __builtin_fma(y, __builtin_fma(-pd, y, 1.0), y);
    const double y0 = d1 * y, a0 = (double)c0 * y0;
    s0 += __builtin_fma(__builtin_fma(-d0, a0, (double)c0), y0, a0);
    const double y1 = d0 * y, a1 = (double)c1 * y1;
    s1 += __builtin_fma(__builtin_fma(-d1, a1, (double)c1), y1, a1);
}

// WK 3 member scatter of a lane's 8 member codes (k_fcode: counter word
// byte offset code >> 5, u16 half increment 1 << code) under the lane's
// mask bits m: per member one v_cmpx sets EXEC to the lanes holding it, three
// VALU ops form the address and the increment, ds_add_u32, and one s_mov
// restores EXEC -- instead of the compiler's v_cmp + s_and_saveexec +
// s_cbranch_execz + s_or_b64 around four VALU ops (2 VALU and 2 SALU fewer
// per member slot).  base = the LDS byte address of counter word 0
// (acc - cc0 / 2).  The atomics are waited for before the barrier
// (s_waitcnt lgkmcnt(0)).  (Two 4-member blocks, so the first waits for the
// first 16-B load only, spill 12-16 VGPRs.)
__device__ __forceinline__ void pl_scatter8_code(uint4 c, uint4 ch, uint32_t m, uint32_t base) {
    uint64_t sv;
    uint32_t t, u;
#define PL_SLOT(BIT, R)                              \
    "v_and_b32 %[t], " #BIT ", %[m]\n\t"              \
    "v_cmpx_ne_u32_e32 vcc, 0, %[t]\n\t"              \
    "v_lshrrev_b32 %[t], 5, %[" R "]\n\t"             \
    "v_add_u32 %[t], %[base], %[t]\n\t"               \
    "v_lshlrev_b32_e64 %[u], %[" R "], 1\n\t"         \
    "ds_add_u32 %[t], %[u]\n\t"                       \
    "s_mov_b64 exec, %[sv]\n\t"
    asm volatile("s_mov_b64 %[sv], exec\n\t" PL_SLOT(1, "c0") PL_SLOT(2, "c1") PL_SLOT(4, "c2") PL_SLOT(8, "c3")
                     PL_SLOT(16, "c4") PL_SLOT(32, "c5") PL_SLOT(64, "c6") PL_SLOT(128, "c7")
                 : [sv] "=&s"(sv), [t] "=&v"(t), [u] "=&v"(u)
                 : [m] "v"(m), [base] "s"(base), [c0] "v"(c.x), [c1] "v"(c.y), [c2] "v"(c.z), [c3] "v"(c.w),
                   [c4] "v"(ch.x), [c5] "v"(ch.y), [c6] "v"(ch.z), [c7] "v"(ch.w)
                 : "vcc", "memory");
#undef PL_SLOT
}

// pl_scatter8_code's slots for a third 16-B piece (T24: members 8-11 of the lane)
__device__ __forceinline__ void pl_scatter4_code(uint4 c, uint32_t m, uint32_t base) {
    uint64_t sv;
    uint32_t t, u;
#define PL_SLOT(BIT, R)                              \
    "v_and_b32 %[t], " #BIT ", %[m]\n\t"              \
    "v_cmpx_ne_u32_e32 vcc, 0, %[t]\n\t"              \
    "v_lshrrev_b32 %[t], 5, %[" R "]\n\t"             \
    "v_add_u32 %[t], %[base], %[t]\n\t"               \
    "v_lshlrev_b32_e64 %[u], %[" R "], 1\n\t"         \
    "ds_add_u32 %[t], %[u]\n\t"                       \
    "s_mov_b64 exec, %[sv]\n\t"
    asm volatile("s_mov_b64 %[sv], exec\n\t" PL_SLOT(1, "c0") PL_SLOT(2, "c1") PL_SLOT(4, "c2") PL_SLOT(8, "c3")
                 : [sv] "=&s"(sv), [t] "=&v"(t), [u] "=&v"(u)
                 : [m] "v"(m), [base] "s"(base), [c0] "v"(c.x), [c1] "v"(c.y), [c2] "v"(c.z), [c3] "v"(c.w)
                 : "vcc", "memory");
#undef PL_SLOT
}

// S5's read of a finished counter word, which also clears it for the protein
// two iterations on: one ds_wrxchg_rtn_b32 (exchange with 0) instead of a
// read and, for a nonzero word, a second LDS store
__device__ __forceinline__ uint32_t pl_take(uint32_t* w) {
    return __hip_atomic_exchange(w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// CLK (diagnostics, PFAAI_PL_CLK): every wave of the first kClkBlocks
// workgroups sums the shader-clock time of each stage of the protein loop
// into clk[(block * (NT / 64) + wave) * 8 + stage] (pfaai_debug_clocks,
// tools/gpu/stage_clocks.py).
constexpr int kClkBlocks = 256;

// NK: where the per-column counts N live.  0: u16 pairs in registers (KW
// VGPRs, any P); 1: u8 pairs in LDS (P <= 255): u32 n32[tid + (k >> 1) * NT]
// holds word tid + k * NT's two columns, k even in bytes (0, 2), k odd in
// bytes (1, 3), updated by one packed min (+ a shift) and a no-return LDS
// atomic.
// S5 divides with exact_div_small (v_rcp_f64, one Newton step, residual
// correction) per nonzero counter.  MODE 2 under REF_COMPAT (the QT T-index
// quirk) can give d < c, d <= 0: it takes per-column
// branches with exact_div_any.  (An LDS table of RN(1/d) -- q = c * r plus
// one residual correction is exact -- measured slower: 5.28 -> 6.13 ms on
// the KW 4 rows of 10k, profiles/r05/ab_s5_rcp_table_kw4.txt; the table reads queue
// behind the member atomics in LDS.)
// V (variant bits): 1 S5 divides both columns of a nonzero counter word (no
// per-column branches: the SALU of six exec-mask updates per word); 2 the
// WK 3 member scatter by pl_scatter8_code over k_fcode's member codes; 8
// S5's two divisions of a word by one reciprocal (exact_div_pair, with 1);
// 16 the G entries one protein ahead instead of two (WK 3, ONE below); 32
// 24-member tasks, 12 members per lane (WK 4, T24 below); 4
// S5 without the max(d, 1) clamp outside WK 3 too (launched only on loads
// whose T is every list's length, t_exact -- WK 3 implies it); 64
// the reference-compat quirks compiled out (MODE 2 launches it only without
// PFAAI_FLAG_REF_COMPAT: its per-column general division then leaves the
// kernel, and V 9 fits 64 VGPRs -- with it, 114 spilled).  The
// WK 3 launches take V = 27 (pfaai_launch.hpp kPlV), the other forms V = 0.
// Measured (tools/gpu/ab_rows.py, 10k all-vs-all, single launches of the
// diagnostics build, profiles/r05/ab_v_*.txt): V 0 -> 3: 8.11-8.24 -> 8.07
// ms; 3 -> 19: 8.16 -> 7.91; 3 -> 27: 8.16 -> 7.84 (the first 894 rows 1.148
// -> 1.099, the 512-thread narrow rows alone 1.087 -> 1.054 at V 0 -> 27);
// V 2 alone on the narrow rows spilled (1.09 -> 1.12 ms) until V 16 freed
// two VGPRs, and so did V 8 without V 16 (a 16-B spill of two accumulators
// per protein).  Rejected: a guard-free member issue (both 16-B loads at the
// task's offsets whatever the mask, the mask by one v_bfi: 8.08 -> 8.30 ms,
// it spilled); the S1-S3 entries on the last waves and the extra member
// rounds on the middle ones (a per-wave balance): 8.11 -> 8.28.
template <int MODE, int KW, int NT, int WPE = 4, bool CLK = false, int NK = 0, bool BIGF = false, int WK = 0,
          int V = 0>
__global__ __launch_bounds__(NT, WPE) void k_rows_pl(Dev d, int64_t row_begin, int32_t chunk_cols, int32_t abs_chunk,
                                                   uint32_t flags,
                                                   const unsigned long long* __restrict__ first_key,
                                                   double* __restrict__ aji, double* __restrict__ s_out,
                                                   int32_t* __restrict__ n_out,
                                                   unsigned long long* __restrict__ n_events,
                                                   unsigned long long* __restrict__ clk = nullptr) {
    constexpr int W = KW * NT;            // counter words per row chunk
    constexpr int EPT = kPlEntries / NT;  // G entries per thread
    constexpr bool NL = NK == 1;
    constexpr int NN = NK == 0 ? KW : 1;  // N registers
    constexpr int TC = NL ? kPlTaskCap / 2 : kPlTaskCap;  // line tasks per stage (half where LDS holds N)
    // T24 (V bit 32, WK 4 with the member codes): 24-member tasks per lane
    // pair (12 members a lane, three 16-B loads) instead of 16.  A protein's
    // window sub-runs at C4 / C5 sizes are mostly one clade's clump of ~18
    // members: 16-member tasks from an 8-aligned start take two tasks for it,
    // and a protein's tasks needed 1.64 rounds of 512 lane pairs on average
    // (C4 shape, 25k targets: the rounds after the first, each with its load
    // latency exposed, were a third of the loop, profiles/r06/
    // stage_clocks_qt25k.txt); 24-member tasks need 1.29 -- yet measured
    // slower (C4 rows 6.62 -> 6.87 ms, C5 531 -> 557 ms: a third load and four
    // scatter slots per lane on every round, one spilled VGPR), so a
    // diagnostics variant only.  (8-member tasks, one per lane, overflowed the
    // task list: C4 rows 6.92 -> 11.05 ms.)
    constexpr bool T24 = (V & 32) != 0 && WK == 4 && (V & 2) != 0;
    constexpr int NGX = NT / 2;                           // task takers per round (lane pairs)
    extern __shared__ uint32_t pl_smem[];                 // acc[2][W], goff[P + 1], (NL) n32, taL
    __shared__ uint2 rt[2][kPlEntries];                   // runs of a protein stage: member range [lo, hi)
    __shared__ uint16_t tk[2][TC];                        // line tasks
    __shared__ uint32_t wmask[3][kPlEntries / 32];        // whole-workgroup runs, by protein % 3
    __shared__ uint32_t ntask[3], nwhole[3];              // by protein % 3

    const int tid = threadIdx.x, lane = tid & 63;
    const int64_t rl = xcd_row(blockIdx.x, gridDim.x, d.xcd_chunk);
    const int32_t a = d.row_genome[row_begin + rl];
    int32_t clo, chi;
    row_cols<MODE>(d, a, clo, chi);
    // chunks start at even columns so a counter word / T word holds columns (2w, 2w+1).
    // abs_chunk (pl_win): >= 0 one absolute column window [abs_chunk * chunk_cols,
    // +chunk_cols), the one the run table was built for (k_blk<true>); kWinRow per-row
    // chunks blockIdx.y; kWinDiag the window holding the row's first column (all-vs-all:
    // the rows' diagonal blocks, none where the row starts a window); <= kWinGrid0 the
    // window (kWinGrid0 - abs_chunk) + blockIdx.y (all-vs-all: off-diagonal only, a row
    // whose columns start past the window's start skips it).  With a window index the
    // window's table is d.blk + w * P * 160000.
    int32_t win = abs_chunk;
    if (abs_chunk == kWinDiag) {
        win = clo / chunk_cols;
        if (MODE == 0 && clo == win * chunk_cols) return;  // uniform: the row starts a window (off-diagonal)
    } else if (abs_chunk <= kWinGrid0) {
        win = (kWinGrid0 - abs_chunk) + (int32_t)blockIdx.y;
        if (MODE == 0 && clo > win * chunk_cols) return;  // uniform: the diagonal launch's (or no) columns
    }
    const int32_t cc0 = win >= 0 ? win * chunk_cols : (clo & ~1) + (int32_t)blockIdx.y * chunk_cols;
    const int32_t wlo = max(cc0, clo), whi = min(chi, cc0 + chunk_cols);
    if (wlo >= whi) return;  // uniform
    const int32_t ncw = (whi - cc0 + 1) >> 1;
    const bool compat = (V & 64) != 0 ? false : (flags & 1u) != 0;  // V 64: launched only without REF_COMPAT
    const uint32_t min_len = win >= 0 ? 0u : 1u;  // window sub-runs: one member may be a partner
    // the scheduling switches of flags bits 16-21 (pfaai_run sets them, kPl*
    // defaults above), read at run time in both builds: compiling the release
    // defaults in measured slower (C3 6.80 -> 6.84 ms, C4 rows 6.58 -> 6.66 ms,
    // profiles/r06/ab_const_flags.txt -- a different code layout of the loop)
    const uint32_t prio = (flags >> 16) & 3u;
    const bool rev = ((flags >> 21) & 1u) != 0;  // S4b's further rounds from the last lane pair
    const uint32_t stag = (flags >> 18) & 7u;   // S5 entry order
    const int P = d.n_prot;
    uint32_t* acc = pl_smem;
    uint32_t* goff = pl_smem + 2 * W;
    constexpr int NWORDS = NL ? (KW + 1) / 2 * NT : 0;
    uint32_t* n32 = pl_smem + 2 * W + P + 1;
    uint16_t* taL = reinterpret_cast<uint16_t*>(pl_smem + 2 * W + P + 1 + NWORDS);  // T[p][A], p < P

    const int64_t g0 = d.G_off[(int64_t)a * P];
    for (int p = tid; p <= P; p += NT) goff[p] = (uint32_t)(d.G_off[(int64_t)a * P + p] - g0);
    for (int w = tid; w < 2 * W; w += NT) acc[w] = 0u;
    if (NL)
        for (int w = tid; w < NWORDS; w += NT) n32[w] = 0u;
    if (tid < 3) { ntask[tid] = 0u; nwhole[tid] = 0u; }
    for (int w = tid; w < 3 * (kPlEntries / 32); w += NT) (&wmask[0][0])[w] = 0u;
    const int32_t tca = compat ? d.tcol_row[a] : a;  // T column of genomeA (row Q quirk only in compat)
    for (int p = tid; p < P; p += NT) taL[p] = (uint16_t)d.T[(int64_t)p * d.t_cols + tca];
    const uint16_t* T16 = compat ? d.T16c : d.T16;
    const int64_t t16w = d.t16_cols >> 1;            // u32 words per protein row of T16
    double S[2 * KW];
    uint32_t N[NN];  // NK 0: u16 pair of word k in N[k]
#pragma unroll
    for (int k = 0; k < KW; ++k) { S[2 * k] = 0.0; S[2 * k + 1] = 0.0; }
#pragma unroll
    for (int k = 0; k < NN; ++k) N[k] = 0u;
    __syncthreads();

    // Fg carries 16 padding entries and the range covers them: a 16-B load
    // that crosses num_records reads all zeros, not just its tail
    const rsrc_t r_fg = mk_rsrc(d.Fg, (uint64_t)(d.n_f + 16) * 4u);
    // member loads read the codes (k_fcode): the WK 3 walks, and the WK 4 window
    // spans (every member a partner: all-vs-all off-diagonal, query vs target)
    constexpr bool CODE = (V & 2) != 0 && ((WK == 3 && MODE == 0) || (WK == 4 && (MODE == 0 || MODE == 2)));
    const rsrc_t r_fm = CODE ? mk_rsrc(d.Fcode, (uint64_t)(d.n_f + 16) * 4u) : r_fg;
    const int32_t* Fm = CODE ? reinterpret_cast<const int32_t*>(d.Fcode) : d.Fg;
    const rsrc_t r_g = mk_rsrc(d.G_tet + g0, (uint64_t)uni_u32(goff[P]) * 4u);
    // the run table: 16-B entries (k_blk; a window's own table under a window
    // grid); unused by WK 3
    const uint4* blk_w = d.blk + (abs_chunk < kWinRow ? (int64_t)win * P * kNTetramers : 0);
    const rsrc_t r_blk = mk_rsrc(blk_w, (uint64_t)P * kNTetramers * 16u);  // < 4 GiB: P <= 1600 (host-checked)
    const rsrc_t r_t16 = mk_rsrc(T16, (uint64_t)P * d.t16_cols * 2u);
    // S1 / S2 return the raw loads: nothing may touch a prefetched value
    // before its consumer, or the compiler waits for it on the spot.
    auto glen = [&](int p) -> uint32_t { return p < P ? uni_u32(goff[p + 1]) - uni_u32(goff[p]) : 0u; };
    // a wave none of whose entries tid + j*NT is below the list length n has
    // nothing to do in S2-S3 for that protein (the typical list holds ~290 of
    // the 1024 entries: 11 of 16 waves are idle), so it skips them -- a
    // wave-uniform branch (10.17 -> 9.96 ms at 10k)
    const uint32_t wbase0 = uni_u32((uint32_t)tid & ~63u);
    // WK 3: S1 loads each entry's (G_pos, G_end) (the end of its F run,
    // built at load; one 8-B load from the interleaved G_pe) -- no tetramer
    // id and no run-table lookup; S3 cuts [G_pos + 1, G_end) into 16-member
    // tasks from an 8-aligned start (pl_issue_m2<A8>)
    constexpr bool GP = WK == 3;
    const rsrc_t r_gpe = mk_rsrc(GP ? d.G_pe + g0 : nullptr, GP ? (uint64_t)uni_u32(goff[P]) * 8u : 0u);
    // WK 3: S1's loads are issued by every wave (out-of-range offsets read
    // 0): a load issued under the wave skip made the number of loads in
    // flight path-dependent, and the compiler then waited for everything
    // (vmcnt(0)) wherever an older load was consumed -- the member loads in
    // S4b waited for this iteration's G_pos / G_end loads
    constexpr bool kSkipS1 = !GP;
    auto s1 = [&](int p, int32_t (&gt)[EPT], uint32_t (&gq)[EPT]) {  // G entries tid + j*NT of protein p (tetramer ids)
        const uint32_t o = p < P ? uni_u32(goff[p]) : 0u, n = glen(p);
        if constexpr (kSkipS1) {
            if (wbase0 >= n) return;
        }
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
            const uint32_t e = (uint32_t)(tid + j * NT);
            if constexpr (GP) {
                const uint2 pe = bld_u64(r_gpe, e < n ? e * 8u : kOOB, o * 8u);  // (0, 0) past the list
                gq[j] = pe.x;
                gt[j] = (int32_t)pe.y;  // run end
            } else {
                gt[j] = (int32_t)bld_u32(r_g, e < n ? e * 4u : kOOB, o * 4u);
            }
        }
    };
    auto s2 = [&](int p, const int32_t (&gt)[EPT], uint4 (&r4)[EPT], const uint32_t (&gq)[EPT], uint32_t (&gq2)[EPT]) {
        // run-table entries ({0..} past the list)
        const uint32_t n = glen(p);
        if (wbase0 >= n) return;
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
            const uint32_t e = (uint32_t)(tid + j * NT);
            if constexpr (GP) {
                (void)e;
                gq2[j] = gq[j];
                r4[j].y = (uint32_t)gt[j];  // G_end (S1)
            } else if constexpr (WK == 4) {  // the window sub-run (lo, hi) only
                const uint2 v = bld_u64(r_blk, e < n ? (uint32_t)gt[j] * 16u : kOOB,
                                        (uint32_t)min(p, P - 1) * (kNTetramers * 16u));
                r4[j] = make_uint4(v.x, v.y, 0u, 0u);
            } else {
                r4[j] = bld_u128(r_blk, e < n ? (uint32_t)gt[j] * 16u : kOOB,
                                 (uint32_t)min(p, P - 1) * (kNTetramers * 16u));
            }
        }
    };
    // ONE (WK 3, V bit 16): the G entries' (G_pos, G_end) are loaded one
    // protein ahead and cut straight from the S1 registers -- S2 is only a
    // register copy under WK 3, and its second stage holds 2 VGPRs across the
    // whole iteration
    constexpr bool ONE = GP && (V & 16) != 0;
    // |E| (the sum of the counters) under WK 3 / 4 is the sum of the walked
    // run lengths -- every member of [r.x, r.y) is one event in the window --
    // so S3 counts it per entry instead of S5 per counter word
    constexpr bool EV3 = WK == 3 || WK == 4;
    uint32_t ev = 0;
    auto s3 = [&](int q, const uint4 (&r4)[EPT], const uint32_t (&gq2)[EPT], const int32_t (&gt1)[EPT]) {  // line tasks of protein q
        const int st = q & 1, cs = q % 3;
        if (wbase0 >= glen(q)) return;
        uint32_t nl[EPT], v = 0;
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
            const int e = tid + j * NT;
            uint2 r;
            if constexpr (GP) {
                r = make_uint2(gq2[j] + 1u, ONE ? (uint32_t)gt1[j] : r4[j].y);  // OOB entries: (1, 0), empty
                nl[j] = r.y > r.x ? (r.y - (r.x & ~7u) + 15u) >> 4 : 0u;
            } else if constexpr (WK == 4) {
                // the window sub-run is exactly A's partners in the window:
                // 16-member tasks from an 8-aligned start, as WK 3 (T24: 24-member
                // tasks; x / 24 = x * 43691 >> 20 exactly below 2^16, and any
                // span past that is a whole-workgroup run either way)
                r = make_uint2(r4[j].x, r4[j].y);  // OOB entries: (0, 0), empty
                nl[j] = r.y > r.x ? (T24 ? (min(r.y - (r.x & ~7u) + 23u, 65535u) * 43691u) >> 20
                                         : (r.y - (r.x & ~7u) + 15u) >> 4)
                                  : 0u;
            } else {
                nl[j] = run_lines(r4[j], wlo, whi, r, min_len, !(MODE == 2 && win >= 0));
            }
            rt[st][e] = r;
            if constexpr (EV3) ev += r.y > r.x ? r.y - r.x : 0u;
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
    int32_t gt[EPT];
    uint4 r4[EPT];
    uint32_t gq[EPT], gq2[EPT];
#pragma unroll
    for (int j = 0; j < EPT; ++j) { r4[j] = make_uint4(0u, 0u, 0u, 0u); gq[j] = gq2[j] = 0u; }
    if constexpr (ONE) {
        s1(0, gt, gq);
        s3(0, r4, gq, gt);
        s1(1, gt, gq);
    } else {
        s1(0, gt, gq);
        s2(0, gt, r4, gq, gq2);
        s1(1, gt, gq);
        s3(0, r4, gq2, gt);
        s2(1, gt, r4, gq, gq2);
        s1(2, gt, gq);
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
    auto n_add = [&](int k, uint32_t v) {
        if constexpr (NK == 0) {
            N[k] += min(v & 0xFFFFu, 1u) | (min(v >> 16, 1u) << 16);
        } else {
            const uint32_t x = pk_min1_u16(v);  // (min(c0, 1), min(c1, 1)) at bits 0, 16
            atomicAdd(&n32[tid + (k >> 1) * NT], (k & 1) ? x << 8 : x);
        }
    };
    // S5 of protein i-1 on counter row (i-1)&1 with its T words (fp64,
    // ascending protein order per pair).  Words past the row's last column
    // stay 0: under WK 3 a wave whose words are all past it stops
    // (wave-uniform: later words are further out).
    auto s5 = [&](int i, const uint32_t (&tw)[KW], int32_t ta) {
        if (!(i >= 1 && glen(i - 1) > 0u)) return;
        uint32_t* acc_p = acc + ((i - 1) & 1) * W;
        const int32_t wbase = (int32_t)uni_u32((uint32_t)tid & ~63u);
        auto div = [&](int32_t c, int32_t dd) -> double {
            if (MODE == 2 && compat) return exact_div_any((double)c, (double)dd);
            return exact_div_small((double)c, (double)dd);
        };
        if ((V & 1) != 0 && !(MODE == 2 && compat)) {
            // both columns of a nonzero word: a zero counter divides 0 by
            // max(d, 1) and adds an exact +0.0 (S >= +0).  WK 3 runs only
            // on loads whose T is every list's length (pl_uses_ends,
            // t_exact): then d = T[p][A] + T[p][B] - c >= T[p][A] >= 1 for a
            // row with entries in p, and the clamp (2 VALU a word) goes
#pragma unroll
            for (int k = 0; k < KW; ++k) {
                if (WK == 3 && wbase + k * NT >= ncw) break;
                const int32_t w = tid + k * NT;
                const uint32_t v = pl_take(acc_p + w);
                if (v) {
                    const int32_t c0 = (int32_t)(v & 0xFFFFu), c1 = (int32_t)(v >> 16);
                    if constexpr (!EV3) ev += (uint32_t)(c0 + c1);
                    n_add(k, v);
                    int32_t d0 = ta + (int32_t)(tw[k] & 0xFFFFu) - c0, d1 = ta + (int32_t)(tw[k] >> 16) - c1;
                    if constexpr (WK != 3 && (V & 4) == 0) {
                        d0 = max(d0, 1);
                        d1 = max(d1, 1);
                    }
                    if constexpr ((V & 8) != 0) {
                        exact_div_pair(c0, d0, c1, d1, S[2 * k], S[2 * k + 1]);
                    } else {
                        S[2 * k] += exact_div_small((double)c0, (double)d0);
                        S[2 * k + 1] += exact_div_small((double)c1, (double)d1);
                    }
                }
            }
            return;
        }
#pragma unroll
        for (int k = 0; k < KW; ++k) {
            // (WK 3 only, where row widths vary within a launch; in the other
            // forms the early stop spilled 6 VGPRs -- 100k streamed 613 -> 689 ms)
            if (WK == 3 && wbase + k * NT >= ncw) break;
            const int32_t w = tid + k * NT;
            const uint32_t v = pl_take(acc_p + w);
            if (v) {
                const int32_t c0 = (int32_t)(v & 0xFFFFu), c1 = (int32_t)(v >> 16);
                if constexpr (!EV3) ev += (uint32_t)(c0 + c1);
                n_add(k, v);
                const int32_t d0 = ta + (int32_t)(tw[k] & 0xFFFFu) - c0, d1 = ta + (int32_t)(tw[k] >> 16) - c1;
                if (c0) S[2 * k] += div(c0, d0);
                if (c1) S[2 * k + 1] += div(c1, d1);
            }
        }
    };
    uint32_t twc[KW];  // T words of the previous protein, carried across the barrier
#pragma unroll
    for (int k = 0; k < KW; ++k) twc[k] = 0u;
    const uint32_t gl8 = (T24 ? 12u : 8u) * (uint32_t)(tid & 1);
    const uint32_t wspan = (uint32_t)(whi - wlo);
    const int grpx = tid >> 1;
    int st_cur = 0;
    uint4 bx = make_uint4(0u, 0u, 0u, 0u);  // T24: the lane's members 8-11
    auto issue2 = [&](int k, int ntk, uint4& bb, uint4& bbh) -> uint32_t {
        if constexpr (T24)
            return pl_issue_m3<TC, BIGF>(r_fm, Fm, tk[st_cur], rt[st_cur], k, ntk, gl8, bb, bbh, bx);
        else
            return pl_issue_m2<TC, BIGF, GP || WK == 4>(r_fm, Fm, tk[st_cur], rt[st_cur], k, ntk, gl8, bb, bbh);
    };
    auto scatter8 = [&](uint32_t* acc_x, uint4 bb, uint4 bbh, uint32_t m) {
        if constexpr (CODE) {
            const uint32_t base = uni_u32((uint32_t)(uintptr_t)acc_x - 2u * (uint32_t)cc0);
            pl_scatter8_code(bb, bbh, m, base);
            if constexpr (T24) pl_scatter4_code(bx, m >> 8, base);
        } else {
            pl_scatter4_m<MODE, WK>(d, a, bb, m & 15u, acc_x - (cc0 >> 1), wlo, wspan);
            pl_scatter4_m<MODE, WK>(d, a, bbh, m >> 4, acc_x - (cc0 >> 1), wlo, wspan);
        }
    };

#pragma unroll 1
    for (int i = 0; i <= P; ++i) {
        const int st = i & 1, cs = i % 3;
        st_cur = st;
        uint32_t* acc_i = acc + st * W;
        const bool has_i = i < P && glen(i) > 0u;
        // S5 first: it waits only for loads of the previous iteration (T
        // words, and with KW = 5 the reloads of spilled registers, if any).
        // (S5 after the first member round's issue, so those loads land
        // while it computes, spills 12 VGPRs at KW = 5: the round's 8
        // member registers live across S5's fp64 temporaries; round 5.)
        // How the 16 waves enter S5 together after the barrier (VERDICT r05
        // #6; flags bits 18-20, set by pfaai_run: the release default 2,
        // PFAAI_PL_STAG in the diagnostics build for A/B).  They all run S5's
        // fp64 work at once and contend for the SIMDs' VALU; 2 drops the
        // first-dispatched half (waves 0-7, which also carry S3 and the second
        // member round) to priority 0 for S5, so the second half's S5 goes
        // first -- 10k rows (diagnostics build, single launches, 7 rounds,
        // profiles/r06/ab_stag.txt) 8.07 -> 7.88 ms; 1 the other way round
        // 7.96; 3 / 5 the second half sleeping 128 / 512 cycles first 8.09 /
        // 8.29; 4 waves 0-3 at priority 3: 8.24.  (6: the first half at 0 and
        // the second at 2; 7: waves 0-3 at 0.)
        if (const uint32_t sg = stag) {
            const int wv = tid >> 6;
            const bool late = wv >= NT / 128;
            if (sg == 2) {
                if (!late) __builtin_amdgcn_s_setprio(0);
            } else if (sg == 1) {
                if (late) __builtin_amdgcn_s_setprio(0);
            } else if (sg == 6) {
                if (!late) __builtin_amdgcn_s_setprio(0);
                else __builtin_amdgcn_s_setprio(2);
            } else if (sg == 7) {
                if (wv < 4) __builtin_amdgcn_s_setprio(0);
            } else if (sg == 3) {
                if (late) __builtin_amdgcn_s_sleep(2);
            } else if (sg == 4) {
                if (wv < 4) __builtin_amdgcn_s_setprio(3);
            } else if (sg == 5) {
                if (late) __builtin_amdgcn_s_sleep(8);
            }
        }
        s5(i, twc, i >= 1 ? (int32_t)uni_u32(taL[i - 1]) : 0);
        stamp(7);
        const int pt = min(i, P - 1);
        if (prio & 1u) __builtin_amdgcn_s_setprio(2);  // loads issue ahead of other waves' S5 (flags bits 16-17)
        const uint32_t tso = (uint32_t)((int64_t)pt * t16w + (cc0 >> 1)) * 4u;
        // S4a: first round of member loads of protein i (one task per lane pair)
        const int nt = has_i ? min((int)uni_u32(ntask[cs]), TC) : 0;
        uint4 b, bh;
        uint32_t okm = issue2(grpx, nt, b, bh);
        stamp(0);
        // S3(i+1), then the prefetches S2(i+2), S1(i+3)
        if constexpr (ONE) {
            if (i + 1 < P) s3(i + 1, r4, gq, gt);
            stamp(1);
            s1(i + 2, gt, gq);
        } else {
            if (i + 1 < P) s3(i + 1, r4, gq2, gt);
            stamp(1);
            s2(i + 2, gt, r4, gq, gq2);
            s1(i + 3, gt, gq);
        }
        stamp(2);
        if (prio) __builtin_amdgcn_s_setprio(0);
        stamp(3);
        if (prio & 2u) __builtin_amdgcn_s_setprio(1);
        // S4b: atomics of the first round, further rounds, whole-workgroup runs
        if (has_i) {
            scatter8(acc_i, b, bh, okm);
            stamp(4);
            // the rounds after the first: from the last lane pair down when
            // flags bit 21 is set -- the first waves hold the G entries (S1-S3)
            // and the first round's low task slots, the last waves idle in both
            for (int k = rev ? 2 * NGX - 1 - grpx : grpx + NGX; k < nt; k += NGX) {
                okm = issue2(k, nt, b, bh);
                scatter8(acc_i, b, bh, okm);
            }
            if (uni_u32(nwhole[cs])) {  // e.g. a tetramer shared by every genome
                for (int wd = 0; wd < kPlEntries / 32; ++wd) {
                    uint32_t m = uni_u32(wmask[cs][wd]);
                    while (m) {
                        const int s = __builtin_ctz(m);
                        m &= m - 1u;
                        const uint32_t rx = uni_u32(rt[st][wd * 32 + s].x), ry = uni_u32(rt[st][wd * 32 + s].y);
                        // four loads in flight per lane (a run of 10 240 members
                        // otherwise took ten dependent HBM round trips)
                        uint32_t mm = rx + tid;
                        const uint32_t lim = ry > 3u * NT ? ry - 3u * NT : 0u;
                        for (; mm < lim; mm += 4u * NT) {
                            const int32_t b0 = d.Fg[mm], b1 = d.Fg[mm + NT], b2 = d.Fg[mm + 2u * NT],
                                          b3 = d.Fg[mm + 3u * NT];
                            pl_add<MODE>(d, a, b0, acc_i, cc0, wlo, whi);
                            pl_add<MODE>(d, a, b1, acc_i, cc0, wlo, whi);
                            pl_add<MODE>(d, a, b2, acc_i, cc0, wlo, whi);
                            pl_add<MODE>(d, a, b3, acc_i, cc0, wlo, whi);
                        }
                        for (; mm < ry; mm += NT) pl_add<MODE>(d, a, d.Fg[mm], acc_i, cc0, wlo, whi);
                    }
                }
            }
        }
        // T words of protein i for the next S5, loaded after the member
        // rounds: live across the barrier only; T[p][A] comes from taL
#pragma unroll
        for (int k = 0; k < KW; ++k) twc[k] = bld_u32(r_t16, (uint32_t)tid * 4u, tso + (uint32_t)k * (NT * 4u));
        stamp(5);
        // recycle the protein-(i+2) counter set (last read by S4(i-1))
        if (tid < kPlEntries / 32) wmask[(i + 2) % 3][tid] = 0u;
        if (tid == 32) { ntask[(i + 2) % 3] = 0u; nwhole[(i + 2) % 3] = 0u; }
        if constexpr (CODE) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // pl_scatter8_code's atomics
        __syncthreads();
        stamp(6);
    }
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
            int32_t n = NK == 1 ? (int32_t)((n32[tid + (k >> 1) * NT] >> (8 * (k & 1) + 16 * h)) & 0xFFu)
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
        put_pair<MODE>(d, a, cc0 + 2 * w + 0, ok, sv, nv, compat, aji, s_out, n_out);
    }
}

// Dynamic LDS of a k_rows_pl launch: the counter rows, goff, the N bytes
// (NK 1) and T[p][A].
template <int KW, int NT, int NK>
constexpr size_t pl_lds_bytes(int P) {
    return (2 * (size_t)KW * NT + (size_t)P + 1 + (NK == 1 ? (size_t)(KW + 1) / 2 * NT : 0) + ((size_t)P + 1) / 2) * 4;
}

}  // namespace pfaai
