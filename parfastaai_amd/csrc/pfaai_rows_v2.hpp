// pfaai_rows_v2.hpp -- k_rows_v2: the row kernel with every load of a protein
// issued one protein ahead (genome-major input).
//
// Computes exactly what k_rows_pl computes (pfaai_rows_pl.hpp): for output
// row A and every protein p in ascending order, the intersection counts
// c(p, A, B) = |{t : A, B both in run (t, p)}| -- the run-lengths of the
// reference's sorted E (ds_helper.hpp:270-357, psort.hpp:27-53) -- then
// S += c / (T[p][A] + T[p][B] - c), N += 1 over c > 0
// (algorithm_impl.hpp:240-275) and AJI = S / N (algorithm_impl.hpp:318).
//
// Why a second form.  k_rows_pl builds one line-task list per protein shared
// by the whole workgroup, so a protein's member loads can only be issued
// after the barrier that publishes its list -- each protein pays at least
// one exposed member-load latency (measured: 5.3 us per (row, protein) at
// 10k with two workgroups per CU, and 6.9 of 10.4 ms left with no member
// work at all), and the 64-VGPR budget of two workgroups per CU spills.
// Here the line tasks are WAVE-LOCAL: G entry e of a protein belongs to wave
// e % 16 (so every wave gets ~1/16 of the row's runs), the wave cuts its
// runs into 16-member line tasks with a DPP scan -- no LDS atomics, no
// barrier -- and issues the member loads of protein i+1 right away, into
// registers that are consumed after the next barrier.  One 1024-thread
// workgroup per CU (128 VGPRs): the latency of every load of a protein is
// covered by one whole iteration of the previous protein's work.
//
//   iteration i:  T(i)     T16 words of the thread's columns, T[i][A]  (for S5 next iteration)
//                 S3(i+1)  wave-local line tasks of protein i+1 (runs too long or over the
//                          wave's capacity -> the workgroup's long-run list, by protein % 3)
//                 M(i+1)   member loads of the first kV2Rounds rounds of protein i+1
//                 S2(i+2)  run-table lookups, S1(i+3) G-list load
//                 S5(i-1)  normalise counter row (i-1)&1 into S, N; clear it
//                 S4(i)    ds_add_u32 of M(i) (loaded one iteration ago), further rounds
//                          of protein i's tasks, the long runs of protein i (whole workgroup)
//                 barrier
//
// Loads are issued in the order they are consumed and never under a branch
// (gfx9 retires vector loads in order): raw buffer loads with out-of-range
// offsets stand in for absent work.  Variable-trip loops (further rounds,
// long runs) come last in the iteration, after every prefetch.
//
// Preconditions (host-checked, pfaai_hip.hip): genome-major input, every
// (genome, protein) G list <= kPlEntries, the row chunk <= KW * 1024 counter
// words, T < 2^16, P * 160000 * 16 B < 4 GiB.
#pragma once
#include "pfaai_rows_pl.hpp"

namespace pfaai {

constexpr int kV2Threads = 1024;
constexpr int kV2Waves = kV2Threads / 64;
constexpr int kV2Rounds = 2;        // member rounds (16 line tasks each) issued one protein ahead
constexpr int kV2TaskCap = 256;     // line tasks per wave and protein: lane | line << 6
constexpr int kV2MaxLines = 63;     // longer runs: whole-workgroup walk
constexpr int kV2LongCap = kPlEntries;  // long runs per protein: at most one per G entry

// E triple (p, A, b): +1 into the u32 counter of column b (one LDS word per
// column: the address is one shift-add and the operand the constant 1).
// acc_w points at the counter of column wlo; o = b - wlo out of range also
// drops b = -1 (no member).
template <int MODE>
__device__ __forceinline__ void v2_add(const Dev& d, int32_t a, int32_t b, int32_t wlo, uint32_t* acc_w,
                                       uint32_t width) {
    const uint32_t o = (uint32_t)(b - wlo);
    if (o >= width) return;
    if (MODE == 1 && !(b != a && (!d.is_q[b] || b > a))) return;  // isValidPair, ds_impl.hpp:270-273
    if (MODE == kModeFull && b == a) return;
    atomicAdd(acc_w + o, 1u);
}

template <int MODE>
__device__ __forceinline__ void v2_scatter4(const Dev& d, int32_t a, uint4 b, uint32_t ok, int32_t wlo,
                                            uint32_t* acc_w, uint32_t width) {
    v2_add<MODE>(d, a, (ok & 1u) ? (int32_t)b.x : -1, wlo, acc_w, width);
    v2_add<MODE>(d, a, (ok & 2u) ? (int32_t)b.y : -1, wlo, acc_w, width);
    v2_add<MODE>(d, a, (ok & 4u) ? (int32_t)b.z : -1, wlo, acc_w, width);
    v2_add<MODE>(d, a, (ok & 8u) ? (int32_t)b.w : -1, wlo, acc_w, width);
}

// CLK (diagnostics library only, PFAAI_V2_CLK): per wave of the first
// kClkBlocks workgroups, shader clocks of the loop's stages into
// clk[(block * 16 + wave) * 8 + stage] -- 0 T issue + S3, 1 member / run /
// G issue, 2 S5, 3 S4 prefetched rounds, 4 S4 further rounds, 5 long runs,
// 6 barrier; slot 7 counts further rounds (tools/gpu/stage_clocks.py --v2).
template <int MODE, int KW, bool BIGF = false, bool CLK = false>
__global__ __launch_bounds__(kV2Threads, 4) void k_rows_v2(Dev d, int64_t row_begin, int32_t chunk_cols,
                                                          int32_t abs_chunk, uint32_t flags,
                                                          const unsigned long long* __restrict__ first_key,
                                                          double* __restrict__ aji, double* __restrict__ s_out,
                                                          int32_t* __restrict__ n_out,
                                                          unsigned long long* __restrict__ n_events,
                                                          unsigned long long* __restrict__ clk = nullptr) {
    constexpr int NT = kV2Threads;
    constexpr int W = 2 * KW * NT;  // u32 column counters per row chunk
    extern __shared__ uint32_t v2_smem[];              // acc[2][W], goff[P + 1]
    __shared__ uint16_t tk[kV2Waves][2][kV2TaskCap];    // wave-local line tasks, by protein & 1
    __shared__ uint2 rt[kV2Waves][2][64];               // the wave's runs: member range [lo, hi)
    __shared__ uint2 lr[3][kV2LongCap];                 // long runs, by protein % 3
    __shared__ uint32_t nlong[3];

    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int grp = lane >> 2, gl = lane & 3;  // 16 four-lane groups per wave
    const int64_t rl = xcd_row(blockIdx.x, gridDim.x, d.xcd_chunk);
    const int32_t a = d.row_genome[row_begin + rl];
    int32_t clo, chi;
    row_cols<MODE>(d, a, clo, chi);
    const int32_t cc0 = abs_chunk >= 0 ? abs_chunk * chunk_cols : (clo & ~1) + (int32_t)blockIdx.y * chunk_cols;
    const int32_t wlo = max(cc0, clo), whi = min(chi, cc0 + chunk_cols);
    if (wlo >= whi) return;  // uniform
    const int32_t ncw = (whi - cc0 + 1) >> 1;  // column pairs (2w, 2w+1) of the chunk
    const uint32_t width = (uint32_t)(whi - wlo);
    const bool compat = flags & 1u;
    const uint32_t min_len = abs_chunk >= 0 ? 0u : 1u;
    const int P = d.n_prot;
    uint32_t* acc = v2_smem;
    uint32_t* goff = v2_smem + 2 * W;

    const int64_t g0 = d.G_off[(int64_t)a * P];
    for (int p = tid; p <= P; p += NT) goff[p] = (uint32_t)(d.G_off[(int64_t)a * P + p] - g0);
    for (int w = tid; w < 2 * W; w += NT) acc[w] = 0u;
    if (tid < 3) nlong[tid] = 0u;
    const int32_t tca = compat ? d.tcol_row[a] : a;
    const uint16_t* T16 = compat ? d.T16c : d.T16;
    const int64_t t16w = d.t16_cols >> 1;
    double S[2 * KW];
    uint32_t N[KW];
#pragma unroll
    for (int k = 0; k < KW; ++k) { S[2 * k] = 0.0; S[2 * k + 1] = 0.0; N[k] = 0u; }
    uint32_t ev = 0;
    __syncthreads();

    const rsrc_t r_fg = mk_rsrc(d.Fg, (uint64_t)(d.n_f + 16) * 4u);
    const rsrc_t r_g = mk_rsrc(d.G_tet + g0, (uint64_t)uni_u32(goff[P]) * 4u);
    const rsrc_t r_blk = mk_rsrc(d.blk, (uint64_t)P * kNTetramers * 16u);
    const rsrc_t r_t16 = mk_rsrc(T16, (uint64_t)P * d.t16_cols * 2u);
    const rsrc_t r_t = mk_rsrc(d.T, (uint64_t)P * d.t_cols * 4u);
    auto glen = [&](int p) -> uint32_t { return p < P ? uni_u32(goff[p + 1]) - uni_u32(goff[p]) : 0u; };
    // G entry of this lane for protein p: e = lane * 16 + wave (every wave gets ~1/16 of the list)
    const uint32_t e_lane = (uint32_t)(lane * kV2Waves + wv);
    auto s1 = [&](int p) -> int32_t {
        const uint32_t o = p < P ? uni_u32(goff[p]) : 0u;
        return (int32_t)bld_u32(r_g, e_lane < glen(p) ? e_lane * 4u : kOOB, o * 4u);
    };
    auto s2 = [&](int p, int32_t gt) -> uint4 {
        return bld_u128(r_blk, e_lane < glen(p) ? (uint32_t)gt * 16u : kOOB,
                        (uint32_t)min(p, P - 1) * (kNTetramers * 16u));
    };
    // wave-local tasks of protein q from this lane's run-table entry; returns the wave's task count
    auto s3 = [&](int q, const uint4& r4) -> uint32_t {
        const int st = q & 1, cs = q % 3;
        uint2 r;
        const uint32_t nl = run_lines(r4, wlo, whi, r, min_len);
        rt[wv][st][lane] = r;
        bool lng = nl > (uint32_t)kV2MaxLines;
        const uint32_t v = lng ? 0u : nl;
        const uint32_t inc = wave_scan_dpp(v);
        const uint32_t e0 = inc - v;
        // tasks past the wave's capacity: the run goes to the long list; the
        // offsets ascend with the lane, so the kept tasks are a prefix
        if (inc > (uint32_t)kV2TaskCap) lng = lng || v > 0u;
        const unsigned long long kept = __ballot(inc <= (uint32_t)kV2TaskCap);  // lane 0 always (v <= 63)
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63 - __builtin_clzll(kept));
        if (lng) {
            const uint32_t slot = atomicAdd(&nlong[cs], 1u);  // < kV2LongCap: one per G entry
            lr[cs][slot] = r;
        } else {
            uint16_t* t = tk[wv][st];
#pragma unroll
            for (uint32_t l = 0; l < 4; ++l)
                if (l < v) t[e0 + l] = (uint16_t)(lane | (l << 6));
#pragma unroll 1
            for (uint32_t l = 4; l < v; ++l) t[e0 + l] = (uint16_t)(lane | (l << 6));
        }
        __builtin_amdgcn_wave_barrier();  // the wave reads its own tasks next
        return tot;
    };
    // one member round of protein q: task k of this lane's group, 4 members (16 B)
    auto issue = [&](int q, int k, uint32_t nt, uint4& b) -> uint32_t {
        const int st = q & 1;
        const uint32_t t = tk[wv][st][min(k, kV2TaskCap - 1)];
        const uint2 rr = rt[wv][st][t & 63u];
        const uint32_t m0 = (rr.x & ~(uint32_t)(kGroup - 1)) + (t >> 6) * kGroup + 4u * (uint32_t)gl;
        const bool task = (uint32_t)k < nt;
        uint32_t ok = 0u;
#pragma unroll
        for (int j = 0; j < 4; ++j) ok |= (uint32_t)(task && m0 + j >= rr.x && m0 + j < rr.y) << j;
        if constexpr (BIGF)
            b = *reinterpret_cast<const uint4*>(d.Fg + (ok ? m0 : 0u));
        else
            b = bld_u128(r_fg, ok ? m0 * 4u : kOOB, 0u);
        return ok;
    };

    // prologue: tasks + member loads of protein 0, run-table entries of protein 1, G of protein 2
    int32_t gt = s1(0);
    uint4 r4 = s2(0, gt);
    gt = s1(1);
    uint32_t nt_cur = s3(0, r4);
    uint4 mb[kV2Rounds];
    uint32_t okb[kV2Rounds];
#pragma unroll
    for (int r = 0; r < kV2Rounds; ++r) okb[r] = issue(0, r * 16 + grp, nt_cur, mb[r]);
    r4 = s2(1, gt);
    gt = s1(2);
    uint32_t tw[KW];
#pragma unroll
    for (int k = 0; k < KW; ++k) tw[k] = 0u;
    int32_t ta = 0;
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
#pragma unroll 1
    for (int i = 0; i <= P; ++i) {
        const int pt = min(i, P - 1);
        // T(i): issued first, consumed by S5(i) in the next iteration
        uint32_t twn[KW];
        const uint32_t tso = (uint32_t)((int64_t)pt * t16w + (cc0 >> 1)) * 4u;
#pragma unroll
        for (int k = 0; k < KW; ++k) {
            const int32_t w = tid + k * NT;
            twn[k] = bld_u32(r_t16, w < ncw ? (uint32_t)tid * 4u : kOOB, tso + (uint32_t)k * (NT * 4u));
        }
        const int32_t tan = (int32_t)bld_u32(r_t, 0u, (uint32_t)((int64_t)pt * d.t_cols + tca) * 4u);
        // S3(i+1) + M(i+1)
        uint32_t nt_next = 0u;
        if (i + 1 < P) nt_next = s3(i + 1, r4);  // uniform branch, no loads inside
        stamp(0);
        uint4 mbn[kV2Rounds];
        uint32_t okn[kV2Rounds];
#pragma unroll
        for (int r = 0; r < kV2Rounds; ++r) okn[r] = issue(i + 1, r * 16 + grp, nt_next, mbn[r]);
        // S2(i+2), S1(i+3)
        r4 = s2(i + 2, gt);
        gt = s1(i + 3);
        stamp(1);
        // S5(i-1): normalise (fp64, ascending protein order per pair); both
        // columns of a pair computed together (a zero count divides 0 by 1)
        if (i >= 1 && glen(i - 1) > 0u) {
            uint32_t* acc_p = acc + ((i - 1) & 1) * W;
#pragma unroll
            for (int k = 0; k < KW; ++k) {
                const int32_t w = tid + k * NT;
                if (w < ncw) {
                    uint2* cw = reinterpret_cast<uint2*>(acc_p) + w;
                    const uint2 v = *cw;
                    if (v.x | v.y) {
                        *cw = make_uint2(0u, 0u);
                        const int32_t c0 = (int32_t)v.x, c1 = (int32_t)v.y;
                        ev += (uint32_t)(c0 + c1);
                        const int32_t d0 = c0 ? ta + (int32_t)(tw[k] & 0xFFFFu) - c0 : 1;
                        const int32_t d1 = c1 ? ta + (int32_t)(tw[k] >> 16) - c1 : 1;
                        S[2 * k] += exact_div_any((double)c0, (double)d0);
                        S[2 * k + 1] += exact_div_any((double)c1, (double)d1);
                        N[k] += (uint32_t)(c0 != 0) + ((uint32_t)(c1 != 0) << 16);
                    }
                }
            }
        }
        stamp(2);
        // S4(i): the member rounds loaded one iteration ago, then further
        // rounds and the long runs of protein i
        if (i < P && glen(i) > 0u) {
            uint32_t* acc_i = acc + (i & 1) * W;
            uint32_t* acc_w = acc_i + (wlo - cc0);
#pragma unroll
            for (int r = 0; r < kV2Rounds; ++r) v2_scatter4<MODE>(d, a, mb[r], okb[r], wlo, acc_w, width);
            stamp(3);
            for (int k = kV2Rounds * 16 + grp; (uint32_t)(k - grp) < nt_cur; k += 32) {
                uint4 b0, b1;
                const uint32_t o0 = issue(i, k, nt_cur, b0);
                const uint32_t o1 = issue(i, k + 16, nt_cur, b1);
                v2_scatter4<MODE>(d, a, b0, o0, wlo, acc_w, width);
                v2_scatter4<MODE>(d, a, b1, o1, wlo, acc_w, width);
                if constexpr (CLK) ck[7] += 1;
            }
            stamp(4);
            const uint32_t nl = min(uni_u32(nlong[i % 3]), (uint32_t)kV2LongCap);
            for (uint32_t q = 0; q < nl; ++q) {  // e.g. a tetramer shared by every genome
                const uint32_t rx = uni_u32(lr[i % 3][q].x), ry = uni_u32(lr[i % 3][q].y);
                for (uint32_t mm = rx + tid; mm < ry; mm += NT) v2_add<MODE>(d, a, d.Fg[mm], wlo, acc_w, width);
            }
            stamp(5);
        }
        // the long-run list of protein i+2 (last read by S4(i-1)) starts empty
        if (tid == 0) nlong[(i + 2) % 3] = 0u;
#pragma unroll
        for (int k = 0; k < KW; ++k) tw[k] = twn[k];
        ta = tan;
#pragma unroll
        for (int r = 0; r < kV2Rounds; ++r) { mb[r] = mbn[r]; okb[r] = okn[r]; }
        nt_cur = nt_next;
        __syncthreads();
        stamp(6);
    }
    if constexpr (CLK) {
        if (lane == 0 && blockIdx.x < kClkBlocks && blockIdx.y == 0)
            for (int j = 0; j < 8; ++j) clk[((int64_t)blockIdx.x * kV2Waves + wv) * 8 + j] = ck[j];
    }

    ev = wave_sum_u32(ev);
    if (lane == 0 && ev) atomicAdd(n_events, (unsigned long long)ev);

    // epilogue: JAC S/N and AJI at the reference's JAC index
#pragma unroll
    for (int k = 0; k < KW; ++k) {
        const int32_t w = tid + k * NT;
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
