// pfaai_counts.hpp -- two-phase row path (the default on genome-major input).
//
//   k_counts  E construction.  One workgroup per item (output row A, protein
//             p, column chunk): the runs (t, p) of A's own G entries (A, p, t)
//             -- looked up in the run table k_blk builds -- are cut into
//             16-member line tasks; 16-lane groups load the member ids and
//             ds_add_u32 +1 into an LDS row of packed u16 counters.  The row
//             is the run-length encoding of the reference's sorted E for
//             (A, p, *) (ds_helper.hpp:270-357 + psort.hpp:27-53 +
//             algorithm_impl.hpp:123-219): c(p, A, B) = |{t : A, B in run
//             (t, p)}|.  It is written to HBM densely: cnt[p][cell], one u16
//             per (row, column) cell.
//   k_norm    computeJAC / computeAJI.  One workgroup per row streams the
//             row's cells; each thread owns 8 columns and walks p = 0..P-1
//             in ascending order: S += c / (T[p][A] + T[p][B] - c), N += 1
//             over c > 0 (algorithm_impl.hpp:240-275), AJI = S / N
//             (algorithm_impl.hpp:318), written at the reference's JAC index.
//
// Why two phases: a one-row-per-workgroup kernel must finish protein p's
// scatter before it may normalise p (the fp64 sum is protein-ordered), so
// every protein is a barrier-separated chain of dependent loads; measured
// on MI355X that structure is latency- and barrier-bound.  Here the items
// of phase 1 are independent (no order at all -- integer counts commute),
// small (256 threads, 4 workgroups per CU) and scheduled so that the rows
// of one row group meet the same runs on the same XCD; phase 2 is a
// coalesced stream.  The price is the count tensor: P x cells x 2 B of HBM
// (10 GB at 10 000 genomes), written once and read once; pfaai_run cuts
// the rows into tiles whose tensor fits a budget.
//
// Cell layout (row-major per protein): row r's window of columns
// [clo, chi) (row_cols) starts at base0 = clo & ~7 so every row begins on a
// 16-B boundary of both the count tensor and T16; its length is rounded up
// to 8 cells.  cell(r, B) = cbase[r] + (B - base0(r)), cbase = prefix sum.
#pragma once
#include "pfaai_kernels.hpp"

namespace pfaai {

constexpr int kCntThreads = 256;
constexpr int kCntGroups = kCntThreads / kGroup;    // 16-lane groups
constexpr int kCntChunkW = 4096;                    // counter words per item (8192 columns)
constexpr int kCntRuns = 1024;                      // G entries per pass
constexpr int kCntGPT = kCntRuns / kCntThreads;     // G entries per thread per pass
constexpr int kCntTaskCap = 4096;                   // u16 line tasks per pass
constexpr int kCntMaxLines = 63;                    // longer runs: whole-workgroup walk
constexpr int kCntUnroll = 8;                       // member loads in flight per lane
constexpr int kCntRowGroup = 16;                    // rows scheduled together (shared runs)
constexpr uint16_t kCntNoTask = 0xFFFFu;

using rsrc_t = __amdgpu_buffer_rsrc_t;
constexpr int kRsrcWord3 = 0x00020000;  // gfx9 raw buffer: 32-bit data, no swizzle

// Raw buffer loads: a 4-SGPR resource, a 32-bit per-lane byte offset and a
// scalar byte offset instead of a 64-bit address per lane.  Out-of-range
// offsets read 0 and fetch nothing, so loads can be issued unconditionally.
__device__ __forceinline__ rsrc_t mk_rsrc(const void* p, uint64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0,
                                             (int)(bytes > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)bytes), kRsrcWord3);
}
__device__ __forceinline__ uint32_t bld_u32(rsrc_t r, uint32_t voff, uint32_t soff) {
    return (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff, 0);
}
__device__ __forceinline__ uint4 bld_u128(rsrc_t r, uint32_t voff, uint32_t soff) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, 0);
    return make_uint4((uint32_t)v[0], (uint32_t)v[1], (uint32_t)v[2], (uint32_t)v[3]);
}
__device__ __forceinline__ uint32_t uni_u32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
constexpr uint32_t kOOB = 0xFFFFFFF0u;

// Inclusive wave64 prefix sum with DPP row shifts and row broadcasts.
__device__ __forceinline__ uint32_t wave_scan_dpp(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

// Run-table entry -> member range [lo, hi) and its line count after pruning
// to the column window [wlo, whi) with the run's line splitters (k_blk).
__device__ __forceinline__ uint32_t run_lines(uint4 r4, int32_t wlo, int32_t whi, uint2& r) {
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
                if (f <= wlo) l0 = i;            // lines < i hold ids < f <= wlo
                if (f >= whi && l1 > i) l1 = i;  // lines >= i hold ids >= f >= whi
            }
        }
        if (l1 <= l0) return 0u;
        if (l0) r.x = first + l0 * kGroup;
        if (l1 < nl) r.y = first + l1 * kGroup;
        nl = l1 - l0;
    }
    return nl;
}

// One E triple (p, A, b): +1 into the u16 counter of column b.
template <int MODE>
__device__ __forceinline__ void cnt_add(const Dev& d, int32_t a, int32_t b, uint32_t* acc, int32_t cc0, int32_t wlo,
                                        int32_t whi, uint32_t& ev) {
    if (b < wlo || b >= whi) return;  // also drops b = -1 (no member)
    if (MODE == 1 && !(b != a && (!d.is_q[b] || b > a))) return;  // isValidPair, ds_impl.hpp:270-273
    const uint32_t o = (uint32_t)(b - cc0);
    atomicAdd(&acc[o >> 1], 1u << ((o & 1u) << 4));
    ++ev;
}

// Row-local helpers shared by both phases.
struct RowWin {
    int32_t a, clo, chi, base0, ncell;  // ncell: cells of the row in the tensor (multiple of 8)
};
template <int MODE>
__device__ __forceinline__ RowWin row_win(const Dev& d, int64_t row) {
    RowWin w;
    w.a = d.row_genome[row];
    row_cols<MODE>(d, w.a, w.clo, w.chi);
    w.base0 = w.clo & ~7;
    w.ncell = w.chi > w.clo ? ((w.chi - w.base0 + 7) & ~7) : 0;  // = the host's cbase step
    return w;
}

// ---------------------------------------------------------------------------
// k_counts: phase 1.  Items are ordered (row group of 16, chunk, protein,
// row) and dealt to the 8 XCDs in contiguous ranges, so the 16 rows of a
// group -- in practice related genomes, which share most runs -- read the
// same member lines out of one L2 at about the same time.
// ---------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(kCntThreads) void k_counts(Dev d, int64_t row_begin, int32_t n_rows, int32_t n_chunks,
                                                        const unsigned long long* __restrict__ cbase,
                                                        uint64_t pitch, uint32_t* __restrict__ cnt,
                                                        unsigned long long* __restrict__ n_events,
                                                        unsigned long long* __restrict__ prof, uint32_t dbg) {
    __shared__ uint32_t acc[kCntChunkW];
    __shared__ uint2 rt[kCntRuns];
    __shared__ uint16_t tk[kCntTaskCap];
    __shared__ uint32_t wmask[kCntRuns / 32];
    __shared__ uint32_t ntask, nwhole;

    const int tid = threadIdx.x, lane = tid & 63;
    const int grp = tid / kGroup, gl = tid % kGroup;
    const int P = d.n_prot;
    // diagnostics: per-stage clocks of wave 0 summed into prof[0..7]
    uint64_t tl = prof ? clock64() : 0;
    auto tick = [&](int slot) {
        if (prof) {
            const uint64_t t = clock64();
            if (tid == 0) atomicAdd(&prof[slot], (unsigned long long)(t - tl));
            tl = t;
        }
    };
    // item -> (row, chunk, protein), XCD-contiguous
    const int64_t n_groups = (n_rows + kCntRowGroup - 1) / kCntRowGroup;
    const int64_t total = n_groups * kCntRowGroup * n_chunks * P;
    const int64_t per = (total + kXcds - 1) / kXcds;
    const int64_t L = (dbg & 4u) ? (int64_t)blockIdx.x : (int64_t)(blockIdx.x % kXcds) * per + blockIdx.x / kXcds;
    if (L >= total) return;
    const int rig = (int)(L % kCntRowGroup);
    int64_t q = L / kCntRowGroup;
    const int p = (int)(q % P);
    q /= P;
    const int chunk = (int)(q % n_chunks);
    const int64_t r = (q / n_chunks) * kCntRowGroup + rig;
    if (r >= n_rows) return;
    const RowWin rw = row_win<MODE>(d, row_begin + r);
    const int32_t a = rw.a;
    const int32_t cc0 = rw.base0 + chunk * (2 * kCntChunkW);
    const int32_t wlo = max(cc0, rw.clo), whi = min(rw.chi, cc0 + 2 * kCntChunkW);
    if (cc0 - rw.base0 >= rw.ncell) return;  // this chunk lies past the row (uniform)
    // uint4 (8 cells) of this chunk in the tensor
    const int32_t ncw4 = min(rw.ncell - (cc0 - rw.base0), 2 * kCntChunkW) >> 3;
    uint4* out4 = reinterpret_cast<uint4*>(cnt + (uint64_t)p * pitch + (cbase[row_begin + r] - cbase[row_begin]) / 2 +
                                           (uint64_t)chunk * kCntChunkW);
    uint4* acc4 = reinterpret_cast<uint4*>(acc);
    for (int w = tid; w < ncw4; w += kCntThreads) acc4[w] = make_uint4(0u, 0u, 0u, 0u);
    if (tid == 0) { ntask = 0u; nwhole = 0u; }
    if (tid < kCntRuns / 32) wmask[tid] = 0u;

    uint32_t ev = 0;
    tick(0);
    const int64_t gk = (int64_t)a * P + p;
    const int64_t gb = d.G_off[gk], ge = d.G_off[gk + 1];
    if (wlo < whi && gb < ge) {
        const rsrc_t r_fg = mk_rsrc(d.Fg, (uint64_t)d.n_f * 4u);
        const rsrc_t r_g = mk_rsrc(d.G_tet + gb, (uint64_t)(ge - gb) * 4u);
        const rsrc_t r_blk = mk_rsrc(d.blk + (int64_t)p * kNTetramers, (uint64_t)kNTetramers * 16u);
        for (int64_t pass = 0; pass < ge - gb; pass += kCntRuns) {  // uniform; one pass unless > 1024 runs
            const uint32_t n = (uint32_t)min<int64_t>(ge - gb - pass, kCntRuns);
            __syncthreads();  // counters / staging of the previous pass are consumed
            // G entries tid + 256 j of this pass: tetramer -> run -> lines
            int32_t t[kCntGPT];
            uint4 r4[kCntGPT];
#pragma unroll
            for (int j = 0; j < kCntGPT; ++j) {
                const uint32_t k = (uint32_t)(tid + j * kCntThreads);
                t[j] = (int32_t)bld_u32(r_g, k < n ? k * 4u : kOOB, (uint32_t)pass * 4u);
            }
#pragma unroll
            for (int j = 0; j < kCntGPT; ++j) {
                const uint32_t k = (uint32_t)(tid + j * kCntThreads);
                r4[j] = bld_u128(r_blk, k < n ? (uint32_t)t[j] * 16u : kOOB, 0u);
            }
            tick(1);
            uint32_t nl[kCntGPT], v = 0;
#pragma unroll
            for (int j = 0; j < kCntGPT; ++j) {
                uint2 rr;
                nl[j] = run_lines(r4[j], wlo, whi, rr);
                rt[tid + j * kCntThreads] = rr;
                if (nl[j] > (uint32_t)kCntMaxLines) {  // whole-workgroup walk
                    atomicOr(&wmask[(tid + j * kCntThreads) >> 5], 1u << (tid & 31));
                    atomicAdd(&nwhole, 1u);
                    nl[j] = 0;
                }
                v += nl[j];
            }
            // wave-level reservation of the lane's line tasks (no block scan)
            const uint32_t inc = wave_scan_dpp(v);
            const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
            uint32_t base = 0;
            if (tot) {
                if (lane == 63) base = atomicAdd(&ntask, tot);
                base = (uint32_t)__builtin_amdgcn_readlane((int)base, 63);
            }
            uint32_t e = base + inc - v;
#pragma unroll
            for (int j = 0; j < kCntGPT; ++j) {
                const uint32_t slot = (uint32_t)(tid + j * kCntThreads);
                if (e + nl[j] <= (uint32_t)kCntTaskCap) {
#pragma unroll 1
                    for (uint32_t l = 0; l < nl[j]; ++l) tk[e + l] = (uint16_t)(slot | (l << 10));
                } else if (nl[j]) {  // over capacity: the whole workgroup walks this run
#pragma unroll 1
                    for (uint32_t l = e; l < (uint32_t)kCntTaskCap; ++l) tk[l] = kCntNoTask;
                    atomicOr(&wmask[slot >> 5], 1u << (slot & 31));
                    atomicAdd(&nwhole, 1u);
                }
                e += nl[j];
            }
            tick(2);
            __syncthreads();
            tick(3);
            // line tasks: 16-lane group g takes tasks g, g+16, ...; 8 loads in flight
            const int nt = (dbg & 2u) ? 0 : (int)min(uni_u32(ntask), (uint32_t)kCntTaskCap);  // 2: no member loads
            for (int k0 = grp; k0 < nt; k0 += kCntGroups * kCntUnroll) {
                int32_t b[kCntUnroll];
                uint32_t okm = 0u;
#pragma unroll
                for (int h = 0; h < kCntUnroll; h += 4) {
                    uint32_t tt[4];
                    uint2 rr[4];
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj) tt[jj] = tk[min(k0 + (h + jj) * kCntGroups, kCntTaskCap - 1)];
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj) rr[jj] = rt[tt[jj] & 1023u];
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj) {
                        const uint32_t m = (rr[jj].x & ~(uint32_t)(kGroup - 1)) + (tt[jj] >> 10) * kGroup + (uint32_t)gl;
                        const bool ok = k0 + (h + jj) * kCntGroups < nt && tt[jj] != kCntNoTask && m >= rr[jj].x &&
                                        m < rr[jj].y;
                        okm |= (uint32_t)ok << (h + jj);
                        b[h + jj] = (int32_t)bld_u32(r_fg, ok ? m * 4u : kOOB, 0u);
                    }
                }
                if (dbg & 1u) {  // diagnostics: count, no atomics
#pragma unroll
                    for (int u = 0; u < kCntUnroll; ++u) ev += ((okm >> u) & 1u) && b[u] >= wlo && b[u] < whi;
                    continue;
                }
#pragma unroll
                for (int u = 0; u < kCntUnroll; ++u) cnt_add<MODE>(d, a, (okm >> u) & 1u ? b[u] : -1, acc, cc0, wlo, whi, ev);
            }
            tick(4);
            // runs too long for line tasks (e.g. a tetramer shared by every genome)
            if (uni_u32(nwhole)) {
                for (int wd = 0; wd < kCntRuns / 32; ++wd) {
                    uint32_t m = uni_u32(wmask[wd]);
                    while (m) {
                        const int s = __builtin_ctz(m);
                        m &= m - 1u;
                        const uint32_t rx = uni_u32(rt[wd * 32 + s].x), ry = uni_u32(rt[wd * 32 + s].y);
                        for (uint32_t mm = rx + tid; mm < ry; mm += 4 * kCntThreads) {
                            int32_t bb[4];
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                const uint32_t x = mm + u * kCntThreads;
                                bb[u] = x < ry ? (int32_t)bld_u32(r_fg, x * 4u, 0u) : -1;
                            }
#pragma unroll
                            for (int u = 0; u < 4; ++u) cnt_add<MODE>(d, a, bb[u], acc, cc0, wlo, whi, ev);
                        }
                    }
                }
            }
            tick(5);
            __syncthreads();
            if (tid == 0) { ntask = 0u; nwhole = 0u; }
            if (tid < kCntRuns / 32) wmask[tid] = 0u;
        }
    }
    __syncthreads();
    tick(6);
    if (dbg & 8u) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        for (int w = tid; w < ncw4; w += kCntThreads) {
            const uint4 v = acc4[w];
            __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4*>(out4 + w));
        }
    } else {
        for (int w = tid; w < ncw4; w += kCntThreads) out4[w] = acc4[w];
    }
    tick(7);
    ev = wave_sum_u32(ev);
    if (lane == 0 && ev) atomicAdd(n_events, (unsigned long long)ev);
}

// ---------------------------------------------------------------------------
// k_norm: phase 2.  One workgroup per row; thread owns 8 consecutive cells
// (one uint4 of the count tensor, one uint4 of T16) per sweep and walks the
// proteins in ascending order, 4 proteins' loads in flight.
// ---------------------------------------------------------------------------
constexpr int kNormThreads = 256;
constexpr int kNormUnroll = 4;

__device__ __forceinline__ void norm_cell(uint32_t c, uint32_t tb, int32_t ta, double& S, uint32_t& N, uint32_t inc) {
    if (c) {
        S += (double)c / (double)(ta + (int32_t)tb - (int32_t)c);
        N += inc;
    }
}

template <int MODE>
__global__ __launch_bounds__(kNormThreads) void k_norm(Dev d, int64_t row_begin, const unsigned long long* __restrict__ cbase,
                                                       uint64_t pitch, const uint32_t* __restrict__ cnt, uint32_t flags,
                                                       const unsigned long long* __restrict__ first_key,
                                                       double* __restrict__ aji, double* __restrict__ s_out,
                                                       int32_t* __restrict__ n_out) {
    extern __shared__ int32_t ta_lds[];  // T[p][A] for p < P
    const int tid = threadIdx.x;
    const int64_t r = blockIdx.x;
    const RowWin rw = row_win<MODE>(d, row_begin + r);
    const int32_t a = rw.a;
    const bool compat = flags & 1u;
    const int P = d.n_prot;
    const int32_t tca = compat ? d.tcol_row[a] : a;
    for (int p = tid; p < P; p += kNormThreads) ta_lds[p] = d.T[(int64_t)p * d.t_cols + tca];
    __syncthreads();
    const uint16_t* T16 = compat ? d.T16c : d.T16;
    const int32_t ncell = rw.ncell;
    const uint64_t cofs = (cbase[row_begin + r] - cbase[row_begin]) / 2;  // words
    const rsrc_t r_t = mk_rsrc(T16, (uint64_t)P * d.t16_cols * 2u);
    for (int32_t c8 = tid * 8; c8 < ncell; c8 += kNormThreads * 8) {
        double S[8];
        uint32_t N[4];  // packed u16 pairs
#pragma unroll
        for (int k = 0; k < 8; ++k) S[k] = 0.0;
#pragma unroll
        for (int k = 0; k < 4; ++k) N[k] = 0u;
        const uint32_t vc = (uint32_t)(cofs * 4u + (uint64_t)c8 * 2u);  // byte offset in a protein's slab
        const uint32_t vt = (uint32_t)(rw.base0 + c8) * 2u;
        for (int p0 = 0; p0 < P; p0 += kNormUnroll) {
            uint4 cw[kNormUnroll], tw[kNormUnroll];
#pragma unroll
            for (int u = 0; u < kNormUnroll; ++u) {
                const bool in = p0 + u < P;
                const uint32_t pc = (uint32_t)min(p0 + u, P - 1);
                const rsrc_t r_c = mk_rsrc(cnt + (uint64_t)pc * pitch, pitch * 4u);  // one protein's slab (< 4 GiB)
                cw[u] = bld_u128(r_c, in ? vc : kOOB, 0u);
                tw[u] = bld_u128(r_t, in ? vt : kOOB, (uint32_t)(d.t16_cols * 2u * pc));
            }
#pragma unroll
            for (int u = 0; u < kNormUnroll; ++u) {
                if ((cw[u].x | cw[u].y | cw[u].z | cw[u].w) == 0u) continue;
                const int32_t ta = ta_lds[min(p0 + u, P - 1)];
                const uint32_t cv[4] = {cw[u].x, cw[u].y, cw[u].z, cw[u].w};
                const uint32_t tv[4] = {tw[u].x, tw[u].y, tw[u].z, tw[u].w};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    norm_cell(cv[k] & 0xFFFFu, tv[k] & 0xFFFFu, ta, S[2 * k], N[k], 1u);
                    norm_cell(cv[k] >> 16, tv[k] >> 16, ta, S[2 * k + 1], N[k], 1u << 16);
                }
            }
        }
        // epilogue: JAC S/N and AJI at the reference's JAC index
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int32_t b = rw.base0 + c8 + k;
            if (b < rw.clo || b >= rw.chi || !col_valid<MODE>(d, a, b)) continue;
            const int64_t idx = pair_index<MODE>(d, a, b, compat);
            double s = S[k];
            int32_t n = (int32_t)((N[k >> 1] >> (16 * (k & 1))) & 0xFFFFu);
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
