// pfaai_kernels.hpp -- gfx950 kernels of the all-pairs AJI hot path.
//
// The reference materialises E = every (protein, gA, gB) triple sharing a
// tetramer (ds_helper.hpp:270-357), comparison-sorts it by (gA, gB, p)
// (psort.hpp:27-53, 86 % of its wall time) and walks the sorted runs
// (algorithm_impl.hpp:123-277).  Here E is never built and nothing is sorted:
//
//   K-W  k_tetra_records  one workgroup per tetramer block of F: finds the
//        (tetramer, protein) runs with a wavefront ballot + prefix count,
//        then turns every F entry whose genome is an output row into
//        "member ranges" [lo, hi) of that run (the genomes it pairs with),
//        bucketed per (row, protein) by a counting sort (pass 0 counts,
//        exclusive scan, pass 1 fills).
//   K-S+J k_rows          one workgroup per output row (genome A): for each
//        protein in ascending order, scatters +1 into an LDS row of packed
//        u16 intersection counters for every member B of every range
//        (= the E triples (p, A, B) of that row), then normalises the row
//        J = c / (T[p][A] + T[p][B] - c) in fp64 into per-column register
//        accumulators S, N -- the exact protein-ordered sum of
//        algorithm_impl.hpp:240-275 -- and finally writes AJI = S / N
//        (algorithm_impl.hpp:318) at the reference's JAC index.
//
// Integer counts are exact (integer LDS atomics); fp64 sums are built in
// ascending protein order per pair, so results are bit-identical to the
// reference.  No fast-math: divisions are IEEE (v_div_scale/fmas/fixup).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pfaai {

constexpr int kNTetramers = 160000;
constexpr int kTetraThreads = 256;      // K-W workgroup
constexpr int kMaxRuns = 4096;          // proteins per tetramer block (checked at load)
constexpr int kRowThreads = 1024;       // K-S+J workgroup (16 waves)
constexpr int kGroup = 16;              // lanes per member range in the scatter
constexpr int kNumGroups = kRowThreads / kGroup;
constexpr uint32_t kRangeMax = 64;      // members per range (longer runs are split)
constexpr uint32_t kFilterBit = 0x80000000u;

// Device view of a loaded problem (pfaai_problem + derived maps).
struct Dev {
    int32_t mode, n_ids, n_prot, t_cols, n_qry, n_tgt;
    int64_t n_f;
    const int64_t* Lp;
    const int32_t* Fp;
    const int32_t* Fg;
    const int32_t* T;
    const uint8_t* is_q;
    const int32_t* q_index;
    const int32_t* t_rank;
    const int32_t* row_of;      // [n_ids] output row of a genome, -1 if none
    const int32_t* row_genome;  // [n_rows] genome id of an output row
    const int32_t* tcol_row;    // [n_ids] T column used when the genome is genomeA
    const int32_t* tcol_col;    // [n_ids] T column used when the genome is genomeB
};

// ---------------------------------------------------------------------------
// mode index maps (ds_impl.hpp:83-96, 251-276, 411-426)
// ---------------------------------------------------------------------------
template <int MODE>
__device__ __forceinline__ bool col_valid(const Dev& d, int32_t a, int32_t b) {
    if constexpr (MODE == 0) return b > a;
    else if constexpr (MODE == 1) return b != a && (!d.is_q[b] || b > a);
    else return b < d.n_tgt;
}

template <int MODE>
__device__ __forceinline__ int64_t pair_index(const Dev& d, int32_t a, int32_t b, bool compat) {
    if constexpr (MODE == 0) {
        return (int64_t)d.n_ids * a + b - (int64_t)(a + 2) * (a + 1) / 2;
    } else if constexpr (MODE == 1) {
        if (!d.is_q[b]) return (int64_t)d.q_index[a] * d.n_tgt + d.t_rank[b];
        int64_t gia = d.q_index[a], gib = d.q_index[b];
        if (!compat && gia > gib) { int64_t x = gia; gia = gib; gib = x; }
        return (int64_t)d.n_qry * d.n_tgt +
               ((int64_t)d.n_qry * gia + gib - (gia + 2) * (gia + 1) / 2);
    } else {
        return (int64_t)(a - d.n_tgt) * d.n_tgt + b;
    }
}

// Column window of a row in genome-id space: [lo, hi).
template <int MODE>
__device__ __forceinline__ void row_cols(const Dev& d, int32_t a, int32_t& lo, int32_t& hi) {
    if constexpr (MODE == 0) { lo = a + 1; hi = d.n_ids; }
    else if constexpr (MODE == 1) { lo = 0; hi = d.n_ids; }
    else { lo = 0; hi = d.n_tgt; }
}

// First position in Fg[lo, hi) whose genome id is >= key (Fg sorted there).
__device__ __forceinline__ int64_t lower_bound_g(const int32_t* Fg, int64_t lo, int64_t hi, int32_t key) {
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (Fg[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ uint32_t n_pieces(int64_t len) {
    return len <= 0 ? 0u : (uint32_t)((len + kRangeMax - 1) / kRangeMax);
}

// ---------------------------------------------------------------------------
// K-W: member-range work lists per (row, protein).
//   PASS 0: cnt[(row-row_begin)*P + p] += #ranges
//   PASS 1: recs[cursor[...]++] = {lo, hi | filter}
//   PASS 2: first_key = min over all events of (gA, gB, p)  (ref-compat row Z)
// ---------------------------------------------------------------------------
template <int MODE, int PASS>
__global__ __launch_bounds__(kTetraThreads) void k_tetra_records(
    Dev d, int64_t row_begin, int64_t row_end, uint32_t* __restrict__ cnt,
    unsigned long long* __restrict__ cursor, uint2* __restrict__ recs,
    unsigned long long* __restrict__ first_key, int* __restrict__ err) {
    __shared__ int32_t runs[kMaxRuns + 1];
    __shared__ int32_t wave_cnt[kTetraThreads / 64];
    __shared__ int32_t n_runs;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int P = d.n_prot;

    for (int t = blockIdx.x; t < kNTetramers; t += gridDim.x) {
        const int64_t s = d.Lp[t], e = d.Lp[t + 1];
        if (s >= e) continue;  // uniform
        if (tid == 0) n_runs = 0;
        __syncthreads();
        // (t, p) run heads, compacted in order: ballot per wave + wave prefix.
        for (int64_t base = s; base < e; base += kTetraThreads) {
            const int64_t i = base + tid;
            bool head = false;
            if (i < e) head = (i == s) || (d.Fp[i] != d.Fp[i - 1]);
            const unsigned long long m = __ballot(head);
            if (lane == 0) wave_cnt[wid] = __popcll(m);
            __syncthreads();
            int off = n_runs;
            for (int w = 0; w < wid; ++w) off += wave_cnt[w];
            if (head) {
                const int pos = off + __popcll(m & ((1ull << lane) - 1ull));
                if (pos < kMaxRuns) runs[pos] = (int32_t)(i - s);
                else atomicOr(err, 1);
            }
            __syncthreads();
            if (tid == 0) {
                int add = 0;
                for (int w = 0; w < kTetraThreads / 64; ++w) add += wave_cnt[w];
                n_runs += add;
            }
            __syncthreads();
        }
        const int nr = min(n_runs, kMaxRuns);
        if (tid == 0) runs[nr] = (int32_t)(e - s);
        __syncthreads();

        for (int64_t i = s + tid; i < e; i += kTetraThreads) {
            const int32_t a = d.Fg[i];
            const int32_t row = d.row_of[a];
            if (row < 0) continue;
            if (PASS != 2 && (row < row_begin || row >= row_end)) continue;
            // run containing i: last head <= i - s
            const int32_t rel = (int32_t)(i - s);
            int lo = 0, hi = nr;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (runs[mid] <= rel) lo = mid + 1; else hi = mid;
            }
            const int64_t bs = s + runs[lo - 1], be = s + runs[lo];
            const int32_t p = d.Fp[i];
            // member ranges of this entry (the valid partners in its run)
            int64_t r0lo = 0, r0hi = 0, r1lo = 0, r1hi = 0;  // r0 may carry the filter bit
            if constexpr (MODE == 0) {
                r1lo = i + 1; r1hi = be;
            } else if constexpr (MODE == 1) {
                r0lo = bs; r0hi = i;      // members before a: valid iff non-query
                r1lo = i + 1; r1hi = be;  // members after a: always valid
            } else {
                r0lo = bs; r0hi = lower_bound_g(d.Fg, bs, be, d.n_tgt);  // targets
            }
            if constexpr (PASS == 0) {
                const uint32_t np = n_pieces(r0hi - r0lo) + n_pieces(r1hi - r1lo);
                if (np) atomicAdd(&cnt[(int64_t)(row - row_begin) * P + p], np);
            } else if constexpr (PASS == 1) {
                const uint32_t n0 = n_pieces(r0hi - r0lo), n1 = n_pieces(r1hi - r1lo);
                if (n0 + n1 == 0) continue;
                unsigned long long k =
                    atomicAdd(&cursor[(int64_t)(row - row_begin) * P + p], (unsigned long long)(n0 + n1));
                const uint32_t f0 = (MODE == 1) ? kFilterBit : 0u;
                for (int64_t x = r0lo; x < r0hi; x += kRangeMax, ++k)
                    recs[k] = make_uint2((uint32_t)x, (uint32_t)min(r0hi, x + (int64_t)kRangeMax) | f0);
                for (int64_t x = r1lo; x < r1hi; x += kRangeMax, ++k)
                    recs[k] = make_uint2((uint32_t)x, (uint32_t)min(r1hi, x + (int64_t)kRangeMax));
            } else {
                // smallest valid partner of a in this run
                int32_t b = -1;
                if constexpr (MODE == 0) {
                    if (i + 1 < be) b = d.Fg[i + 1];
                } else if constexpr (MODE == 2) {
                    if (r0hi > r0lo) b = d.Fg[r0lo];
                } else {
                    for (int64_t j = bs; j < be; ++j) {
                        const int32_t g = d.Fg[j];
                        if (j != i && (!d.is_q[g] || g > a)) { b = g; break; }
                    }
                }
                if (b >= 0) {
                    const unsigned long long key = ((unsigned long long)a << 42) |
                                                   ((unsigned long long)b << 21) |
                                                   (unsigned long long)p;
                    atomicMin(first_key, key);
                }
            }
        }
        __syncthreads();  // runs[] is reused by the next tetramer
    }
}

// ---------------------------------------------------------------------------
// exclusive scan u32 -> u64 (rowptr), three phases
// ---------------------------------------------------------------------------
constexpr int kScanThreads = 256;
constexpr int kScanItems = 4;
constexpr int kScanTile = kScanThreads * kScanItems;

__device__ __forceinline__ unsigned long long wave_incl_scan(unsigned long long v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long u = __shfl_up(v, o, 64);
        if (lane >= o) v += u;
    }
    return v;
}

// Block-wide exclusive scan of one value per thread; returns the total too.
__device__ __forceinline__ unsigned long long block_excl_scan(unsigned long long v,
                                                              unsigned long long& total) {
    __shared__ unsigned long long wsum[kScanThreads / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const unsigned long long inc = wave_incl_scan(v);
    if (lane == 63) wsum[wid] = inc;
    __syncthreads();
    unsigned long long off = 0, tot = 0;
    for (int w = 0; w < kScanThreads / 64; ++w) {
        if (w < wid) off += wsum[w];
        tot += wsum[w];
    }
    __syncthreads();
    total = tot;
    return off + inc - v;
}

__global__ __launch_bounds__(kScanThreads) void k_scan_tiles(const uint32_t* __restrict__ in, int64_t n,
                                                             unsigned long long* __restrict__ out,
                                                             unsigned long long* __restrict__ sums) {
    const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
    unsigned long long v[kScanItems], acc = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        v[k] = (base + k < n) ? in[base + k] : 0u;
        acc += v[k];
    }
    unsigned long long total;
    unsigned long long off = block_excl_scan(acc, total);
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        if (base + k < n) out[base + k] = off;
        off += v[k];
    }
    if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

__global__ __launch_bounds__(kScanThreads) void k_scan_sums(unsigned long long* __restrict__ sums, int64_t n,
                                                            unsigned long long* __restrict__ grand) {
    unsigned long long carry = 0;
    for (int64_t base = 0; base < n; base += kScanThreads) {
        const int64_t i = base + threadIdx.x;
        const unsigned long long v = i < n ? sums[i] : 0ull;
        unsigned long long total;
        const unsigned long long ex = block_excl_scan(v, total);
        if (i < n) sums[i] = carry + ex;
        carry += total;
    }
    if (threadIdx.x == 0) *grand = carry;
}

__global__ __launch_bounds__(kScanThreads) void k_scan_add(unsigned long long* __restrict__ out, int64_t n,
                                                           const unsigned long long* __restrict__ sums,
                                                           const unsigned long long* __restrict__ grand,
                                                           unsigned long long* __restrict__ cursor) {
    const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
    const unsigned long long add = sums[blockIdx.x];
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const int64_t i = base + k;
        if (i < n) {
            const unsigned long long v = out[i] + add;
            out[i] = v;
            if (cursor) cursor[i] = v;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        out[n] = *grand;
        if (cursor) cursor[n] = *grand;
    }
}

// ---------------------------------------------------------------------------
// K-S: scatter the E triples (p, A, *) of one row and protein into LDS
// counters.  acc word w holds columns cc0+2w (low u16) and cc0+2w+1 (high).
// Each 16-lane group walks one member range (<= 64 genome ids, contiguous in
// F, so each group load is one 64-B segment).
// ---------------------------------------------------------------------------
template <int MODE>
__device__ __forceinline__ uint32_t scatter_row_protein(const Dev& d, const uint2* __restrict__ recs,
                                                        uint64_t rb, uint64_t re, uint32_t* acc,
                                                        int32_t cc0, int32_t cc1) {
    const int tid = threadIdx.x;
    const int grp = tid / kGroup, gl = tid % kGroup;
    uint32_t ev = 0;
    for (uint64_t k = rb + grp; k < re; k += kNumGroups) {
        const uint2 r = recs[k];
        const uint32_t lo = r.x, hi = r.y & ~kFilterBit;
        const bool filt = (MODE == 1) && (r.y & kFilterBit);
        for (uint32_t m = lo + gl; m < hi; m += kGroup) {
            const int32_t b = d.Fg[m];
            if (MODE == 1 && filt && d.is_q[b]) continue;
            if (b >= cc0 && b < cc1) {
                const uint32_t o = (uint32_t)(b - cc0);
                atomicAdd(&acc[o >> 1], 1u << ((o & 1u) << 4));
                ++ev;
            }
        }
    }
    return ev;
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// ---------------------------------------------------------------------------
// K-S+J: one workgroup per (output row, column chunk).  Thread t owns the
// counter words w = t + k*1024 (k < KW), i.e. columns cc0+2w, cc0+2w+1, and
// keeps their S (fp64) and N (packed u16) in registers across all proteins.
// ---------------------------------------------------------------------------
template <int MODE, int KW>
__global__ __launch_bounds__(kRowThreads) void k_rows(
    Dev d, int64_t row_begin, const unsigned long long* __restrict__ rowptr,
    const uint2* __restrict__ recs, int32_t chunk_cols, uint32_t flags,
    const unsigned long long* __restrict__ first_key, double* __restrict__ aji, double* __restrict__ s_out, int32_t* __restrict__ n_out,
    unsigned long long* __restrict__ n_events) {
    extern __shared__ uint32_t acc[];
    const int tid = threadIdx.x;
    const int64_t rl = blockIdx.x;  // local row
    const int32_t a = d.row_genome[row_begin + rl];
    int32_t clo, chi;
    row_cols<MODE>(d, a, clo, chi);
    const int32_t cc0 = clo + (int32_t)blockIdx.y * chunk_cols;
    const int32_t cc1 = min(chi, cc0 + chunk_cols);
    if (cc0 >= cc1) return;  // uniform
    const int32_t ncw = (cc1 - cc0 + 1) >> 1;
    const bool compat = flags & 1u;
    const int P = d.n_prot;

    for (int w = tid; w < ncw; w += kRowThreads) acc[w] = 0u;
    double S[2 * KW];
    uint32_t N[KW];
#pragma unroll
    for (int k = 0; k < KW; ++k) { S[2 * k] = 0.0; S[2 * k + 1] = 0.0; N[k] = 0u; }
    const int32_t tca = compat ? d.tcol_row[a] : a;  // T column of genomeA (row Q quirk only in compat)
    uint32_t ev = 0;
    __syncthreads();

    for (int p = 0; p < P; ++p) {
        const uint64_t rb = rowptr[rl * P + p], re = rowptr[rl * P + p + 1];
        if (rb == re) continue;  // uniform: no E triple (p, a, *)
        ev += scatter_row_protein<MODE>(d, recs, rb, re, acc, cc0, cc1);
        __syncthreads();
        const int32_t* Tp = d.T + (int64_t)p * d.t_cols;
        const int32_t ta = Tp[tca];
#pragma unroll
        for (int k = 0; k < KW; ++k) {
            const int32_t w = tid + k * kRowThreads;
            if (w < ncw) {
                const uint32_t v = acc[w];
                if (v) {
                    acc[w] = 0u;
                    const int32_t c0 = (int32_t)(v & 0xFFFFu), c1 = (int32_t)(v >> 16);
                    const int32_t b0 = cc0 + 2 * w;
                    if (c0) {
                        const int32_t tb = Tp[compat ? d.tcol_col[b0] : b0];
                        S[2 * k] += (double)c0 / (double)(ta + tb - c0);
                        N[k] += 1u;
                    }
                    if (c1) {
                        const int32_t tb = Tp[compat ? d.tcol_col[b0 + 1] : b0 + 1];
                        S[2 * k + 1] += (double)c1 / (double)(ta + tb - c1);
                        N[k] += 1u << 16;
                    }
                }
            }
        }
        __syncthreads();
    }

    // |E| of this row chunk
    ev = wave_sum_u32(ev);
    if ((tid & 63) == 0 && ev) atomicAdd(n_events, (unsigned long long)ev);

    // epilogue: write JAC S/N and AJI at the reference's JAC index
#pragma unroll
    for (int k = 0; k < KW; ++k) {
        const int32_t w = tid + k * kRowThreads;
        if (w >= ncw) continue;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int32_t b = cc0 + 2 * w + h;
            if (b >= cc1 || !col_valid<MODE>(d, a, b)) continue;
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

// Debug: dump the per-protein counts of one row (integer parity vs E).
template <int MODE>
__global__ __launch_bounds__(kRowThreads) void k_row_counts(
    Dev d, int64_t row_begin, const unsigned long long* __restrict__ rowptr,
    const uint2* __restrict__ recs, int32_t chunk_cols, int32_t* __restrict__ counts) {
    extern __shared__ uint32_t acc[];
    const int tid = threadIdx.x;
    const int32_t a = d.row_genome[row_begin];
    int32_t clo, chi;
    row_cols<MODE>(d, a, clo, chi);
    const int32_t cc0 = clo + (int32_t)blockIdx.y * chunk_cols;
    const int32_t cc1 = min(chi, cc0 + chunk_cols);
    if (cc0 >= cc1) return;
    const int32_t ncw = (cc1 - cc0 + 1) >> 1;
    for (int w = tid; w < ncw; w += kRowThreads) acc[w] = 0u;
    __syncthreads();
    for (int p = 0; p < d.n_prot; ++p) {
        const uint64_t rb = rowptr[p], re = rowptr[p + 1];
        scatter_row_protein<MODE>(d, recs, rb, re, acc, cc0, cc1);
        __syncthreads();
        for (int w = tid; w < ncw; w += kRowThreads) {
            const uint32_t v = acc[w];
            const int32_t b0 = cc0 + 2 * w;
            counts[(int64_t)p * d.n_ids + b0] = (int32_t)(v & 0xFFFFu);
            if (b0 + 1 < cc1) counts[(int64_t)p * d.n_ids + b0 + 1] = (int32_t)(v >> 16);
            acc[w] = 0u;
        }
        __syncthreads();
    }
}

}  // namespace pfaai
