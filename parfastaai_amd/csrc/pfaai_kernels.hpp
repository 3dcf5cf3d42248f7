// pfaai_kernels.hpp -- gfx950 kernels of the all-pairs AJI hot path.
//
// The reference materialises E = every (protein, gA, gB) triple sharing a
// tetramer (ds_helper.hpp:270-357), comparison-sorts it by (gA, gB, p)
// (psort.hpp:27-53, 86 % of its wall time) and walks the sorted runs
// (algorithm_impl.hpp:123-277).  Here E is never built and nothing is sorted:
//
//   K-W   k_blk (genome-major input): the run table, (protein, tetramer) ->
//         run of F; the row kernels walk each row genome's own G entries.
//         F-only input: k_entries + k_rs_* + k_rowptr -- one workgroup per
//         tetramer block of F finds the (tetramer, protein) runs with a
//         wavefront ballot + prefix count and turns every F entry whose
//         genome is an output row into a "member range" [lo, hi) of its run,
//         keyed by (row, protein); a hand-written stable LSD radix sort
//         groups them per (row, protein) and rowptr marks the groups.
//   K-S+J k_rows_pl (pfaai_rows_pl.hpp, the default) and k_rows (here: the
//         fallback for very long G lists, and the F-only form): one
//         workgroup per output row (genome A); for each protein in ascending
//         order, scatter +1 into an LDS row of packed u16 intersection
//         counters for every member B of every run holding A (= the E
//         triples (p, A, B) of that row), then normalise the row
//         J = c / (T[p][A] + T[p][B] - c) in fp64 into per-column register
//         accumulators S, N -- the exact protein-ordered sum of
//         algorithm_impl.hpp:240-275 -- and finally write AJI = S / N
//         (algorithm_impl.hpp:318) at the reference's JAC index.
//
// Integer counts are exact (integer LDS atomics); fp64 sums are built in
// ascending protein order per pair, so results are bit-identical to the
// reference.  No fast-math: divisions are IEEE (or the bit-identical
// exact_div_small of pfaai_util.hpp).
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
constexpr int kSplitters = 3, kSplitBits = 21;  // run-line splitters in blk (genome ids < 2^21)
constexpr uint64_t kSplitNone = (1ull << kSplitBits) - 1;

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
    const int64_t* G_off;       // [n_ids * n_prot + 1] genome-major CSR (optional)
    const int32_t* G_tet;
    const uint2* G_pe;          // [|G|] (F index, end of its F run) of each G entry: the all-vs-all
                                // walk data (G_pos, G_end interleaved; nullptr if not built)
    const uint32_t* Fcode;      // [|F| + 16] member codes of F for the WK 3 walks (k_fcode), or nullptr
    uint4* blk;                 // [n_prot * 160000] (protein, tetramer) -> F run, see k_blk
    const uint16_t* Fp16;       // [|F|] protein of each F entry, u16 (k_blk)
    const uint16_t* T16;        // [n_prot][t16_cols] T by column genome id, u16 (k_rows_pl)
    const uint16_t* T16c;       // same through tcol_col (ref-compat QT quirk); == T16 otherwise
    int64_t t16_cols;           // even, >= n_ids
    int32_t xcd_chunk;          // consecutive rows per XCD in xcd_row (PFAAI_XCD_CHUNK, default kXcdChunk)
};

// XCD-aware row order (MI355X_MICROARCH.md: workgroups are dealt round-robin
// over the 8 XCDs, each with a private 4 MiB L2).  Consecutive rows -- in
// practice genomes of one clade, which read the same F blocks -- should share
// an L2: workgroup b (on XCD b % 8) takes row chunk (b/8 / C) * 8 + b % 8,
// i.e. XCD x walks chunks x, x+8, ... of C consecutive rows.  A bijection on
// [0, n); the tail that does not fill 8 chunks keeps the identity.  Speed
// only -- any order is correct.
constexpr int kXcds = 8;
constexpr int kXcdChunk = 32;

__device__ __forceinline__ int64_t xcd_row(int64_t b, int64_t n, int64_t ch = kXcdChunk) {
    const int64_t full = (n / (kXcds * ch)) * (kXcds * ch);
    if (b >= full) return b;
    const int64_t x = b % kXcds, i = b / kXcds;
    return (i / ch) * (kXcds * ch) + x * ch + (i % ch);
}

// ---------------------------------------------------------------------------
// mode index maps (ds_impl.hpp:83-96, 251-276, 411-426)
// ---------------------------------------------------------------------------
// MODE 3 (kModeFull) is not a reference mode: the full output row of
// printOutput's dense matrix (main.cpp:143-154) for an all-vs-all or query-
// subset row genome A -- every column B != A, the mirror half included,
// written at row(A) * n_ids + B (pfaai_stream_matrix).  AJI(A, B) and
// AJI(B, A) are bit-identical (the same counts, denominators and protein
// order), so the mirror half equals the reference's mirrored copy.
constexpr int kModeFull = 3;

template <int MODE>
__device__ __forceinline__ bool col_valid(const Dev& d, int32_t a, int32_t b) {
    if constexpr (MODE == 0) return b > a;
    else if constexpr (MODE == 1) return b != a && (!d.is_q[b] || b > a);
    else if constexpr (MODE == kModeFull) return b != a;
    else return b < d.n_tgt;
}

template <int MODE>
__device__ __forceinline__ int64_t pair_index(const Dev& d, int32_t a, int32_t b, bool compat) {
    if constexpr (MODE == 0) {
        return (int64_t)d.n_ids * a + b - (int64_t)(a + 2) * (a + 1) / 2;
    } else if constexpr (MODE == kModeFull) {
        return (int64_t)d.row_of[a] * d.n_ids + b;
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

// Output of one counter word: columns b0 and b0 + 1 of row a (ok[h]: column
// b0 + h is in the row's window and valid) with their S and N.  Outside the
// QSUB mode (1) the two columns are consecutive output indices, so a lane
// writes both with one 16-B store and a wave's stores cover whole lines; two
// 8-B stores per lane wrote every line twice, half-masked (0.79 GB of
// WRITE_SIZE for 0.40 GB of AJI at 10k all-vs-all, 7.58 -> 7.45 ms per step,
// profiles/r03y); non-temporal AJI stores on top made no difference (7.441
// vs 7.445 ms, profiles/r03z/ab_nt_aji_store.txt).  The paired types are
// element-aligned: a row's first output index has either parity.
typedef double f64x2_a8 __attribute__((ext_vector_type(2), aligned(8)));
typedef int32_t i32x2_a4 __attribute__((ext_vector_type(2), aligned(4)));

template <int MODE>
__device__ __forceinline__ void put_pair(const Dev& d, int32_t a, int32_t b0, const bool ok[2], const double sv[2],
                                         const int32_t nv[2], bool compat, double* __restrict__ aji,
                                         double* __restrict__ s_out, int32_t* __restrict__ n_out) {
    if constexpr (MODE != 1) {
        const int64_t idx = pair_index<MODE>(d, a, b0, compat);
        const double o0 = nv[0] ? sv[0] / (double)nv[0] : 0.0;
        const double o1 = nv[1] ? sv[1] / (double)nv[1] : 0.0;
        if (ok[0] && ok[1]) {
            if (aji) *reinterpret_cast<f64x2_a8*>(aji + idx) = f64x2_a8{o0, o1};
            if (s_out) *reinterpret_cast<f64x2_a8*>(s_out + idx) = f64x2_a8{sv[0], sv[1]};
            if (n_out) *reinterpret_cast<i32x2_a4*>(n_out + idx) = i32x2_a4{nv[0], nv[1]};
        } else {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                if (!ok[h]) continue;
                if (aji) aji[idx + h] = h ? o1 : o0;
                if (s_out) s_out[idx + h] = sv[h];
                if (n_out) n_out[idx + h] = nv[h];
            }
        }
    } else {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (!ok[h]) continue;
            const int64_t idx = pair_index<MODE>(d, a, b0 + h, compat);
            if (aji) aji[idx] = nv[h] ? sv[h] / (double)nv[h] : 0.0;
            if (s_out) s_out[idx] = sv[h];
            if (n_out) n_out[idx] = nv[h];
        }
    }
}

// Column window of a row in genome-id space: [lo, hi).
template <int MODE>
__device__ __forceinline__ void row_cols(const Dev& d, int32_t a, int32_t& lo, int32_t& hi) {
    if constexpr (MODE == 0) { lo = a + 1; hi = d.n_ids; }
    else if constexpr (MODE == 1 || MODE == kModeFull) { lo = 0; hi = d.n_ids; }
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

// ---------------------------------------------------------------------------
// K-W1: work-list entries.  One workgroup per tetramer block of F: the
// (tetramer, protein) run heads are found with a wavefront ballot + prefix
// count and kept in LDS; every F entry whose genome is an output row in
// [row_begin, row_end) becomes one entry
//      key = (row - row_begin) * P + protein,  rec = member range [lo, hi)
//   ALL  : [i+1, run end)              -- partners B > A (ds_impl.hpp:90-92)
//   QSUB : [run start, run end)        -- filtered per member at scatter time
//   QT   : [run start, first query)    -- target partners (ds_impl.hpp:421-423)
// compacted with one global atomic per 256 entries.  FIRST also finds the
// lexicographically first E triple (gA, gB, p) over all rows (ref-compat row
// Z).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wave_sum_u32_fwd(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <int MODE, bool FIRST>
__global__ __launch_bounds__(kTetraThreads) void k_entries(
    Dev d, int64_t row_begin, int64_t row_end, uint32_t* __restrict__ key_c, uint2* __restrict__ rec_c,
    const unsigned long long* __restrict__ off_t, unsigned long long* __restrict__ first_key, int* __restrict__ err) {
    __shared__ int32_t runs[kMaxRuns + 1];
    __shared__ int32_t wave_cnt[kTetraThreads / 64];
    __shared__ int32_t n_runs;
    __shared__ unsigned long long chunk_base;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int P = d.n_prot;
    const unsigned long long lt = (1ull << lane) - 1ull;

    for (int t = blockIdx.x; t < kNTetramers; t += gridDim.x) {
        const int64_t s = d.Lp[t], e = d.Lp[t + 1];
        if (s >= e) continue;  // uniform
        if (tid == 0) n_runs = 0;
        __syncthreads();
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
                const int pos = off + __popcll(m & lt);
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
        if (tid == 0) {
            runs[nr] = (int32_t)(e - s);
            chunk_base = off_t ? off_t[t] : 0ull;
        }
        __syncthreads();

        for (int64_t base = s; base < e; base += kTetraThreads) {  // uniform trip count
            const int64_t i = base + tid;
            bool valid = false;
            uint32_t key = 0;
            uint2 rec = make_uint2(0u, 0u);
            unsigned long long fk = ~0ull;  // FIRST: this lane's candidate
            if (i < e) {
                const int32_t a = d.Fg[i];
                const int32_t row = d.row_of[a];
                if (row >= 0) {
                    const int32_t rel = (int32_t)(i - s);
                    int lo = 0, hi = nr;
                    while (lo < hi) {
                        const int mid = (lo + hi) >> 1;
                        if (runs[mid] <= rel) lo = mid + 1; else hi = mid;
                    }
                    const int64_t bs = s + runs[lo - 1], be = s + runs[lo];
                    const int32_t p = d.Fp[i];
                    int64_t rlo, rhi;
                    if constexpr (MODE == 0) { rlo = i + 1; rhi = be; }
                    else if constexpr (MODE == 1) { rlo = bs; rhi = be; }
                    else { rlo = bs; rhi = lower_bound_g(d.Fg, bs, be, d.n_tgt); }
                    rec = make_uint2((uint32_t)rlo, (uint32_t)rhi);
                    if (row >= row_begin && row < row_end) {
                        valid = true;
                        key = (uint32_t)((row - row_begin) * P + p);
                    }
                    if constexpr (FIRST) {  // smallest valid partner of A in this run
                        int32_t b = -1;
                        if constexpr (MODE == 0) {
                            if (i + 1 < be) b = d.Fg[i + 1];
                        } else if constexpr (MODE == 2) {
                            if (rhi > rlo) b = d.Fg[rlo];
                        } else {
                            for (int64_t j = bs; j < be; ++j) {
                                const int32_t g = d.Fg[j];
                                if (j != i && (!d.is_q[g] || g > a)) { b = g; break; }
                            }
                        }
                        if (b >= 0)
                            fk = ((unsigned long long)a << 42) | ((unsigned long long)b << 21) | (unsigned long long)p;
                    }
                }
            }
            if constexpr (FIRST) {
                // one atomic per wave, and only if it lowers the minimum: an
                // atomicMin per F entry on the one address serialised at the
                // L2 (C2's 5.8e7 entries: 11 ms inside the CLI's compat run)
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) {
                    const unsigned long long v = __shfl_xor(fk, o, 64);
                    fk = v < fk ? v : fk;
                }
                if (lane == 0 && fk != ~0ull && fk < __hip_atomic_load(first_key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                    atomicMin(first_key, fk);
            }
            // compaction at this tetramer's offset (per-tetramer counts, scanned)
            const unsigned long long m = __ballot(valid);
            if (lane == 0) wave_cnt[wid] = __popcll(m);
            __syncthreads();
            if (valid && key_c) {
                unsigned long long off = chunk_base + __popcll(m & lt);
                for (int w = 0; w < wid; ++w) off += wave_cnt[w];
                key_c[off] = key;
                rec_c[off] = rec;
            }
            __syncthreads();
            if (tid == 0) {
                int tot = 0;
                for (int w = 0; w < kTetraThreads / 64; ++w) tot += wave_cnt[w];
                chunk_base += tot;
            }
            __syncthreads();
        }
    }
}

// ---------------------------------------------------------------------------
// K-W1g (genome-major input): the run table.
//   k_blk:    blk[p * 160000 + t] = {start, end, splitters} of run (t, p) in
//             F, one workgroup per tile of 16 tetramers: (1) run heads and
//             tails where the protein id changes (16-B loads of u16 ids,
//             neighbours by DPP wave shifts), (2) the splitters -- genome ids
//             at the run's 64-B line boundaries 1..3 (21 bits each), which
//             let a row skip whole lines outside its column window -- from
//             one streamed id per line, (3) the tile's entries written
//             densely (no memset pass).  p-major keeps the rows' lookups of
//             one protein within 2.56 MB (t-major was 15 % slower in the row
//             kernel).  0.64 ms at 10k (was 0.96 ms).  The row kernels then
//             walk each row genome's own G entries (A, p, t): the runs
//             holding A, i.e. its E triples (ds_helper.hpp:270-357).
// ---------------------------------------------------------------------------
constexpr int kBlkTileMax = 16;        // tetramers per k_blk workgroup (fewer for many proteins)
constexpr int kBlkLdsBytes = 80 << 10;  // LDS per workgroup (two workgroups share a CU's 160 KB)
// k_blk's dynamic staging (n_prot x tile x 16 B) gets what its static LDS
// (lp[]) leaves of kBlkLdsBytes, so two workgroups still fit a CU at any P
constexpr int kBlkDynLds = kBlkLdsBytes - 256;

// dbg: bit 0 skips (1), bit 1 (2), bit 2 (3) -- PFAAI_BLK_ABLATE (diagnostics) and, for
// query-vs-target window tables, bit 1 (no splitters: nothing there prunes by them).
// WIN (column windows for rows wider than one row-kernel chunk): one table
// per absolute column window w = [w * wcols, (w + 1) * wcols), all built in
// this one pass over F, window-major at blk + w * P * 160000 -- each entry is
// the sub-run of the run's members in window w (contiguous: a run is sorted
// by genome), so a row-kernel launch over window w loads only the lines of
// that window, and all its workgroups work on the same 1/nwin of F (L2 / MALL
// locality).  The LDS staging then holds nwin tables (fewer tetramers per tile).
// Ids >= gmax belong to no window (query vs target: gmax = n_tgt, so a window's
// sub-run holds targets only -- every member a partner of a query row, the
// row kernel's WK 4 span -- and no id can index past the nwin tables).
__device__ __forceinline__ int32_t win_of(int32_t g, int32_t wcols, float inv) {
    int32_t w = (int32_t)((float)g * inv);  // g < 2^21: off by at most one, fixed below
    if (w * wcols > g) --w;
    if ((w + 1) * wcols <= g) ++w;
    return w;
}

template <bool WIN = false, int NTH = kTetraThreads>
__global__ __launch_bounds__(NTH) void k_blk(Dev d, int kBlkTile, int dbg, int32_t wcols = 0,
                                                       int32_t nwin = 1, int32_t gmax = 0x7FFFFFFF) {
    // [nwin][kBlkTile][n_prot]: tetramer-major in LDS, so the heads / tails of
    // one tetramer's runs (consecutive proteins) land in different banks
    extern __shared__ uint4 ent[];
    __shared__ int64_t lp[kBlkTileMax + 1];
    const int tid = threadIdx.x, P = d.n_prot;
    const int t0 = blockIdx.x * kBlkTile;
    const int nt = min(kBlkTile, kNTetramers - t0);
    const float inv = WIN ? 1.0f / (float)wcols : 0.0f;
    const int PW = P * kBlkTile;  // entries per window
    // splitter fields start all-ones (kSplitNone); present ones are ANDed in
    for (int k = tid; k < (WIN ? nwin : 1) * PW; k += NTH) ent[k] = make_uint4(0u, 0u, 0xFFFFFFFFu, 0x7FFFFFFFu);
    if (tid <= nt) lp[tid] = d.Lp[t0 + tid];
    __syncthreads();
    const int64_t S = lp[0], E = lp[nt];
    auto tet_of = [&](int64_t i) {  // tetramer of F entry i within the tile: last tl with lp[tl] <= i
        int lo = 0, hi = nt - 1;       // binary search over <= 16 block starts (was a linear scan)
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (lp[mid] <= i) lo = mid; else hi = mid - 1;
        }
        return lo;
    };
    // (1) F is sorted by (tetramer, protein, genome): a run starts where the
    // protein changes and ends where it changes again -- each protein has one
    // run per tetramer, so heads and tails land in slots of their own.  Each
    // lane reads 8 consecutive u16 protein ids (one 16-B load); the ids just
    // before and after its chunk come from the neighbouring lanes (DPP wave
    // shifts) or, at wave edges, from one extra load.
    const int lane = tid & 63;
    for (int64_t c0 = (S & ~(int64_t)7) + (int64_t)tid * 8; c0 - (int64_t)lane * 8 < E && !(dbg & 1);
         c0 += (int64_t)NTH * 8) {  // wave-uniform trip count (DPP needs the whole wave)
        const bool in = c0 < E;
        const uint4 v = in ? *reinterpret_cast<const uint4*>(d.Fp16 + c0) : make_uint4(0u, 0u, 0u, 0u);
        uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(v.w >> 16), 0x138, 0xf, 0xf, false);  // wave_shr:1
        uint32_t next = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(v.x & 0xFFFFu), 0x130, 0xf, 0xf, false);  // wave_shl:1
        if (lane == 0) prev = c0 > S && in ? d.Fp16[c0 - 1] : 0xFFFFu;
        if (lane == 63) next = c0 + 8 < E ? d.Fp16[c0 + 8] : 0xFFFFu;
        // WIN: the 8 genome ids too (Fg carries 16 padding entries), neighbours likewise
        int32_t gg[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        int32_t gprev = 0, gnext = 0;
        if constexpr (WIN) {
            const uint4 ga = in ? *reinterpret_cast<const uint4*>(d.Fg + c0) : make_uint4(0u, 0u, 0u, 0u);
            const uint4 gb = in ? *reinterpret_cast<const uint4*>(d.Fg + c0 + 4) : make_uint4(0u, 0u, 0u, 0u);
            gg[0] = (int32_t)ga.x; gg[1] = (int32_t)ga.y; gg[2] = (int32_t)ga.z; gg[3] = (int32_t)ga.w;
            gg[4] = (int32_t)gb.x; gg[5] = (int32_t)gb.y; gg[6] = (int32_t)gb.z; gg[7] = (int32_t)gb.w;
            gprev = __builtin_amdgcn_update_dpp(0, (int)gb.w, 0x138, 0xf, 0xf, false);  // wave_shr:1
            gnext = __builtin_amdgcn_update_dpp(0, (int)ga.x, 0x130, 0xf, 0xf, false);  // wave_shl:1
            if (lane == 0) gprev = c0 > S && in ? d.Fg[c0 - 1] : -1;
            if (lane == 63) gnext = c0 + 8 < E ? d.Fg[c0 + 8] : 0x7FFFFFFF;
        }
        if (!in) continue;
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        int tl = tet_of(max(c0, S));
        int64_t cur = lp[tl], nb = lp[tl + 1];  // block [cur, nb) of tetramer tl, kept in registers
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int64_t i = c0 + j;
            const uint32_t q = (w[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
            const uint32_t qp = j == 0 ? prev : (w[(j - 1) >> 1] >> (16 * ((j - 1) & 1))) & 0xFFFFu;
            const uint32_t qn = j == 7 ? next : (w[(j + 1) >> 1] >> (16 * ((j + 1) & 1))) & 0xFFFFu;
            if (i < S || i >= E) continue;
            if (i >= nb) {  // crossed into a later tetramer block (rare: blocks hold ~1800 entries)
                while (tl + 1 < nt && lp[tl + 1] <= i) ++tl;
                cur = lp[tl];
                nb = lp[tl + 1];
            }
            bool head = i == cur || qp != q, tail = i + 1 == nb || qn != q;
            int wo = 0;  // window table offset
            if constexpr (WIN) {  // sub-runs by window: ids ascend along a run
                const int32_t g = gg[j], gp = j == 0 ? gprev : gg[j - 1], gn = j == 7 ? gnext : gg[j + 1];
                if (g >= gmax) continue;  // in no window (query-vs-target: the queries)
                const int32_t w = win_of(g, wcols, inv);
                head = head || gp < w * wcols;
                tail = tail || gn >= min((w + 1) * wcols, gmax);
                wo = w * PW;
            }
            if (head) ent[wo + tl * P + q].x = (uint32_t)i;
            if (tail) ent[wo + tl * P + q].y = (uint32_t)(i + 1);
        }
    }
    __syncthreads();
    constexpr int U = 8;
    // (2) run-line splitters: the genome id at the start of lines 1..3 of
    // every run.  Line starts are the 16-aligned F positions, so the tile's
    // share of Fg is streamed once, one id per 64-B line, instead of being
    // gathered run by run.
    for (int64_t i0 = ((S + kGroup - 1) & ~(int64_t)(kGroup - 1)) + (int64_t)tid * kGroup; i0 < E && !(dbg & 2);
         i0 += (int64_t)U * NTH * kGroup) {
        uint32_t g[U], q[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + (int64_t)u * NTH * kGroup;
            g[u] = i < E ? (uint32_t)d.Fg[i] : 0u;
            q[u] = i < E ? d.Fp16[i] : 0u;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + (int64_t)u * NTH * kGroup;
            if (i >= E || (WIN && (int32_t)g[u] >= gmax)) continue;
            uint4* r = &ent[(WIN ? win_of((int32_t)g[u], wcols, inv) * PW : 0) + tet_of(i) * P + q[u]];
            const uint32_t k = (uint32_t)(i - (r->x & ~(uint32_t)(kGroup - 1))) / kGroup;  // line of the run
            if (k < 1 || k > (uint32_t)kSplitters) continue;
            const uint64_t field = ~(kSplitNone << (kSplitBits * (k - 1))) | ((uint64_t)g[u] << (kSplitBits * (k - 1)));
            atomicAnd(&r->z, (uint32_t)field);
            atomicAnd(&r->w, (uint32_t)(field >> 32));
        }
    }
    __syncthreads();
    // (3) write out: consecutive entries of one protein (and window) per tile
    for (int k = tid; k < (WIN ? nwin : 1) * PW && !(dbg & 4); k += NTH) {
        const int tl = k % kBlkTile;
        const int wq = k / kBlkTile;  // w * P + q: global writes stay 16 consecutive tetramers of one protein
        if (tl < nt) d.blk[(int64_t)wq * kNTetramers + t0 + tl] = ent[(wq / P) * PW + tl * P + wq % P];
    }
}

// k_blk_end: the run-END table alone, ends[p * 160000 + t] = one past the
// last F entry of run (t, p), u32, p-major.  It is all k_rows_pl WK 3 reads
// (all-vs-all rows in one chunk with G_pos loaded: a run walk starts at the
// row genome's own F position + 1, so neither the run start nor the line
// splitters are needed): k_blk's phase (1) for tails only, staged as u32 in
// LDS for up to 64 tetramers per workgroup.  Reads 2 B per F entry (Fp16),
// writes 4 B per (protein, tetramer) slot -- a quarter of k_blk's table, and
// no pass over Fg.
constexpr int kBlkEndTileMax = 64;
constexpr int kBlkEndGranMax = 8192;  // granule table entries (u8)
// the dynamic staging's share of kBlkLdsBytes: k_blk_end's static LDS (the
// granule table and lp[]) comes first -- at n_prot >= 320 a full 80 KB of
// staging on top of it left room for one workgroup per CU
constexpr int kBlkEndDynLds = kBlkLdsBytes - kBlkEndGranMax - (kBlkEndTileMax + 1) * 8 - 64;

template <int NTH, int U = 1>
__global__ __launch_bounds__(NTH, 2048 / 256) void k_blk_end(Dev d, int tile) {
    // (two 1024-thread workgroups per CU: <= 64 VGPRs)
    extern __shared__ uint32_t ende[];  // [tile][n_prot], tetramer-major
    __shared__ int64_t lp[kBlkEndTileMax + 1];
    // the tile's tetramer at the start of every 64-entry granule of F: one
    // LDS read per 8-entry chunk instead of a 6-step binary search (a chain
    // of dependent LDS reads) -- tiles with more granules (a tetramer held by
    // most genomes) keep the search
    constexpr int kGran = 6, kGranMax = kBlkEndGranMax;
    __shared__ uint8_t gtl[kGranMax];
    const int tid = threadIdx.x, lane = tid & 63, P = d.n_prot;
    const int t0 = blockIdx.x * tile;
    const int nt = min(tile, kNTetramers - t0);
    for (int k = tid; k < tile * P; k += NTH) ende[k] = 0u;
    if (tid <= nt) lp[tid] = d.Lp[t0 + tid];
    __syncthreads();
    const int64_t S = lp[0], E = lp[nt];
    auto search = [&](int64_t i) {  // last tl with lp[tl] <= i
        int lo = 0, hi = nt - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (lp[mid] <= i) lo = mid; else hi = mid - 1;
        }
        return lo;
    };
    const int64_t G0 = S & ~(int64_t)((1 << kGran) - 1);
    const int64_t ng = ((E - G0) >> kGran) + 1;
    const bool gran = ng <= kGranMax;  // uniform
    if (gran) {
        for (int64_t g = tid; g < ng; g += NTH) gtl[g] = (uint8_t)search(max(G0 + (g << kGran), S));
        __syncthreads();
    }
    // U: 16-B loads per lane in flight before the first is used
    for (int64_t cb = (S & ~(int64_t)7) + (int64_t)tid * 8; cb - (int64_t)lane * 8 < E; cb += (int64_t)U * NTH * 8) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t c0 = cb + (int64_t)u * NTH * 8;
            v[u] = c0 < E ? *reinterpret_cast<const uint4*>(d.Fp16 + c0) : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t c0 = cb + (int64_t)u * NTH * 8;
            // wave-uniform up to the DPP (it needs the whole wave)
            uint32_t next = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(v[u].x & 0xFFFFu), 0x130, 0xf, 0xf, false);  // wave_shl:1
            if (lane == 63) next = c0 + 8 < E ? d.Fp16[c0 + 8] : 0xFFFFu;
            if (c0 >= E) continue;
            const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
            const int64_t i0 = max(c0, S);
            int tl;  // tetramer of entry i0
            if (gran) {
                tl = gtl[(i0 - G0) >> kGran];  // the granule start's; a boundary may follow inside it
                while (tl + 1 < nt && lp[tl + 1] <= i0) ++tl;
            } else {
                tl = search(i0);
            }
            int64_t nb = lp[tl + 1];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int64_t i = c0 + j;
                const uint32_t q = (w[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
                const uint32_t qn = j == 7 ? next : (w[(j + 1) >> 1] >> (16 * ((j + 1) & 1))) & 0xFFFFu;
                if (i < S || i >= E) continue;
                if (i >= nb) {  // crossed into a later tetramer block
                    while (tl + 1 < nt && lp[tl + 1] <= i) ++tl;
                    nb = lp[tl + 1];
                }
                if (i + 1 == nb || qn != q) ende[tl * P + q] = (uint32_t)(i + 1);
            }
        }
    }
    __syncthreads();
    uint32_t* ends = reinterpret_cast<uint32_t*>(d.blk);
    for (int k = tid; k < tile * P; k += NTH) {
        const int tl = k % tile, q = k / tile;  // one protein's consecutive tetramers per run of lanes
        if (tl < nt) ends[(int64_t)q * kNTetramers + t0 + tl] = ende[tl * P + q];
    }
}

// ---------------------------------------------------------------------------
// K-W2: stable LSD radix sort of the (key, entry) pairs, 8-bit digits.
// Tiles of 4096 keys (256 threads x 16, striped so loads coalesce).  Per
// pass: k_rs_hist (LDS histogram per tile -> hist[digit][tile]), an
// exclusive scan of hist (digit-major: global base of every (digit, tile)),
// k_rs_scatter (stable in-tile rank: per 256-key round, peers with the same
// digit found with 8 wavefront ballots, wave counts prefixed in LDS).  The
// last pass writes the final work list rec_c[entry] at the sorted position.
// ---------------------------------------------------------------------------
constexpr int kRsThreads = 256;
constexpr int kRsRounds = 16;
constexpr int kRsTile = kRsThreads * kRsRounds;
constexpr int kRsBins = 256;

template <bool FIRSTPASS, bool LAST>
__global__ __launch_bounds__(kRsThreads) void k_rs_scatter(
    const uint32_t* __restrict__ keys_in, const uint32_t* __restrict__ vals_in, int64_t n, int shift,
    const unsigned long long* __restrict__ offs, const uint32_t* __restrict__ hist, int64_t ntiles,
    uint32_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out, const uint2* __restrict__ rec_c,
    uint2* __restrict__ recs_out) {
    __shared__ uint32_t lkey[kRsTile];
    __shared__ uint32_t lval[kRsTile];
    __shared__ uint32_t lstart[kRsBins];  // tile-local start of each digit
    __shared__ uint32_t base[kRsBins];    // running tile-local position of each digit
    __shared__ uint32_t wpos[kRsThreads / 64][kRsBins];
    __shared__ uint32_t wcnt[kRsThreads / 64][kRsBins];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const unsigned long long lt = (1ull << lane) - 1ull;
    {  // exclusive scan of this tile's digit counts (hist[digit][tile])
        const uint32_t c = hist[(int64_t)tid * ntiles + blockIdx.x];
        uint32_t inc = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t u = __shfl_up(inc, o, 64);
            if (lane >= o) inc += u;
        }
        if (lane == 63) wcnt[0][wid] = inc;
        __syncthreads();
        uint32_t off = 0;
        for (int w = 0; w < wid; ++w) off += wcnt[0][w];
        lstart[tid] = off + inc - c;
        base[tid] = off + inc - c;
        __syncthreads();
    }
    const int64_t t0 = (int64_t)blockIdx.x * kRsTile;
    const int tn = (int)((n - t0) < kRsTile ? (n - t0) : kRsTile);
    for (int r = 0; r < kRsRounds; ++r) {
        const int li = r * kRsThreads + tid;
        const bool valid = li < tn;
        const int64_t j = t0 + li;
        const uint32_t k = valid ? keys_in[j] : 0u;
        const uint32_t v = valid ? (FIRSTPASS ? (uint32_t)j : vals_in[j]) : 0u;
        const uint32_t dig = (k >> shift) & (kRsBins - 1);
        unsigned long long peers = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < 8; ++bit) {
            const bool on = (dig >> bit) & 1u;
            const unsigned long long m = __ballot(on);
            peers &= on ? m : ~m;
        }
        const uint32_t rank = __popcll(peers & lt);
#pragma unroll
        for (int w = 0; w < kRsThreads / 64; ++w) wcnt[w][tid] = 0u;
        __syncthreads();
        if (valid && rank == 0) wcnt[wid][dig] = __popcll(peers);
        __syncthreads();
        {
            uint32_t run = base[tid];
#pragma unroll
            for (int w = 0; w < kRsThreads / 64; ++w) {
                wpos[w][tid] = run;
                run += wcnt[w][tid];
            }
            base[tid] = run;
        }
        __syncthreads();
        if (valid) {
            const uint32_t lp = wpos[wid][dig] + rank;  // stable tile-local position
            lkey[lp] = k;
            lval[lp] = v;
        }
    }
    __syncthreads();
    // write each digit's run of the tile contiguously
    for (int li = tid; li < tn; li += kRsThreads) {
        const uint32_t k = lkey[li], v = lval[li];
        const uint32_t dig = (k >> shift) & (kRsBins - 1);
        const unsigned long long pos = offs[(int64_t)dig * ntiles + blockIdx.x] + (li - lstart[dig]);
        keys_out[pos] = k;
        if (LAST) recs_out[pos] = rec_c[v];
        else vals_out[pos] = v;
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

// ---------------------------------------------------------------------------
// K-S: scatter the E triples (p, A, *) of one row and protein into LDS
// counters.  acc word w holds columns cc0+2w (low u16) and cc0+2w+1 (high).
// The (row, protein) member ranges are first staged in LDS with one
// coalesced load; then each 16-lane group takes kUnroll ranges at a time and
// issues their first member loads together (kUnroll independent 64-B loads
// in flight per group, 256 per workgroup) before the LDS atomics -- the
// scatter is bound by load latency, so memory-level parallelism is the lever.
// Ranges hold <= 64 members (longer runs are split at build time).
// ---------------------------------------------------------------------------
template <int MODE>
__device__ __forceinline__ void scatter_one(const Dev& d, int32_t a, int32_t b, uint32_t* acc, int32_t cc0,
                                            int32_t cc1, uint32_t& ev) {
    if (b < 0) return;
    if (MODE == 1 && !(b != a && (!d.is_q[b] || b > a))) return;  // isValidPair, ds_impl.hpp:270-273
    if (MODE == kModeFull && b == a) return;
    if (b >= cc0 && b < cc1) {
        const uint32_t o = (uint32_t)(b - cc0);
        atomicAdd(&acc[o >> 1], 1u << ((o & 1u) << 4));
        ++ev;
    }
}

constexpr uint32_t kLongCut = 4 * kGroup;  // a group walks at most this many members of a range

// rec_lds: kRowThreads staged ranges; long_lds: tails of long ranges, walked
// by the whole workgroup.
template <int MODE, int kUnroll, bool LONGQ = true>
__device__ __forceinline__ uint32_t scatter_row_protein(const Dev& d, int32_t a, const uint2* __restrict__ recs,
                                                        uint64_t rb, uint64_t re, uint32_t* acc,
                                                        uint2* rec_lds, uint2* long_lds, int* n_long,
                                                        int32_t cc0, int32_t cc1) {
    const int tid = threadIdx.x;
    const int grp = tid / kGroup, gl = tid % kGroup;
    uint32_t ev = 0;
    for (uint64_t base = rb; base < re; base += kRowThreads) {  // uniform trip count
        const int n = (int)((re - base) < (uint64_t)kRowThreads ? (re - base) : (uint64_t)kRowThreads);
        __syncthreads();  // previous readers of rec_lds / long_lds are done
        if (tid < n) rec_lds[tid] = recs[base + tid];
        if (tid == 0) *n_long = 0;
        __syncthreads();
        for (int j = grp; j < n; j += kNumGroups * kUnroll) {
            uint32_t lo[kUnroll], hi[kUnroll];
            int32_t b[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const int k = j + u * kNumGroups;
                const uint2 r = k < n ? rec_lds[k] : make_uint2(0u, 0u);
                lo[u] = r.x;
                hi[u] = r.y;
            }
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) b[u] = lo[u] + gl < hi[u] ? d.Fg[lo[u] + gl] : -1;
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) scatter_one<MODE>(d, a, b[u], acc, cc0, cc1, ev);
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const uint32_t cut = (LONGQ && hi[u] - lo[u] > kLongCut) ? lo[u] + kLongCut : hi[u];
                for (uint32_t m = lo[u] + kGroup + gl; m < cut; m += kGroup)
                    scatter_one<MODE>(d, a, d.Fg[m], acc, cc0, cc1, ev);
                if (cut < hi[u] && gl == 0) {  // hand the tail to the whole workgroup
                    const int slot = atomicAdd(n_long, 1);
                    long_lds[slot] = make_uint2(cut, hi[u]);
                }
            }
        }
        if (!LONGQ) continue;
        __syncthreads();
        const int nl = *n_long;
        for (int q = 0; q < nl; ++q) {  // e.g. a core tetramer shared by every genome
            const uint2 r = long_lds[q];
            for (uint32_t m = r.x + tid; m < r.y; m += kRowThreads) scatter_one<MODE>(d, a, d.Fg[m], acc, cc0, cc1, ev);
        }
    }
    return ev;
}

// ---------------------------------------------------------------------------
// Fused genome-major scatter (k_rows<FUSED>): no work list at all.  The rows'
// (row, protein) member ranges are exactly the runs (t, p) of the row
// genome's own G entries (A, p, t) -- A is a member of each -- and the order
// of ranges inside one protein does not matter to the integer counts.  So per
// protein the workgroup stages run = blk[p][t] for its G entries in LDS,
// cuts every run into 64-B-aligned 16-member "line tasks" (one block scan
// gives both a run's task offset and, for runs longer than kMaxLines lines,
// its slot in the whole-workgroup queue), and each 16-lane group takes
// kUnroll tasks at a time with their loads in flight together.  Members
// outside the row's column window (B <= A for ALL, queries for QT) or not a
// valid QSUB partner are dropped by scatter_one, exactly as before -- the
// member position of A is never searched for.
// ---------------------------------------------------------------------------
constexpr int kMaxLines = 8;                       // lines a run may hand out as tasks
constexpr int kTaskCap = kMaxLines * kRowThreads;  // u16 tasks: (run slot | line << 10)

__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(v, o, 64);
        if (lane >= o) v += u;
    }
    return v;
}

template <int MODE, int kUnroll, bool PRUNE>
__device__ __forceinline__ uint32_t scatter_row_g(const Dev& d, int32_t a, int p, int64_t gb, int64_t ge,
                                                  uint32_t* acc, uint2* rec_lds, uint16_t* task_lds,
                                                  uint32_t* wsum, uint2* long_lds, int32_t cc0, int32_t cc1) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int grp = tid / kGroup, gl = tid % kGroup;
    const uint4* blk_p = d.blk + (int64_t)p * kNTetramers;
    uint32_t ev = 0;
    for (int64_t base = gb; base < ge; base += kRowThreads) {  // uniform trip count
        const int n = (int)(ge - base < kRowThreads ? ge - base : kRowThreads);
        __syncthreads();  // previous readers of the staging arrays are done
        uint4 r4 = make_uint4(0u, 0u, 0u, 0u);
        if (tid < n) r4 = blk_p[d.G_tet[base + tid]];
        uint2 r = make_uint2(r4.x, r4.y);
        // a run of one member is A alone: no partner
        const uint32_t first = r.x & ~(uint32_t)(kGroup - 1);
        uint32_t nl = r.y - r.x > 1u ? (r.y - first + kGroup - 1) / kGroup : 0u;
        if (PRUNE && nl > 1u) {  // lines [l0, l1) can hold members in [cc0, cc1)
            const uint64_t sp = (uint64_t)r4.z | ((uint64_t)r4.w << 32);
            uint32_t l0 = 0, l1 = nl;
#pragma unroll
            for (uint32_t i = 1; i <= (uint32_t)kSplitters; ++i) {
                const int32_t f = (int32_t)((sp >> (kSplitBits * (i - 1))) & kSplitNone);
                if (i < nl) {
                    if (f <= cc0) l0 = i;               // lines < i hold ids < f <= cc0
                    if (f >= cc1 && l1 > i) l1 = i;     // lines >= i hold ids >= f >= cc1
                }
            }
            if (l1 <= l0) { nl = 0; }
            else {
                if (l0) r.x = first + l0 * kGroup;
                if (l1 < nl) r.y = first + l1 * kGroup;
                nl = l1 - l0;
            }
        }
        const bool lng = nl > (uint32_t)kMaxLines;
        const uint32_t v = lng ? (1u << 16) : nl;  // low half: tasks, high half: long runs
        rec_lds[tid] = r;
        const uint32_t inc = wave_incl_scan_u32(v);
        if (lane == 63) wsum[wid] = inc;
        __syncthreads();
        // wave offsets: lane w < 16 holds wave w's total; scan them across the lanes
        const uint32_t ws = wave_incl_scan_u32(lane < kRowThreads / 64 ? wsum[lane] : 0u);
        const uint32_t off = wid ? (uint32_t)__shfl(ws, wid - 1, 64) : 0u;
        const uint32_t tot = (uint32_t)__shfl(ws, kRowThreads / 64 - 1, 64);
        const uint32_t ex = off + inc - v;
        if (lng) long_lds[ex >> 16] = r;
        else
            for (uint32_t i = 0; i < nl; ++i) task_lds[(ex & 0xFFFFu) + i] = (uint16_t)(tid | (i << 10));
        const int n_tasks = (int)(tot & 0xFFFFu), n_long = (int)(tot >> 16);
        __syncthreads();
        for (int j = grp; j < n_tasks; j += kNumGroups * kUnroll) {
            int32_t b[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const int k = j + u * kNumGroups;
                b[u] = -1;
                if (k < n_tasks) {
                    const uint32_t tk = task_lds[k];
                    const uint2 rr = rec_lds[tk & 1023u];
                    const uint32_t m = (rr.x & ~(uint32_t)(kGroup - 1)) + (tk >> 10) * kGroup + gl;
                    if (m >= rr.x && m < rr.y) b[u] = d.Fg[m];
                }
            }
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) scatter_one<MODE>(d, a, b[u], acc, cc0, cc1, ev);
        }
        for (int q = 0; q < n_long; ++q) {  // e.g. a core tetramer shared by every genome
            const uint2 rr = long_lds[q];
            for (uint32_t m = rr.x + tid; m < rr.y; m += kRowThreads) scatter_one<MODE>(d, a, d.Fg[m], acc, cc0, cc1, ev);
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
// Two workgroups per CU (<= 64 VGPRs).  FUSED: the genome-major walk of
// scatter_row_g (G lists + run table, no work list; the fallback of
// k_rows_pl for G lists longer than it takes); otherwise the work-list walk
// of scatter_row_protein (F-only input), long ranges walked by their group.
template <int MODE, int KW, bool FUSED>
__global__ __launch_bounds__(kRowThreads, 8) void k_rows(
    Dev d, int64_t row_begin, const unsigned long long* __restrict__ rowptr,
    const uint2* __restrict__ recs, int32_t chunk_cols, uint32_t flags,
    const unsigned long long* __restrict__ first_key, double* __restrict__ aji, double* __restrict__ s_out, int32_t* __restrict__ n_out,
    unsigned long long* __restrict__ n_events) {
    extern __shared__ uint32_t acc[];  // KW*1024 counter words
    __shared__ uint2 rec_lds[kRowThreads];
    __shared__ uint2 long_lds[FUSED ? kRowThreads : 1];
    __shared__ uint16_t task_lds[FUSED ? kTaskCap : 1];
    __shared__ uint32_t wsum[kRowThreads / 64];
    __shared__ int n_long;
    const int tid = threadIdx.x;
    const int64_t rl = xcd_row(blockIdx.x, gridDim.x);  // local row
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
        uint64_t rb, re;
        if constexpr (FUSED) {
            rb = (uint64_t)d.G_off[(int64_t)a * P + p];
            re = (uint64_t)d.G_off[(int64_t)a * P + p + 1];
        } else {
            rb = rowptr[rl * P + p];
            re = rowptr[rl * P + p + 1];
        }
        if (rb == re) continue;  // uniform: no E triple (p, a, *)
        if (flags & 0x200u) {  // diagnostics: 0x200 skips the scatter
        } else if constexpr (FUSED) {
            ev += scatter_row_g<MODE, 8, true>(d, a, p, (int64_t)rb, (int64_t)re, acc, rec_lds, task_lds, wsum, long_lds,
                                               cc0, cc1);
        } else {
            ev += scatter_row_protein<MODE, 4, false>(d, a, recs, rb, re, acc, rec_lds, long_lds, &n_long, cc0, cc1);
        }
        __syncthreads();
        if (flags & 0x100u) {  // diagnostics: 0x100 skips the normalisation (counters just cleared)
            for (int w = tid; w < ncw; w += kRowThreads) acc[w] = 0u;
            __syncthreads();
            continue;
        }
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
        double sv[2];
        int32_t nv[2];
        bool ok[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int32_t b = cc0 + 2 * w + h;
            ok[h] = b < cc1 && col_valid<MODE>(d, a, b);
            double s = S[2 * k + h];
            int32_t n = (int32_t)((N[k] >> (16 * h)) & 0xFFFFu);
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

// Debug: dump the per-protein counts of one row (integer parity vs E).
template <int MODE>
__global__ __launch_bounds__(kRowThreads) void k_row_counts(
    Dev d, int64_t row_begin, const unsigned long long* __restrict__ rowptr,
    const uint2* __restrict__ recs, int32_t chunk_cols, int32_t* __restrict__ counts) {
    extern __shared__ uint32_t acc[];
    __shared__ uint2 rec_lds[kRowThreads];
    __shared__ uint2 long_lds[kRowThreads];
    __shared__ int n_long;
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
        scatter_row_protein<MODE, 4>(d, a, recs, rb, re, acc, rec_lds, long_lds, &n_long, cc0, cc1);
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
