// pfaai_sort.hpp -- the load-time transposition sort: a stable LSD radix sort
// of 64-bit records by the low KB bits (the key), in two passes of <= 11-bit
// digits (three of 8 for 24-bit keys).
//
// What it replaces: the reference builds F with an SQL UNION ALL + ORDER BY
// (scp_db.hpp:161-216, ds_helper.hpp:126-162); the engine needs F and its
// genome-major transpose G, and builds whichever the caller did not hand over
// (pfaai_build.hpp).  Each is one stable sort of the other by a small key:
//   G from F   key g * P + p (< 2^21 at 20 480 x 100), F order is t-ascending
//   F from G   the G entries enumerated protein-major, key t (18 bits): a
//              stable sort by tetramer leaves each (t, p) run in genome order
//
// Per pass (digit of DB bits, BINS = 2^DB; tiles of kSortTile = 8192 records):
//   k_sort_hist    per-tile digit counts -> hist[tile][bin] (tile-major, one
//                  coalesced 4-KB row per tile at DB = 10)
//   k_sort_grp     per group of kSortGroup tiles: hist rows -> exclusive prefix
//                  within the group (in place) and the group's sums
//   k_sort_top     one workgroup: exclusive scan of the group sums per bin and
//                  of the bin totals -> binbase[bin]
//   k_sort_scatter per tile: the stable in-tile rank by wave ballots (DB
//                  ballots give each lane its peers with the same digit) and
//                  per-wave u16 digit counters in LDS, the tile reordered by
//                  digit in LDS, then written out in that order: each digit's
//                  run of the tile is contiguous in the output (8 records of 8
//                  B on average at DB = 10), so consecutive lanes store to
//                  consecutive addresses.
// The sources of the first pass and the destination of the last are functors,
// so the first pass reads the caller's arrays directly (no key array) and the
// last writes the product columns -- and, when both orientations were given,
// checks them -- instead of a sorted copy.
#pragma once
#include "pfaai_kernels.hpp"

namespace pfaai {

constexpr int kSortThreads = 1024;
constexpr int kSortItems = 8;                           // records per thread and tile
constexpr int kSortTile = kSortThreads * kSortItems;    // 8192
constexpr int kSortGroup = 128;                         // tiles per group of the hist scan
constexpr int kSortMaxDB = 11;

__device__ __forceinline__ uint32_t sort_digit(uint64_t r, int shift, uint32_t mask) {
    return (uint32_t)(r >> shift) & mask;
}

// ---- sources (first pass) --------------------------------------------------

// F entry i -> key g * P + p (low 32 bits) | i << 32.  The histogram pass
// also writes the u16 protein column of F that k_blk / k_blk_end read.
struct SrcFKeys {
    const int32_t* Fp;
    const int32_t* Fg;
    uint32_t P;
    uint16_t* fp16;  // nullable
    __device__ __forceinline__ uint64_t hist_rec(int64_t i) const {
        const int32_t p = Fp[i], g = Fg[i];
        if (fp16) fp16[i] = (uint16_t)p;
        return (uint64_t)((uint32_t)g * P + (uint32_t)p);
    }
    __device__ __forceinline__ uint64_t load(int64_t i) const {
        return (uint64_t)((uint32_t)Fg[i] * P + (uint32_t)Fp[i]) | ((uint64_t)i << 32);
    }
};

// materialised records (later passes; first passes of the keygen paths)
struct SrcRecs {
    const uint64_t* r;
    __device__ __forceinline__ uint64_t hist_rec(int64_t i) const { return r[i]; }
    __device__ __forceinline__ uint64_t load(int64_t i) const { return r[i]; }
};

// ---- destinations (last pass) ----------------------------------------------

struct DstRecs {
    uint64_t* r;
    __device__ __forceinline__ void store(int64_t pos, uint64_t v) const { r[pos] = v; }
};

// Both F and G given (records key g * P + p | F index << 32, sorted = F's
// genome-major transpose): G_pos[pos] = F index, and the caller's G must BE
// that transpose -- its tetramer at pos is the F entry's (Lp[t] <= i <
// Lp[t + 1]) and its list (g, p) spans pos (G_off[key] <= pos < G_off[key +
// 1]; with |G| = |F| and G_off monotone that pins every list bound).  Any
// mismatch sets *err.
struct DstGposCheck {
    uint32_t* G_pos;
    const int32_t* G_tet;
    const int64_t* G_off;
    const int64_t* Lp;
    int* err;
    __device__ __forceinline__ void store(int64_t pos, uint64_t v) const {
        const uint32_t key = (uint32_t)v, i = (uint32_t)(v >> 32);
        if (G_pos) G_pos[pos] = i;
        const int32_t t = G_tet[pos];
        const bool ok = (uint32_t)t < (uint32_t)kNTetramers && Lp[t] <= (int64_t)i && (int64_t)i < Lp[t + 1] &&
                        G_off[key] <= pos && pos < G_off[key + 1];
        if (!ok) atomicOr(err, 1);
    }
};

// F only (records key g * P + p | t << kb | j << (kb + 18), F index Lp[t] +
// j, from k_fkeys_rec): G_tet / G_pos at the sorted position; G_off comes
// from T (T[p][g] is the length of list (g, p) in a consistent problem) and
// is verified like DstGposCheck's (a mismatch sets *err: the caller rebuilds
// G the general way).
struct DstGFromF {
    uint32_t* G_pos;  // nullable
    int32_t* G_tet;
    const int64_t* G_off;
    const int64_t* Lp;
    int kb;
    int* err;
    __device__ __forceinline__ void store(int64_t pos, uint64_t v) const {
        const uint32_t key = (uint32_t)v & ((1u << kb) - 1u);
        const int32_t t = (int32_t)((v >> kb) & 0x3FFFFu);
        const int64_t i = Lp[t] + (int64_t)(v >> (kb + 18));
        G_tet[pos] = t;
        if (G_pos) G_pos[pos] = (uint32_t)i;
        if (!(G_off[key] <= pos && pos < G_off[key + 1])) atomicOr(err, 1);
    }
};

// G only (records t | p << 18 | g << 30 | j << 51 from k_gkeys_pm, enumerated
// protein-major so that the stable sort by t alone yields F's (t, p, g)
// order): the F columns at the sorted position, the u16 protein column, and
// G_pos of the G entry G_off[g * P + p] + j.
struct DstFFromG {
    int32_t* Fp;
    int32_t* Fg;
    uint16_t* fp16;
    uint32_t* G_pos;  // nullable
    const int64_t* G_off;
    uint32_t P;
    __device__ __forceinline__ void store(int64_t pos, uint64_t v) const {
        const uint32_t p = (uint32_t)(v >> 18) & 0xFFFu, g = (uint32_t)(v >> 30) & 0x1FFFFFu;
        Fp[pos] = (int32_t)p;
        Fg[pos] = (int32_t)g;
        fp16[pos] = (uint16_t)p;
        if (G_pos) G_pos[G_off[(int64_t)g * P + p] + (int64_t)(v >> 51)] = (uint32_t)pos;
    }
};

// ---- the pass kernels -------------------------------------------------------

template <int DB, class Src>
__global__ __launch_bounds__(kSortThreads) void k_sort_hist(Src src, int64_t n, int shift, uint32_t mask,
                                                            uint32_t* __restrict__ hist) {
    constexpr int BINS = 1 << DB;
    __shared__ uint32_t h[BINS];
    for (int b = threadIdx.x; b < BINS; b += kSortThreads) h[b] = 0u;
    __syncthreads();
    const int64_t t0 = (int64_t)blockIdx.x * kSortTile;
    uint32_t d[kSortItems];
#pragma unroll
    for (int k = 0; k < kSortItems; ++k) {  // every load issued before the first LDS atomic
        const int64_t i = t0 + k * kSortThreads + threadIdx.x;
        d[k] = i < n ? sort_digit(src.hist_rec(i), shift, mask) : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int k = 0; k < kSortItems; ++k)
        if (d[k] != 0xFFFFFFFFu) atomicAdd(&h[d[k]], 1u);
    __syncthreads();
    for (int b = threadIdx.x; b < BINS; b += kSortThreads) hist[(int64_t)blockIdx.x * BINS + b] = h[b];
}

// hist rows of one group of tiles -> exclusive prefix within the group (in
// place); gsum[group][bin] = the group's total
template <int DB>
__global__ __launch_bounds__(kSortThreads) void k_sort_grp(uint32_t* __restrict__ hist, int64_t ntiles,
                                                           uint32_t* __restrict__ gsum) {
    constexpr int BINS = 1 << DB;
    const int64_t j0 = (int64_t)blockIdx.x * kSortGroup;
    const int nj = (int)((ntiles - j0) < kSortGroup ? (ntiles - j0) : kSortGroup);
    for (int b = threadIdx.x; b < BINS; b += kSortThreads) {
        uint32_t run = 0;
        int j = 0;
        for (; j + 8 <= nj; j += 8) {
            uint32_t v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = hist[(j0 + j + u) * BINS + b];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                hist[(j0 + j + u) * BINS + b] = run;
                run += v[u];
            }
        }
        for (; j < nj; ++j) {
            const uint32_t v = hist[(j0 + j) * BINS + b];
            hist[(j0 + j) * BINS + b] = run;
            run += v;
        }
        gsum[(int64_t)blockIdx.x * BINS + b] = run;
    }
}

// one workgroup: gsum -> exclusive prefix over groups per bin; binbase[bin] =
// exclusive prefix of the bin totals
template <int DB>
__global__ __launch_bounds__(kSortThreads) void k_sort_top(uint32_t* __restrict__ gsum, int64_t ngroups,
                                                           uint32_t* __restrict__ binbase) {
    constexpr int BINS = 1 << DB;
    constexpr int BPT = BINS > kSortThreads ? BINS / kSortThreads : 1;  // bins per thread
    __shared__ uint32_t wsum[kSortThreads / 64];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    uint32_t tot[BPT];
#pragma unroll
    for (int q = 0; q < BPT; ++q) {
        const int b = tid * BPT + q;
        uint32_t run = 0;
        if (b < BINS) {
            int64_t g = 0;
            for (; g + 8 <= ngroups; g += 8) {
                uint32_t v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = gsum[(g + u) * BINS + b];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    gsum[(g + u) * BINS + b] = run;
                    run += v[u];
                }
            }
            for (; g < ngroups; ++g) {
                const uint32_t v = gsum[g * BINS + b];
                gsum[g * BINS + b] = run;
                run += v;
            }
        }
        tot[q] = run;
    }
    uint32_t mine = 0;
#pragma unroll
    for (int q = 0; q < BPT; ++q) mine += tot[q];
    uint32_t inc = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(inc, o, 64);
        if (lane >= o) inc += u;
    }
    if (lane == 63) wsum[wid] = inc;
    __syncthreads();
    uint32_t off = inc - mine;
    for (int w = 0; w < wid; ++w) off += wsum[w];
#pragma unroll
    for (int q = 0; q < BPT; ++q) {
        const int b = tid * BPT + q;
        if (b < BINS) binbase[b] = off;
        off += tot[q];
    }
}

// dynamic LDS of k_sort_scatter<DB>
template <int DB>
constexpr size_t sort_scatter_lds() {
    return (size_t)(kSortThreads / 64) * (1 << DB) * 2   // per-wave u16 digit counters
           + 2 * (size_t)(1 << DB) * 4                    // lstart, gbase
           + (size_t)kSortTile * 8;                       // the reordered tile
}

template <int DB, class Src, class Dst>
__global__ __launch_bounds__(kSortThreads) void k_sort_scatter(Src src, Dst dst, int64_t n, int shift, uint32_t mask,
                                                               const uint32_t* __restrict__ hist,
                                                               const uint32_t* __restrict__ gsum,
                                                               const uint32_t* __restrict__ binbase) {
    constexpr int BINS = 1 << DB, W = kSortThreads / 64;
    const uint32_t MASK = mask;  // the digit's bits of the key only: record fields follow the key directly
    extern __shared__ __align__(16) unsigned char sort_lds[];
    uint64_t* srt = reinterpret_cast<uint64_t*>(sort_lds);                              // [kSortTile]
    uint32_t* lstart = reinterpret_cast<uint32_t*>(sort_lds + (size_t)kSortTile * 8);  // [BINS]
    uint32_t* gbase = lstart + BINS;                                                    // [BINS]
    uint16_t* cnt = reinterpret_cast<uint16_t*>(gbase + BINS);                          // [W][BINS]
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int64_t tile = blockIdx.x, t0 = tile * kSortTile, grp = tile / kSortGroup;
    // this tile's records: wave w owns [w * 512, (w + 1) * 512) of the tile,
    // round k of it at lanes 0..63 -- rank order = (wave, round, lane) =
    // input order, so the sort is stable
    uint64_t rec[kSortItems];
#pragma unroll
    for (int k = 0; k < kSortItems; ++k) {
        const int64_t i = t0 + (wid * kSortItems + k) * 64 + lane;
        rec[k] = i < n ? src.load(i) : 0ull;
    }
    for (int b = tid; b < BINS; b += kSortThreads) {
        gbase[b] = binbase[b] + gsum[grp * BINS + b] + hist[tile * BINS + b];
#pragma unroll
        for (int w = 0; w < W; ++w) cnt[w * BINS + b] = 0;
    }
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1ull;
    uint16_t lr[kSortItems];
    uint16_t* wc = cnt + wid * BINS;
#pragma unroll
    for (int k = 0; k < kSortItems; ++k) {
        const bool valid = t0 + (wid * kSortItems + k) * 64 + lane < n;
        const uint32_t d = sort_digit(rec[k], shift, MASK);
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < DB; ++bit) {  // (bits above the mask are 0 in every lane: same ballot)
            const bool on = (d >> bit) & 1u;
            const uint64_t m = __ballot(on);
            peers &= on ? m : ~m;
        }
        const uint32_t r = (uint32_t)__popcll(peers & lt), c = (uint32_t)__popcll(peers);
        const uint32_t base = valid ? wc[d] : 0u;
        lr[k] = (uint16_t)(base + r);
        if (valid && r + 1 == c) wc[d] = (uint16_t)(base + c);  // the group's last lane advances the counter
    }
    __syncthreads();
    // per digit: the waves' counts -> exclusive prefix over waves; the tile's total
    for (int b = tid; b < BINS; b += kSortThreads) {
        uint32_t run = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const uint32_t v = cnt[w * BINS + b];
            cnt[w * BINS + b] = (uint16_t)run;
            run += v;
        }
        lstart[b] = run;
    }
    __syncthreads();
    {  // exclusive scan of the digit totals over the digits (BPT consecutive digits per thread)
        constexpr int BPT = BINS > kSortThreads ? BINS / kSortThreads : 1;
        __shared__ uint32_t wsum[W];
        uint32_t v[BPT], mine = 0;
#pragma unroll
        for (int q = 0; q < BPT; ++q) {
            const int b = tid * BPT + q;
            v[q] = b < BINS ? lstart[b] : 0u;
            mine += v[q];
        }
        uint32_t inc = mine;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t u = __shfl_up(inc, o, 64);
            if (lane >= o) inc += u;
        }
        if (lane == 63) wsum[wid] = inc;
        __syncthreads();
        uint32_t off = inc - mine;
        for (int w = 0; w < wid; ++w) off += wsum[w];
#pragma unroll
        for (int q = 0; q < BPT; ++q) {
            const int b = tid * BPT + q;
            if (b < BINS) lstart[b] = off;
            off += v[q];
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSortItems; ++k) {
        if (t0 + (wid * kSortItems + k) * 64 + lane < n) {
            const uint32_t d = sort_digit(rec[k], shift, MASK);
            srt[lstart[d] + cnt[wid * BINS + d] + lr[k]] = rec[k];
        }
    }
    __syncthreads();
    const int tn = (int)((n - t0) < kSortTile ? (n - t0) : kSortTile);
    for (int lp = tid; lp < tn; lp += kSortThreads) {
        const uint64_t v = srt[lp];
        const uint32_t d = sort_digit(v, shift, MASK);
        dst.store((int64_t)gbase[d] + (lp - (int)lstart[d]), v);
    }
}

// ---- keygen kernels (paths whose first pass needs a materialised record) ----

// F only: one workgroup per tetramer block (grid-stride): rec = key g * P + p
// | t << kb | (i - Lp[t]) << (kb + 18), and T-derived list lengths are not
// needed here (G_off comes from T).
__global__ __launch_bounds__(256) void k_fkeys_rec(const int64_t* __restrict__ Lp, const int32_t* __restrict__ Fp,
                                                   const int32_t* __restrict__ Fg, uint32_t P, int kb,
                                                   uint64_t* __restrict__ rec, uint16_t* __restrict__ fp16) {
    for (int t = blockIdx.x; t < kNTetramers; t += gridDim.x) {
        const int64_t s = Lp[t], e = Lp[t + 1];
        for (int64_t i = s + threadIdx.x; i < e; i += blockDim.x) {
            const int32_t p = Fp[i];
            fp16[i] = (uint16_t)p;
            rec[i] = (uint64_t)((uint32_t)Fg[i] * P + (uint32_t)p) | ((uint64_t)t << kb) |
                     ((uint64_t)(i - s) << (kb + 18));
        }
    }
}

// G only: one wave per (genome, protein) list; the list's entries go to the
// protein-major position pm_off[p * n_ids + g] + j as rec = t | p << 18 |
// g << 30 | j << 51, and Lc[t] is counted.
__global__ __launch_bounds__(256) void k_gkeys_pm(const int64_t* __restrict__ G_off, const int32_t* __restrict__ G_tet,
                                                  int64_t n_lists, int32_t P, int32_t n_ids,
                                                  const unsigned long long* __restrict__ pm_off,
                                                  uint64_t* __restrict__ rec, uint32_t* __restrict__ lc) {
    const int lane = threadIdx.x & 63;
    const int64_t waves = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t L = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); L < n_lists; L += waves) {
        const uint32_t g = (uint32_t)(L / P), p = (uint32_t)(L % P);
        const int64_t b = G_off[L], e = G_off[L + 1];
        const int64_t o = (int64_t)pm_off[(int64_t)p * n_ids + g];
        for (int64_t k = b + lane; k < e; k += 64) {
            const uint32_t t = (uint32_t)G_tet[k];
            rec[o + (k - b)] = (uint64_t)t | ((uint64_t)p << 18) | ((uint64_t)g << 30) | ((uint64_t)(k - b) << 51);
            atomicAdd(&lc[t], 1u);
        }
    }
}

// list lengths in protein-major order (the scan input of pm_off)
__global__ void k_len_pm(const int64_t* __restrict__ G_off, int32_t P, int32_t n_ids, uint32_t* __restrict__ len) {
    const int64_t n = (int64_t)P * n_ids;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p = k / n_ids, g = k % n_ids;
        len[k] = (uint32_t)(G_off[g * P + p + 1] - G_off[g * P + p]);
    }
}

// list lengths in (genome, protein) order from T (the F-only G_off)
__global__ void k_len_from_t(const int32_t* __restrict__ T, int32_t P, int32_t n_ids, int32_t t_cols,
                             uint32_t* __restrict__ len) {
    const int64_t n = (int64_t)P * n_ids;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t g = k / P, p = k % P;
        len[k] = (uint32_t)T[p * t_cols + g];
    }
}

}  // namespace pfaai
