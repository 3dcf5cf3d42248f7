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
// The write phase is split so that a tile's dependent loads are issued
// together: fetch(pos, v) loads what store needs (Aux), then store(pos, v,
// aux) writes -- eight records per thread, every fetch before the first store.

struct DstRecs {
    uint64_t* r;
    static constexpr bool kSum = false;
    struct Aux {};
    __device__ __forceinline__ Aux fetch(int64_t, uint64_t) const { return {}; }
    __device__ __forceinline__ uint64_t store(int64_t pos, uint64_t v, Aux) const {
        r[pos] = v;
        return 0;
    }
};

// Both F and G given (records key g * P + p | F index << 32, sorted = F's
// genome-major transpose): G_pos[pos] = F index i, and the caller's G must BE
// that transpose --
//   list bounds: its list (g, p) must span pos (G_off[key] <= pos <
//     G_off[key + 1]; with |G| = |F| and G_off monotone that pins every
//     list bound); a mismatch sets *err;
//   tetramers: its tetramer at pos must be F entry i's.  F entry i's tetramer
//     is not in the record (key 21 + tetramer 18 + index 30 bits do not fit
//     64), so the check is a keyed hash of the pairs: the sum over G of
//     h(G_pos[k], G_tet[k]) (here, from coalesced reads) must equal the sum
//     over F of h(i, t(i)) (k_hash_f, from Lp alone).  G_pos is a bijection
//     onto F by construction, so the sums differ unless every tetramer
//     matches, except with probability ~2^-64 (h is a 64-bit mix of the
//     injective (i, t) code, keyed by a per-load random seed).
__device__ __forceinline__ uint64_t mix64(uint64_t x) {  // splitmix64 finaliser (a bijection)
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
__device__ __forceinline__ uint64_t pair_hash(uint64_t seed, uint64_t i, uint32_t t) {
    return mix64(seed ^ ((i << 18) | t));  // i < 2^32, t < 2^18: an injective 50-bit code
}

struct DstGposHash {
    uint32_t* G_pos;
    const int32_t* G_tet;
    const int64_t* G_off;
    uint64_t seed;
    int* err;
    unsigned long long* sum;
    static constexpr bool kSum = true;
    struct Aux {
        uint32_t lo, hi;  // list bounds (< 2^32: |G| = |F| <= 2^32 - 64)
        int32_t tu;
    };
    __device__ __forceinline__ Aux fetch(int64_t pos, uint64_t v) const {
        const uint32_t key = (uint32_t)v;
        return {(uint32_t)G_off[key], (uint32_t)G_off[key + 1], G_tet[pos]};
    }
    __device__ __forceinline__ uint64_t store(int64_t pos, uint64_t v, Aux a) const {
        const uint32_t i = (uint32_t)(v >> 32);
        G_pos[pos] = i;
        if (!(a.lo <= (uint64_t)pos && (uint64_t)pos < a.hi)) atomicOr(err, 1);
        return pair_hash(seed, i, (uint32_t)a.tu & 0x3FFFFu) + (uint64_t)((uint32_t)a.tu >> 18);  // (t >= 2^18: never equal)
    }
};

// the F side of DstGposHash's sum: h(i, t) over every F entry i of every
// tetramer block t -- from Lp alone, no F read
__global__ __launch_bounds__(256) void k_hash_f(const int64_t* __restrict__ Lp, uint64_t seed,
                                                unsigned long long* __restrict__ sum) {
    uint64_t acc = 0;
    for (int t = blockIdx.x; t < kNTetramers; t += gridDim.x) {
        const int64_t e = Lp[t + 1];
        for (int64_t i = Lp[t] + threadIdx.x; i < e; i += blockDim.x) acc += pair_hash(seed, (uint64_t)i, (uint32_t)t);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
    if ((threadIdx.x & 63) == 0 && acc) atomicAdd(sum, (unsigned long long)acc);
}

// F only (records key g * P + p | t << kb | j << (kb + 18) from k_fkeys_rec,
// F index Lp[t] + j; the tetramer travels with the record): G_tet and G_pos
// (if kept) at the sorted position.  G_off comes from T (T[p][g] is the
// length of list (g, p) in a consistent problem) and must span every
// position: a mismatch sets *err and the caller rebuilds G the general way.
struct DstGFromRecs {
    uint32_t* G_pos;  // nullable
    int32_t* G_tet;
    const int64_t* G_off;
    const int64_t* Lp;
    int kb;
    int* err;
    static constexpr bool kSum = false;
    struct Aux {
        uint32_t lo, hi, lp;  // (all < 2^32: |F| <= 2^32 - 64)
    };
    __device__ __forceinline__ Aux fetch(int64_t, uint64_t v) const {
        const uint32_t key = (uint32_t)v & ((1u << kb) - 1u);
        const int32_t t = (int32_t)((v >> kb) & 0x3FFFFu);
        return {(uint32_t)G_off[key], (uint32_t)G_off[key + 1], G_pos ? (uint32_t)Lp[t] : 0u};
    }
    __device__ __forceinline__ uint64_t store(int64_t pos, uint64_t v, Aux a) const {
        G_tet[pos] = (int32_t)((v >> kb) & 0x3FFFFu);
        if (G_pos) G_pos[pos] = a.lp + (uint32_t)(v >> (kb + 18));
        if (!(a.lo <= (uint64_t)pos && (uint64_t)pos < a.hi)) atomicOr(err, 1);
        return 0;
    }
};

// G only (records t | p << 18 | g << 30 from k_gkeys_pm, enumerated
// protein-major so that the stable sort by t alone yields F's (t, p, g)
// order): the F columns at the sorted position, the u16 protein column, and
// the tetramer of every position (Ft, for Lp by k_rowptr -- counting Lc by
// atomics while generating the records cost 11 ms at 10k: 2.9e8 global
// atomics on 160 000 counters).  No G_pos here: the inverse permutation would
// be 2.9e8 random 4-B stores (8-14 ms at 10k) for a ~5 % faster row kernel,
// which only repeated runs amortise (see pfaai_load).
struct DstFFromG {
    int32_t* Fp;
    int32_t* Fg;
    uint16_t* fp16;
    uint32_t* Ft;
    static constexpr bool kSum = false;
    struct Aux {};
    __device__ __forceinline__ Aux fetch(int64_t, uint64_t) const { return {}; }
    __device__ __forceinline__ uint64_t store(int64_t pos, uint64_t v, Aux) const {
        const uint32_t p = (uint32_t)(v >> 18) & 0xFFFu, g = (uint32_t)(v >> 30) & 0x1FFFFFu;
        Fp[pos] = (int32_t)p;
        Fg[pos] = (int32_t)g;
        fp16[pos] = (uint16_t)p;
        Ft[pos] = (uint32_t)v & 0x3FFFFu;
        return 0;
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
__global__ __launch_bounds__(kSortThreads) void k_sort_scatter(Src src, Dst dst, int64_t n, int64_t ntiles, int shift,
                                                               uint32_t mask, const uint32_t* __restrict__ hist,
                                                               const uint32_t* __restrict__ gsum,
                                                               const uint32_t* __restrict__ binbase) {
    constexpr int BINS = 1 << DB, W = kSortThreads / 64;
    constexpr int BPT = BINS > kSortThreads ? BINS / kSortThreads : 1;  // digits per thread (scans)
    extern __shared__ __align__(16) unsigned char sort_lds[];
    uint64_t* srt = reinterpret_cast<uint64_t*>(sort_lds);                              // [kSortTile]
    uint32_t* lstart = reinterpret_cast<uint32_t*>(sort_lds + (size_t)kSortTile * 8);  // [BINS]
    uint32_t* gbase = lstart + BINS;                                                    // [BINS]
    uint16_t* cnt = reinterpret_cast<uint16_t*>(gbase + BINS);                          // [W][BINS]
    __shared__ uint32_t wsum[W];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint64_t lt = (1ull << lane) - 1ull;
    uint16_t* wc = cnt + wid * BINS;
    // a tile's records: wave w owns [w * 512, (w + 1) * 512) of it, round k
    // at lanes 0..63 -- rank order = (wave, round, lane) = input order, so
    // the sort is stable.  Persistent: each workgroup walks tiles blockIdx.x
    // + j * gridDim.x and loads tile j + 1 (records and digit bases) while it
    // ranks and writes tile j.
    uint64_t rec[kSortItems];
    uint32_t gb[BPT];
    auto fetch_tile = [&](int64_t tile, uint64_t (&r)[kSortItems], uint32_t (&g)[BPT]) {
        const int64_t t0 = tile * kSortTile;
#pragma unroll
        for (int k = 0; k < kSortItems; ++k) {
            const int64_t i = t0 + (wid * kSortItems + k) * 64 + lane;
            r[k] = (tile < ntiles && i < n) ? src.load(i) : 0ull;
        }
        const int64_t grp = tile / kSortGroup;
#pragma unroll
        for (int q = 0; q < BPT; ++q) {
            const int b = tid + q * kSortThreads;
            g[q] = (tile < ntiles && b < BINS) ? binbase[b] + gsum[grp * BINS + b] + hist[tile * BINS + b] : 0u;
        }
    };
    uint64_t hsum = 0;  // Dst::kSum: the destination's per-record sum (DstGposHash)
    fetch_tile(blockIdx.x, rec, gb);
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t t0 = tile * kSortTile;
        uint64_t nrec[kSortItems];
        uint32_t ngb[BPT];
        fetch_tile(tile + gridDim.x, nrec, ngb);  // in flight during this tile
#pragma unroll
        for (int q = 0; q < BPT; ++q) {
            const int b = tid + q * kSortThreads;
            if (b < BINS) {
                gbase[b] = gb[q];
#pragma unroll
                for (int w = 0; w < W; ++w) cnt[w * BINS + b] = 0;
            }
        }
        __syncthreads();
        uint16_t lr[kSortItems];
#pragma unroll
        for (int k = 0; k < kSortItems; ++k) {
            const bool valid = t0 + (wid * kSortItems + k) * 64 + lane < n;
            const uint32_t d = sort_digit(rec[k], shift, mask);
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
        // per digit: the waves' counts -> exclusive prefix over waves; the
        // tile's total, then its exclusive scan over the digits
        uint32_t tot[BPT], mine = 0;
#pragma unroll
        for (int q = 0; q < BPT; ++q) {
            const int b = tid * BPT + q;
            uint32_t run = 0;
            if (b < BINS) {
#pragma unroll
                for (int w = 0; w < W; ++w) {
                    const uint32_t v = cnt[w * BINS + b];
                    cnt[w * BINS + b] = (uint16_t)run;
                    run += v;
                }
            }
            tot[q] = run;
            mine += run;
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
            off += tot[q];
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kSortItems; ++k) {
            if (t0 + (wid * kSortItems + k) * 64 + lane < n) {
                const uint32_t d = sort_digit(rec[k], shift, mask);
                srt[lstart[d] + cnt[wid * BINS + d] + lr[k]] = rec[k];
            }
        }
        __syncthreads();
        // write the tile in digit order: each digit's run is contiguous in the output
        // (positions are < 2^32: n <= 2^32 - 64; records re-read from LDS for the stores)
        const int tn = (int)((n - t0) < kSortTile ? (n - t0) : kSortTile);
#pragma unroll
        for (int h = 0; h < kSortItems; h += kSortItems / 2) {  // two halves: fewer live registers
            uint32_t pos[kSortItems / 2];
            typename Dst::Aux aux[kSortItems / 2];
#pragma unroll
            for (int k = 0; k < kSortItems / 2; ++k) {
                const int lp = tid + (h + k) * kSortThreads;
                if (lp < tn) {
                    const uint64_t v = srt[lp];
                    const uint32_t d = sort_digit(v, shift, mask);
                    pos[k] = gbase[d] + (uint32_t)(lp - (int)lstart[d]);
                    aux[k] = dst.fetch(pos[k], v);
                }
            }
#pragma unroll
            for (int k = 0; k < kSortItems / 2; ++k) {
                const int lp = tid + (h + k) * kSortThreads;
                if (lp < tn) hsum += dst.store(pos[k], srt[lp], aux[k]);
            }
        }
        __syncthreads();  // the LDS tile, counters and bases are rewritten by the next tile
#pragma unroll
        for (int k = 0; k < kSortItems; ++k) rec[k] = nrec[k];
#pragma unroll
        for (int q = 0; q < BPT; ++q) gb[q] = ngb[q];
    }
    if constexpr (Dst::kSum) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) hsum += __shfl_down(hsum, o, 64);
        if (lane == 0 && hsum) atomicAdd(dst.sum, (unsigned long long)hsum);
    }
}

// ---- keygen kernels (paths whose first pass needs a materialised record) ----

// F -> records for DstGFromRecs: one workgroup per tetramer block
// (grid-stride), so the tetramer of every entry is known without a search:
// rec = key g * P + p | t << kb | (i - Lp[t]) << (kb + 18); also the u16
// protein column.
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
// g << 30.
__global__ __launch_bounds__(256) void k_gkeys_pm(const int64_t* __restrict__ G_off, const int32_t* __restrict__ G_tet,
                                                  int64_t n_lists, int32_t P, int32_t n_ids,
                                                  const unsigned long long* __restrict__ pm_off,
                                                  uint64_t* __restrict__ rec) {
    const int lane = threadIdx.x & 63;
    const int64_t waves = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t L = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); L < n_lists; L += waves) {
        const uint32_t g = (uint32_t)(L / P), p = (uint32_t)(L % P);
        const int64_t b = G_off[L], e = G_off[L + 1];
        const int64_t o = (int64_t)pm_off[(int64_t)p * n_ids + g];
        const uint64_t pg = ((uint64_t)p << 18) | ((uint64_t)g << 30);
        for (int64_t k = b + lane; k < e; k += 64) rec[o + (k - b)] = (uint64_t)(uint32_t)G_tet[k] | pg;
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
