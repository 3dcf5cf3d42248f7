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
// Per pass (digit of DB bits, BINS = 2^DB; tiles of NT * kSortItems records,
// NT = kSortNT threads: 4096 records at the default 512):
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

constexpr int kSortThreads = 1024;                      // k_sort_grp / k_sort_top
constexpr int kSortItems = 8;                           // records per thread and tile
// threads of the hist / scatter workgroups: 512 (tiles of 4096 records; the
// scatter's LDS, 56 KB at 10-bit digits, lets two workgroups share a CU, so
// one's barriers and write-phase loads overlap the other's ranking) -- one
// 1024-thread workgroup per CU (8192-record tiles, ~104 KB of LDS) left the
// CU idle at every barrier: 2.9-3.3 ms per pass at 10k, ~1.5 TB/s
constexpr int kSortNT = 512;
constexpr bool kSortPF = false;                          // next-tile prefetch (k_sort_scatter PF)
constexpr int kSortTileMin = 512 * kSortItems;          // the smallest tile (sizes the hist buffer)
constexpr int kSortGroup = 128;                         // tiles per group of the hist scan
constexpr int kSortMaxDB = 11;
template <int NT>
constexpr int sort_tile() { return NT * kSortItems; }

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
    __device__ __forceinline__ uint64_t hist_rec(int64_t i, bool valid) const {
        const int32_t p = Fp[i], g = Fg[i];
        if (fp16 && valid) fp16[i] = (uint16_t)p;
        return (uint64_t)((uint32_t)g * P + (uint32_t)p);
    }
    __device__ __forceinline__ uint64_t load(int64_t i) const {
        return (uint64_t)((uint32_t)Fg[i] * P + (uint32_t)Fp[i]) | ((uint64_t)i << 32);
    }
};

// materialised records (later passes; first passes of the keygen paths)
struct SrcRecs {
    const uint64_t* r;
    __device__ __forceinline__ uint64_t hist_rec(int64_t i, bool) const { return r[i]; }
    __device__ __forceinline__ uint64_t load(int64_t i) const { return r[i]; }
};

// ---- destinations (last pass) ----------------------------------------------
// The write phase is split so that a tile's dependent loads are issued
// together: fetch(pos, v) loads what store needs (Aux), then store(pos, v,
// aux) writes -- eight records per thread, every fetch before the first store.

struct DstRecs {
    uint64_t* r;
    static constexpr int kWH = kSortItems;
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
    static constexpr int kWH = kSortItems;
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
    static constexpr int kWH = kSortItems / 2;  // (three-field Aux: eight in flight spill)
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
    static constexpr int kWH = kSortItems;
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

template <int DB, int NT, class Src>
__global__ __launch_bounds__(NT) void k_sort_hist(Src src, int64_t n, int shift, uint32_t mask,
                                                  uint32_t* __restrict__ hist) {
    constexpr int BINS = 1 << DB;
    __shared__ uint32_t h[BINS];
    for (int b = threadIdx.x; b < BINS; b += NT) h[b] = 0u;
    __syncthreads();
    const int64_t t0 = (int64_t)blockIdx.x * sort_tile<NT>();
    uint32_t d[kSortItems];
    // every load issued before the first LDS atomic, none under a branch: a
    // load in a branch is waited for before the branch joins (vmcnt(0)), so
    // a conditional load per item serialised eight HBM round trips
#pragma unroll
    for (int k = 0; k < kSortItems; ++k) {
        const int64_t i = t0 + k * NT + threadIdx.x;
        const bool valid = i < n;
        d[k] = sort_digit(src.hist_rec(valid ? i : n - 1, valid), shift, mask);
        if (!valid) d[k] = 0xFFFFFFFFu;
    }
#pragma unroll
    for (int k = 0; k < kSortItems; ++k)
        if (d[k] != 0xFFFFFFFFu) atomicAdd(&h[d[k]], 1u);
    __syncthreads();
    for (int b = threadIdx.x; b < BINS; b += NT) hist[(int64_t)blockIdx.x * BINS + b] = h[b];
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

// dynamic LDS of k_sort_scatter<DB, NT>
template <int DB, int NT>
constexpr size_t sort_scatter_lds() {
    return (size_t)(NT / 64) * (1 << DB) * 2   // per-wave u16 digit counters
           + 2 * (size_t)(1 << DB) * 4          // lstart, gbase
           + (size_t)sort_tile<NT>() * 8;       // the reordered tile
}

// waves per SIMD the scatter is compiled for: two 512-thread workgroups per
// CU (<= 128 VGPRs)
template <int NT>
constexpr int sort_scatter_wpe() { return NT == 512 ? 4 : 1; }

// PF: the next tile's records and digit bases are loaded while this tile is
// ranked and written (16 + BPT VGPRs live across the tile)
// VAR (diagnostics A/B, 0 in the product): bit 0 round-robin tile order,
// bit 1 the ranking ballots done twice (their cost), bit 2 records stored straight
// from registers at their ranked positions (no LDS reorder), bit 3 no global
// stores (ablation)
template <int DB, int NT, bool PF, class Src, class Dst, int VAR = 0>
__global__ __launch_bounds__(NT, sort_scatter_wpe<NT>()) void k_sort_scatter(
    Src src, Dst dst, int64_t n, int64_t ntiles, int shift, uint32_t mask, const uint32_t* __restrict__ hist,
    const uint32_t* __restrict__ gsum, const uint32_t* __restrict__ binbase) {
    constexpr int BINS = 1 << DB, W = NT / 64, kTile = sort_tile<NT>();
    constexpr int BPT = BINS > NT ? BINS / NT : 1;  // digits per thread (scans)
    // write phase: Dst::kWH records' destination loads issued before the
    // first store -- all eight where the registers allow (gfx9 counts stores
    // in vmcnt: a second batch's loads wait for the first batch's stores)
    constexpr int kWH = Dst::kWH;
    extern __shared__ __align__(16) unsigned char sort_lds[];
    uint64_t* srt = reinterpret_cast<uint64_t*>(sort_lds);                          // [kTile]
    uint32_t* lstart = reinterpret_cast<uint32_t*>(sort_lds + (size_t)kTile * 8);  // [BINS]
    uint32_t* gbase = lstart + BINS;                                                // [BINS]
    uint16_t* cnt = reinterpret_cast<uint16_t*>(gbase + BINS);                      // [W][BINS], 16-B aligned
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
    // the tile's loads are unconditional (indices clamped into range: a load
    // under a branch is waited for at the branch, which serialised the eight
    // record loads of a tile -- ~2.8 ms per pass at 10k); records past n are
    // never used (every use below checks the position)
    auto fetch_tile = [&](int64_t tile, uint64_t (&r)[kSortItems], uint32_t (&g)[BPT]) {
        const int64_t tc = tile < ntiles ? tile : ntiles - 1;
        const int64_t t0 = tc * kTile;
#pragma unroll
        for (int k = 0; k < kSortItems; ++k) {
            const int64_t i = t0 + (wid * kSortItems + k) * 64 + lane;
            r[k] = src.load(i < n ? i : n - 1);
        }
        const int64_t grp = tc / kSortGroup;
#pragma unroll
        for (int q = 0; q < BPT; ++q) {
            const int b = min(tid + q * NT, BINS - 1);
            g[q] = binbase[b] + gsum[grp * BINS + b] + hist[tc * BINS + b];
        }
    };
    uint64_t hsum = 0;  // Dst::kSum: the destination's per-record sum (DstGposHash)
    // tile order: tile0 + j * tstep.  The workgroups of one XCD (blockIdx %
    // 8: dispatch is round-robin over the 8 XCDs) walk one contiguous eighth
    // of the tiles, so the tiles in flight on an XCD write adjacent pieces of
    // every digit's output run, and whole lines leave its L2 (round-robin
    // tiles: 2.72 -> 2.32 ms for the 10k F -> G first pass); VAR bit 0 keeps
    // the round-robin order (A/B)
    int64_t tile0 = blockIdx.x, tstep = gridDim.x, tend = ntiles;
    if constexpr ((VAR & 1) == 0) {
        const int64_t nx = gridDim.x / 8, x = blockIdx.x % 8;
        if (nx >= 1 && (int64_t)gridDim.x % 8 == 0) {
            const int64_t per = (ntiles + 7) / 8;
            tile0 = x * per + blockIdx.x / 8;
            tstep = nx;
            tend = min(ntiles, (x + 1) * per);
        }
    }
    fetch_tile(tile0 < tend ? tile0 : ntiles, rec, gb);
    for (int64_t tile = tile0; tile < tend; tile += tstep) {
        const int64_t t0 = tile * kTile;
        const int64_t tnext = tile + tstep < tend ? tile + tstep : ntiles;
        uint64_t nrec[kSortItems];
        uint32_t ngb[BPT];
        if constexpr (PF) fetch_tile(tnext, nrec, ngb);  // in flight during this tile
#pragma unroll
        for (int q = 0; q < BPT; ++q) {
            const int b = tid + q * NT;
            if (b < BINS) gbase[b] = gb[q];
        }
        // the per-wave counters cleared by 16-B stores (W * BINS / 8 of them)
        for (int x = tid; x < W * BINS / 8; x += NT) reinterpret_cast<uint4*>(cnt)[x] = make_uint4(0u, 0u, 0u, 0u);
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
            if constexpr ((VAR & 2) != 0) {  // the ballots a second time (their cost, by difference)
                uint64_t p2 = __ballot(valid);
                uint32_t d2 = d;
                asm volatile("" : "+v"(d2));  // opaque: the ballots are not folded into the first set
#pragma unroll
                for (int bit = 0; bit < DB; ++bit) {
                    const bool on = (d2 >> bit) & 1u;
                    const uint64_t m = __ballot(on);
                    p2 &= on ? m : ~m;
                }
                peers = p2;
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
        if constexpr ((VAR & 4) != 0) {  // straight from registers: position gbase + wave prefix + rank
#pragma unroll
            for (int k = 0; k < kSortItems; ++k) {
                if (t0 + (wid * kSortItems + k) * 64 + lane < n) {
                    const uint32_t d = sort_digit(rec[k], shift, mask);
                    const uint32_t pos = gbase[d] + cnt[wid * BINS + d] + lr[k];
                    const auto ax = dst.fetch(pos, rec[k]);
                    if constexpr ((VAR & 8) == 0) hsum += dst.store(pos, rec[k], ax);
                }
            }
            __syncthreads();
            if constexpr (PF) {
#pragma unroll
                for (int k = 0; k < kSortItems; ++k) rec[k] = nrec[k];
#pragma unroll
                for (int q = 0; q < BPT; ++q) gb[q] = ngb[q];
            } else {
                fetch_tile(tnext, rec, gb);
            }
            continue;
        }
        {
            uint32_t slot[kSortItems];  // every LDS read issued before the first write
#pragma unroll
            for (int k = 0; k < kSortItems; ++k) {
                const uint32_t d = sort_digit(rec[k], shift, mask);
                slot[k] = lstart[d] + cnt[wid * BINS + d] + lr[k];
            }
#pragma unroll
            for (int k = 0; k < kSortItems; ++k)
                if (t0 + (wid * kSortItems + k) * 64 + lane < n) srt[slot[k]] = rec[k];
        }
        __syncthreads();
        // write the tile in digit order: each digit's run is contiguous in the output
        // (positions are < 2^32: n <= 2^32 - 64; records re-read from LDS for the stores)
        const int tn = (int)((n - t0) < kTile ? (n - t0) : kTile);
        // (unconditional reads at positions clamped into the tile: no wait per item)
#pragma unroll
        for (int h = 0; h < kSortItems; h += kWH) {  // kWH records per thread in flight
            uint32_t pos[kWH];
            uint64_t val[kWH];
            typename Dst::Aux aux[kWH];
#pragma unroll
            for (int k = 0; k < kWH; ++k) {
                const int lp = min(tid + (h + k) * NT, tn - 1);
                val[k] = srt[lp];
            }
#pragma unroll
            for (int k = 0; k < kWH; ++k) {
                const int lp = min(tid + (h + k) * NT, tn - 1);
                const uint32_t d = sort_digit(val[k], shift, mask);
                pos[k] = gbase[d] + (uint32_t)(lp - (int)lstart[d]);
            }
#pragma unroll
            for (int k = 0; k < kWH; ++k) aux[k] = dst.fetch(pos[k], val[k]);
#pragma unroll
            for (int k = 0; k < kWH; ++k) {
                const int lp = tid + (h + k) * NT;
                if ((VAR & 8) == 0 && lp < tn) hsum += dst.store(pos[k], val[k], aux[k]);
            }
        }
        __syncthreads();  // the LDS tile, counters and bases are rewritten by the next tile
        if constexpr (PF) {
#pragma unroll
            for (int k = 0; k < kSortItems; ++k) rec[k] = nrec[k];
#pragma unroll
            for (int q = 0; q < BPT; ++q) gb[q] = ngb[q];
        } else {
            fetch_tile(tnext, rec, gb);
        }
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
        // four rounds of the workgroup per batch, loads first (clamped, not branched)
        for (int64_t i0 = s + threadIdx.x; i0 < e; i0 += 4 * (int64_t)blockDim.x) {
            int32_t p[4], g[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t i = min(i0 + u * (int64_t)blockDim.x, e - 1);
                p[u] = Fp[i];
                g[u] = Fg[i];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t i = i0 + u * (int64_t)blockDim.x;
                if (i < e) {
                    fp16[i] = (uint16_t)p[u];
                    rec[i] = (uint64_t)((uint32_t)g[u] * P + (uint32_t)p[u]) | ((uint64_t)t << kb) |
                             ((uint64_t)(i - s) << (kb + 18));
                }
            }
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
        // four 64-entry chunks per round, loads first (clamped, not branched)
        for (int64_t k0 = b + lane; k0 < e; k0 += 4 * 64) {
            uint32_t t[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) t[u] = (uint32_t)G_tet[min(k0 + u * 64, e - 1)];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (k0 + u * 64 < e) rec[o + (k0 + u * 64 - b)] = (uint64_t)t[u] | pg;
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
