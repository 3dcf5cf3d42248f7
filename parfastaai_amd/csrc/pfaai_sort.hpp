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
//                  run of the tile is contiguous in the output (4 records of 8
//                  B on average at DB = 10), so consecutive lanes store to
//                  consecutive addresses; the tiles in flight on an XCD are
//                  consecutive (per-XCD tile counters), so neighbouring runs
//                  complete whole lines in its L2.
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
// scatter's LDS, 56 KB at 10-bit digits, lets two workgroups share a CU).
// With the per-XCD tile counters and non-temporal loads it measures 1.84 /
// 1.63 ms for the 10k F -> G passes against 2.13 / 1.85 for one 1024-thread
// workgroup per CU (8192-record tiles, ~104 KB of LDS), and the next-tile
// prefetch (PF) costs more registers than it hides: 2.07 / 1.61
// (profiles/r03u_sort/)
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
    __device__ __forceinline__ uint64_t load_nt(int64_t i) const {  // streamed once: no L2 residency wanted
        return (uint64_t)((uint32_t)__builtin_nontemporal_load(Fg + i) * P + (uint32_t)__builtin_nontemporal_load(Fp + i)) |
               ((uint64_t)i << 32);
    }
};

// materialised records (later passes; first passes of the keygen paths)
struct SrcRecs {
    const uint64_t* r;
    __device__ __forceinline__ uint64_t hist_rec(int64_t i, bool) const { return r[i]; }
    __device__ __forceinline__ uint64_t load(int64_t i) const { return r[i]; }
    __device__ __forceinline__ uint64_t load_nt(int64_t i) const { return __builtin_nontemporal_load(r + i); }
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
// that transpose.  That is a statement about sets: F's memberships (g, p, t)
// and G's must be the same (both hold distinct triples: F strictly sorted by
// (t, p, g), every G list strictly ascending -- host-checked -- and |G| =
// |F|).  Then list (g, p) holds exactly F's entries with key g * P + p, in
// t order = F index order, so the sorted positions ARE G's positions.  The
// set equality is proven by keyed hash sums: the sum over F of h(g * P + p,
// t) (k_hash_f, streaming F block by block) must equal the sum over G of
// h(list, G_tet) (k_gend) -- in two lanes keyed by independent per-load
// random seeds, so different sets agree with probability ~2^-128 (h is a
// 64-bit mix of the injective 50-bit code key << 18 | t).  So the sort's passes load nothing
// beyond their records (the first form checked list bounds by G_off[key],
// G_off[key + 1] and read G_tet[pos] per record in the last pass: ~3 random
// L2 requests per record, 3.4 ms of a 10k load's pass).
__device__ __forceinline__ uint64_t mix64(uint64_t x) {  // splitmix64 finaliser (a bijection)
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
__device__ __forceinline__ uint64_t member_hash(uint64_t seed, uint32_t key, uint32_t t) {
    return mix64(seed ^ (((uint64_t)key << 18) | t));  // key < 2^32, t < 2^18 (host-checked): injective
}

struct DstGpos {
    uint32_t* G_pos;
    static constexpr int kWH = kSortItems;
    static constexpr bool kSum = false;
    struct Aux {};
    __device__ __forceinline__ Aux fetch(int64_t, uint64_t) const { return {}; }
    __device__ __forceinline__ uint64_t store(int64_t pos, uint64_t v, Aux) const {
        G_pos[pos] = (uint32_t)(v >> 32);
        return 0;
    }
};

// the F side of the membership sum: h(g * P + p, t) over every F entry of
// every tetramer block t (one workgroup per block, grid-stride; four entries
// per thread in flight, indices clamped rather than loads under a branch)
// Two lanes (seed, seed2: independent per-load random keys; sums[0] and
// sums[2]): a different multiset passes both with probability ~2^-128.
__global__ __launch_bounds__(256) void k_hash_f(const int64_t* __restrict__ Lp, const int32_t* __restrict__ Fp,
                                                const int32_t* __restrict__ Fg, uint32_t P, uint64_t seed,
                                                uint64_t seed2, unsigned long long* __restrict__ sum) {
    uint64_t acc = 0, acc2 = 0;
    for (int t = blockIdx.x; t < kNTetramers; t += gridDim.x) {
        const int64_t b = Lp[t], e = Lp[t + 1];
        for (int64_t i0 = b + threadIdx.x; i0 < e; i0 += 4 * 256) {
            uint32_t key[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t i = min(i0 + u * 256, e - 1);
                key[u] = (uint32_t)__builtin_nontemporal_load(Fg + i) * P + (uint32_t)__builtin_nontemporal_load(Fp + i);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i0 + u * 256 < e) {
                    acc += member_hash(seed, key[u], (uint32_t)t);
                    acc2 += member_hash(seed2, key[u], (uint32_t)t);
                }
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        acc += __shfl_down(acc, o, 64);
        acc2 += __shfl_down(acc2, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        if (acc) atomicAdd(sum, (unsigned long long)acc);
        if (acc2) atomicAdd(sum + 2, (unsigned long long)acc2);
    }
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
                                                           uint32_t* __restrict__ binbase, uint32_t* __restrict__ tctr) {
    if (threadIdx.x < 8) tctr[threadIdx.x] = 0u;  // the scatter's per-XCD tile counters
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
// bit 1 the ranking ballots done twice (their cost), bit 3 no global stores
// (ablation), bit 4 ordinary (temporal) record loads, bit 5 a static tile
// stride instead of the per-XCD tile counters (tctr[8], zeroed by k_sort_top)
template <int DB, int NT, bool PF, class Src, class Dst, int VAR = 0>
__global__ __launch_bounds__(NT, sort_scatter_wpe<NT>()) void k_sort_scatter(
    Src src, Dst dst, int64_t n, int64_t ntiles, int shift, uint32_t mask, const uint32_t* __restrict__ hist,
    const uint32_t* __restrict__ gsum, const uint32_t* __restrict__ binbase, uint32_t* __restrict__ tctr) {
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
            if constexpr ((VAR & 16) == 0)  // streamed once: non-temporal, the L2 keeps the output lines
                r[k] = src.load_nt(i < n ? i : n - 1);
            else
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
    int64_t tile0 = blockIdx.x, tstep = gridDim.x, tend = ntiles, xbase = 0;
    const int xcd = blockIdx.x % 8;
    bool dyn = false;
    if constexpr ((VAR & 1) == 0) {
        const int64_t nx = gridDim.x / 8;
        if (nx >= 1 && (int64_t)gridDim.x % 8 == 0) {
            const int64_t per = (ntiles + 7) / 8;
            xbase = xcd * per;
            tile0 = xbase + blockIdx.x / 8;
            tstep = nx;
            tend = min(ntiles, (xcd + 1) * per);
            dyn = (VAR & 32) == 0;
        }
    }
    __shared__ uint32_t s_next;
    // the next tile: the XCD's next one, by one atomic per tile, so the
    // tiles in flight on an XCD are consecutive and its L2 sees whole output
    // lines (a static stride let fast workgroups run ahead: 2.33 -> 1.80 ms
    // for the 10k F -> G first pass); VAR bit 5 keeps the static stride
    auto next_tile = [&](int64_t cur) -> int64_t {
        if (!dyn) return cur + tstep;
        if (tid == 0) s_next = atomicAdd(&tctr[xcd], 1u);
        __syncthreads();
        return xbase + (int64_t)s_next;
    };
    int64_t tile = dyn ? next_tile(0) : tile0;
    fetch_tile(tile < tend ? tile : ntiles, rec, gb);
    while (tile < tend) {
        const int64_t t0 = tile * kTile;
        int64_t tnext = 0;
        uint64_t nrec[kSortItems];
        uint32_t ngb[BPT];
        if constexpr (PF) {  // in flight during this tile
            tnext = next_tile(tile);
            fetch_tile(tnext < tend ? tnext : ntiles, nrec, ngb);
        }
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
            tnext = next_tile(tile);
            fetch_tile(tnext < tend ? tnext : ntiles, rec, gb);
        }
        tile = tnext;
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

// k_gend over G, list by list (one pass over G_tet, G_pos):
//   END:  G_end[k] = the end of the F run (t, p) of G entry k of list (g, p),
//         from the run-end table (k_blk_end, u32, p-major) -- looked up once
//         per load, so the WK 3 row kernel reads (G_pos, G_end) coalesced;
//   HASH: the G side of the both-given check (DstGpos): sums[0] +=
//         h(list of k, G_tet[k]) and, keyed by seed2, sums[2] (k_hash_f's
//         second lane).
// The lists are taken protein-major (all genomes of protein p, then p + 1),
// so the table lookups in flight hit one or two protein rows (640 KB each),
// which stay in every XCD's L2 -- genome-major order touched all 100 rows at
// once (4.5 ms at 10k, mostly L2 misses).  A workgroup takes kGendLists
// consecutive lists and walks their entries as one flat range, four entries
// per thread in flight.  (The lookups are random 4-B requests: one L2 request
// per entry bounds it, ~1.8 ms at 10k.)
constexpr int kGendLists = 32;

template <bool END, bool HASH>
__global__ __launch_bounds__(256) void k_gend(const int64_t* __restrict__ G_off, const int32_t* __restrict__ G_tet,
                                              int64_t n_lists, int32_t P, const uint32_t* __restrict__ ends,
                                              uint32_t* __restrict__ G_end, uint64_t seed, uint64_t seed2,
                                              unsigned long long* __restrict__ sums) {
    __shared__ int64_t lb[kGendLists];
    __shared__ uint32_t pre[kGendLists + 1];
    __shared__ int64_t row[kGendLists];
    __shared__ uint32_t lid[kGendLists];
    const int tid = threadIdx.x;
    const int64_t n_ids = n_lists / P;
    uint64_t hm = 0, hm2 = 0;
    for (int64_t q0 = (int64_t)blockIdx.x * kGendLists; q0 < n_lists; q0 += (int64_t)gridDim.x * kGendLists) {
        if (tid < 64) {  // one wave: the block's lists, their lengths and an inclusive scan
            uint32_t len = 0;
            if (tid < kGendLists) {
                const int64_t q = min(q0 + tid, n_lists - 1);
                const int64_t p = q / n_ids, L = (q - p * n_ids) * P + p;
                const int64_t b = G_off[L], e = G_off[L + 1];
                lb[tid] = b;
                row[tid] = p * kNTetramers;
                lid[tid] = (uint32_t)L;
                len = q0 + tid < n_lists ? (uint32_t)(e - b) : 0u;
            }
            uint32_t inc = len;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t u = __shfl_up(inc, o, 64);
                if (tid >= o) inc += u;
            }
            if (tid < kGendLists) pre[tid + 1] = inc;
            if (tid == 0) pre[0] = 0u;
        }
        __syncthreads();
        const uint32_t total = pre[kGendLists];
        for (uint32_t f0 = tid; f0 < total; f0 += 4 * 256) {
            int64_t k[4];
            int64_t rw[4];
            uint32_t li[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t f = min(f0 + (uint32_t)u * 256u, total - 1u);
                int lo = 0;  // the list j with pre[j] <= f < pre[j + 1]
#pragma unroll
                for (int w = kGendLists / 2; w > 0; w >>= 1)
                    if (pre[lo + w] <= f) lo += w;
                k[u] = lb[lo] + (f - pre[lo]);
                rw[u] = row[lo];
                li[u] = lid[lo];
            }
            int32_t t[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)  // (streamed once: non-temporal, the L2 keeps the table rows)
                t[u] = __builtin_nontemporal_load(G_tet + k[u]);
            uint32_t v[4];
            if constexpr (END) {
#pragma unroll
                for (int u = 0; u < 4; ++u) v[u] = ends[rw[u] + t[u]];  // (G_tet < 160000: host-checked)
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (f0 + (uint32_t)u * 256u < total) {
                    if constexpr (END) G_end[k[u]] = v[u];
                    if constexpr (HASH) {
                        hm += member_hash(seed, li[u], (uint32_t)t[u]);
                        hm2 += member_hash(seed2, li[u], (uint32_t)t[u]);
                    }
                }
            }
        }
        __syncthreads();  // lb / pre / row / lid are rewritten by the next block
    }
    if constexpr (HASH) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            hm += __shfl_down(hm, o, 64);
            hm2 += __shfl_down(hm2, o, 64);
        }
        if ((tid & 63) == 0) {
            if (hm) atomicAdd(&sums[0], (unsigned long long)hm);
            if (hm2) atomicAdd(&sums[2], (unsigned long long)hm2);
        }
    }
}

}  // namespace pfaai
