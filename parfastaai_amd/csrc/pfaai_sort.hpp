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
#include "pfaai_util.hpp"

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
    static constexpr bool kFilter = false;  // (SrcFEnds: records outside a genome range are dropped)
    const int32_t* Fp;
    const int32_t* Fg;
    uint32_t P;
    uint16_t* fp16;  // nullable
    __device__ __forceinline__ bool keep(uint64_t) const { return true; }
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
    static constexpr bool kFilter = false;
    const uint64_t* r;
    __device__ __forceinline__ bool keep(uint64_t) const { return true; }
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
    __device__ __forceinline__ uint64_t store(int64_t pos, uint64_t v, Aux, int64_t) const {
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
// random seeds and mixed by two different functions, so a different set has
// to make both 64-bit sums agree at once (h is a 64-bit mix of the injective
// 50-bit code key << 18 | t; one-multiply mixers are not a proven universal
// family, so the ~2^-128 is heuristic).  So the sort's passes load nothing
// beyond their records (the first form checked list bounds by G_off[key],
// G_off[key + 1] and read G_tet[pos] per record in the last pass: ~3 random
// L2 requests per record, 3.4 ms of a 10k load's pass).
// xorshift-multiply-xorshift (a bijection of 64-bit words, nonlinear over
// both Z_2^64 and GF(2)^64): one 64-bit multiply per lane -- the check runs
// two lanes over every F and G entry beside the sort, and splitmix64's two
// multiplies per lane made it the load's largest side cost (2.8 ms at 10k)
// The two lanes use different mixers (shifts and multiplier), so lane 2 is
// not lane 1 applied to a re-keyed code: a swap of one tetramer between two
// lists -- codes {c, c^d1^d2} against {c^d1, c^d2}, an XOR parallelogram --
// has to cancel in two unrelated functions (tests/test_gpu_load_sort.py swaps
// tetramers between two genomes' lists and between two proteins' lists).
__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 32;
    x *= 0xD6E8FEB86659FD93ull;
    return x ^ (x >> 32);
}
__device__ __forceinline__ uint64_t mix64b(uint64_t x) {
    x ^= x >> 29;
    x *= 0xBF58476D1CE4E5B9ull;
    return x ^ (x >> 31);
}
__device__ __forceinline__ uint64_t member_hash(uint64_t seed, uint32_t key, uint32_t t) {
    return mix64(seed ^ (((uint64_t)key << 18) | t));  // key < 2^32, t < 2^18 (host-checked): injective
}
__device__ __forceinline__ uint64_t member_hash_b(uint64_t seed, uint32_t key, uint32_t t) {
    return mix64b(seed ^ (((uint64_t)key << 18) | t));
}

struct DstGpos {
    uint32_t* G_pos;
    static constexpr int kWH = kSortItems;
    static constexpr bool kSum = false;
    struct Aux {};
    __device__ __forceinline__ Aux fetch(int64_t, uint64_t) const { return {}; }
    __device__ __forceinline__ uint64_t store(int64_t pos, uint64_t v, Aux, int64_t) const {
        G_pos[pos] = (uint32_t)(v >> 32);
        return 0;
    }
};

// the F side of the membership sum: h(g * P + p, t) over every F entry of
// every tetramer block t (one workgroup per block, grid-stride; four entries
// per thread in flight, indices clamped rather than loads under a branch)
// Two lanes (seed, seed2: independent per-load random keys; sums[0] and
// sums[2]): a different multiset has to pass both lanes' sums at once.
// [g_lo, g_hi): only the entries of those genomes (a rank's rows, pfaai_load_rows).
__global__ __launch_bounds__(256) void k_hash_f(const int64_t* __restrict__ Lp, const int32_t* __restrict__ Fp,
                                                const int32_t* __restrict__ Fg, uint32_t P, uint64_t seed,
                                                uint64_t seed2, unsigned long long* __restrict__ sum, int32_t g_lo,
                                                int32_t g_hi) {
    uint64_t acc = 0, acc2 = 0;
    for (int t = blockIdx.x; t < kNTetramers; t += gridDim.x) {
        const int64_t b = Lp[t], e = Lp[t + 1];
        for (int64_t i0 = b + threadIdx.x; i0 < e; i0 += 4 * 256) {
            uint32_t key[4];
            bool in[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t i = min(i0 + u * 256, e - 1);
                const int32_t g = __builtin_nontemporal_load(Fg + i);
                key[u] = (uint32_t)g * P + (uint32_t)__builtin_nontemporal_load(Fp + i);
                in[u] = g >= g_lo && g < g_hi;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i0 + u * 256 < e && in[u]) {
                    acc += member_hash(seed, key[u], (uint32_t)t);
                    acc2 += member_hash_b(seed2, key[u], (uint32_t)t);
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
    __device__ __forceinline__ uint64_t store(int64_t pos, uint64_t v, Aux a, int64_t) const {
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
    __device__ __forceinline__ uint64_t store(int64_t pos, uint64_t v, Aux, int64_t) const {
        const uint32_t p = (uint32_t)(v >> 18) & 0xFFFu, g = (uint32_t)(v >> 30) & 0x1FFFFFu;
        Fp[pos] = (int32_t)p;
        Fg[pos] = (int32_t)g;
        fp16[pos] = (uint16_t)p;
        Ft[pos] = (uint32_t)v & 0x3FFFFu;
        return 0;
    }
};

// ---- the F -> G sort that carries run ends (G_pos and G_end in one sort) ----
// The all-vs-all row kernel walks, for every G entry (g, p, t), the F run
// (t, p) from just past g (G_pos + 1) to the run's end (G_end).  G_pos is the
// sorted position of F entry i in the F -> G sort (key g * P + p, F order is
// t order); G_end is the end of i's run, known in F order.  So the first
// pass's histogram kernel, which reads F tile by tile anyway, also finds the
// runs of its tile (a run ends where the protein changes or a tetramer block
// ends: a bitmap of block ends, k_block_ends) and writes each entry's
// distance to its run end (D, u32; kOpenRun for the tile's last run when it
// goes on into the next tiles -- its end is the first run end after the
// tile, ntail, from k_tail_suffix); the first scatter carries the distance
// in the record, the second writes G_pos and G_end side by side.  No run-end
// table and no lookup per G entry (k_blk_end + k_gend: 2.1 ms of the 10k load).
// Records: pass 1 key | rel << kb | dist << (kb + 12) | drop << 63 (rel: the
// position in its 4096-entry tile), written as key >> db | i << hb | dist <<
// (hb + 32) (hb = kb - db: the second digit, all that is left of the key);
// a run spans < 2^21 entries (one per genome id).  drop: the genome lies
// outside [g_lo, g_hi) (pfaai_load_rows: a rank builds the walk data of its
// own rows only).

constexpr uint32_t kNoTail = 0xFFFFFFFFu;
constexpr uint32_t kOpenRun = 0xFFFFFFFFu;
constexpr int kEndsTile = kSortNT * kSortItems;  // 4096 entries: the sort's tiles

// bit i of bend: F position i is the last of a tetramer block; with tcnt
// (the check) also the block ends per tile (tcnt, zeroed) and the non-empty
// flags of the blocks (flag)
__global__ void k_block_ends(const int64_t* __restrict__ Lp, uint32_t* __restrict__ bend, uint32_t* __restrict__ tcnt,
                             uint32_t* __restrict__ flag) {
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < kNTetramers; t += gridDim.x * blockDim.x) {
        const int64_t b = Lp[t], e = Lp[t + 1];
        if (e > b) atomicOr(&bend[(e - 1) >> 5], 1u << ((uint32_t)(e - 1) & 31u));
        if (tcnt) {
            flag[t] = e > b ? 1u : 0u;
            if (e > b) atomicAdd(&tcnt[(e - 1) / kEndsTile], 1u);
        }
    }
}

// The both-given check's tetramer: the F side knows the rank of an entry's
// block among the NON-EMPTY blocks from the block-end bitmap alone (rho(i) =
// block ends before position i; per tile: its block ends, tcnt -> scan ->
// trank; k_block_ends counts them) and takes the tetramer from the list of non-empty blocks (tnz[rho],
// one table row per run of equal rho: the wave's loads coalesce); the G side
// hashes G_tet as it is, so it needs nothing from F and runs from the start
// of the load (k_hash_g).
// tnz[r] = the r-th non-empty tetramer (rho: exclusive scan of the flags)
__global__ void k_tnz(const unsigned long long* __restrict__ rho, uint32_t* __restrict__ tnz) {
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < kNTetramers; t += gridDim.x * blockDim.x)
        if (rho[t + 1] > rho[t]) tnz[rho[t]] = (uint32_t)t;
}

// Pass 1's histogram over F (kept records only) + the u16 protein column +
// each entry's distance to its run end (D) + the tile's first run end
// (ftail, absolute) + (code, nullable) the member codes of k_fcode for every
// entry, kept or not (the row kernel's members are any genome): the tile's
// genome ids are in registers anyway, so the codes cost one store per entry
// here against a 0.49 ms pass over Fg at 10k.  Every global load is issued
// before the first store.
template <int DB, int NT>
__global__ __launch_bounds__(NT) void k_fends_hist(const int32_t* __restrict__ Fp, const int32_t* __restrict__ Fg,
                                                   const uint32_t* __restrict__ bend, int64_t n, uint32_t P,
                                                   int32_t g_lo, int32_t g_hi, uint32_t mask,
                                                   uint16_t* __restrict__ fp16, uint32_t* __restrict__ D,
                                                   uint32_t* __restrict__ hist, uint32_t* __restrict__ ftail,
                                                   uint32_t* __restrict__ ltail,
                                                   const unsigned long long* __restrict__ trank,
                                                   const uint32_t* __restrict__ tnz, uint64_t seed,
                                                   uint64_t seed2, unsigned long long* __restrict__ hpart,
                                                   uint32_t* __restrict__ code) {
    constexpr int BINS = 1 << DB, kTile = NT * kSortItems, kChunks = kTile / 64;
    static_assert(kChunks <= 64, "one wave ballots the tile's chunks");
    __shared__ uint32_t h[BINS];
    __shared__ uint16_t sp[kTile + 1];              // protein of every position (+ the next tile's first)
    __shared__ uint32_t sb[kTile / 32];             // block-end bits of the tile
    __shared__ unsigned long long tm[kChunks];      // run-end bits
    __shared__ uint8_t nextw[kChunks];              // next chunk holding a run end
    __shared__ uint32_t first, last;
    __shared__ uint32_t wpre[kTile / 32];          // block ends before each word of the tile (hpart)
    __shared__ uint64_t hw[2 * (NT / 64)];
    __shared__ uint32_t stz[64];                   // the tile's first 64 tetramers (hpart)
    const int tid = threadIdx.x, lane = tid & 63;
    const int64_t tile = blockIdx.x, t0 = tile * kTile;
    const unsigned long long rb = hpart ? trank[tile] : 0ull;
    if (hpart && tid < 64) {
        const unsigned long long ix = rb + (unsigned long long)tid;
        stz[tid] = tnz[ix < (unsigned long long)kNTetramers ? (int64_t)ix : (int64_t)kNTetramers - 1];
    }
    for (int b = tid; b < BINS; b += NT) h[b] = 0u;
    // tile-relative 32-bit positions (rn: the tile's entries, uniform) -- the
    // VALU-bound kernel (~110 VALU per entry with 64-bit positions) keeps its
    // address arithmetic in the scalar base
    // (raw buffer loads / stores over the tile: out-of-range positions read
    // 0 and write nothing, so no clamps or branches per entry)
    const int rn = (int)min<int64_t>(kTile, n - t0);
    const rsrc_t r_p = mk_rsrc(Fp + t0, (uint64_t)rn * 4u), r_g = mk_rsrc(Fg + t0, (uint64_t)rn * 4u);
    const rsrc_t r_fp16 = mk_rsrc(fp16 ? fp16 + t0 : nullptr, fp16 ? (uint64_t)rn * 2u : 0u);
    const rsrc_t r_code = mk_rsrc(code ? code + t0 : nullptr, code ? (uint64_t)rn * 4u : 0u);
    const uint32_t gspan = (uint32_t)(g_hi - g_lo);
    int32_t p[kSortItems], g[kSortItems];
#pragma unroll
    for (int k = 0; k < kSortItems; ++k) {
        p[k] = (int32_t)bld_u32(r_p, (uint32_t)(k * NT + tid) * 4u, 0u);
        g[k] = (int32_t)bld_u32(r_g, (uint32_t)(k * NT + tid) * 4u, 0u);
    }
    const int nwt = (int)min<int64_t>(kTile / 32, ((n + 31) >> 5) - t0 / 32);  // bend words of the tile
    const uint32_t bw = tid < nwt ? bend[t0 / 32 + tid] : 0u;
    const int32_t p_next = t0 + kTile < n ? Fp[t0 + kTile] : -1;
    __syncthreads();  // (h cleared)
#pragma unroll
    for (int k = 0; k < kSortItems; ++k) {
        const int r = k * NT + tid;
        sp[r] = (uint16_t)p[k];
        if (fp16) __builtin_amdgcn_raw_buffer_store_b16((uint16_t)p[k], r_fp16, r * 2, 0, 0);
        if (code) {
            const uint32_t b = (uint32_t)g[k];
            __builtin_amdgcn_raw_buffer_store_b32(((b >> 1) << 7) | ((b & 1u) << 4), r_code, r * 4, 0, 0);
        }
        if (r < rn && (uint32_t)(g[k] - g_lo) < gspan) atomicAdd(&h[((uint32_t)g[k] * P + (uint32_t)p[k]) & mask], 1u);
    }
    if (tid < kTile / 32) sb[tid] = bw;
    if (tid == 0) sp[kTile] = (uint16_t)p_next;  // (-1: 0xFFFF, no protein id)
    if (hpart && tid < kTile / 32) {  // exclusive prefix of the words' block ends (two waves)
        const uint32_t pc = __popc(bw);
        uint32_t inc = pc;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t u = __shfl_up(inc, o, 64);
            if (lane >= o) inc += u;
        }
        wpre[tid] = inc - pc;
    }
    __syncthreads();
    if (hpart) {  // the F side of the both-given check: h(g * P + p, t) over the kept entries
        const uint32_t carry = wpre[63] + __popc(sb[63]);  // (ends in the tile's first 64 words)
        uint64_t acc = 0, acc2 = 0;
#pragma unroll
        for (int k = 0; k < kSortItems; ++k) {
            const int r = k * NT + tid;
            const uint32_t w = (uint32_t)r >> 5;
            const uint32_t rl = wpre[w] + (w >= 64 ? carry : 0u) + __popc(sb[w] & ((1u << (r & 31)) - 1u));
            const uint32_t t = rl < 64u ? stz[rl] : tnz[r < rn ? (uint32_t)rb + rl : 0u];
            if (r < rn && (uint32_t)(g[k] - g_lo) < gspan) {
                const uint32_t key = (uint32_t)g[k] * P + (uint32_t)p[k];
                acc += member_hash(seed, key, t);
                acc2 += member_hash_b(seed2, key, t);
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            acc += __shfl_down(acc, o, 64);
            acc2 += __shfl_down(acc2, o, 64);
        }
        // the tile's sums to hpart[tile] (k_tail_suffix adds them up: one
        // atomic per wave into one address serialised at ~10 ns each)
        if (lane == 0) {
            hw[2 * (tid >> 6)] = acc;
            hw[2 * (tid >> 6) + 1] = acc2;
        }
        __syncthreads();
        if (tid < 2) {
            uint64_t x = 0;
#pragma unroll
            for (int w = 0; w < NT / 64; ++w) x += hw[2 * w + tid];
            hpart[2 * tile + tid] = x;
        }
    }
#pragma unroll 1
    for (int k = 0; k < kSortItems; ++k) {  // run ends, one 64-position chunk per (wave, k) ballot
        const int r = k * NT + tid;
        const bool tail = r < rn && (t0 + r == n - 1 || ((sb[r >> 5] >> (r & 31)) & 1u) || sp[r] != sp[r + 1]);
        const unsigned long long m = __ballot(tail);
        if (lane == 0) tm[r >> 6] = m;
    }
    __syncthreads();
    if (tid < kChunks) {
        const unsigned long long b =
            __ballot(tm[tid] != 0ull) & (kChunks == 64 ? ~0ull : ((1ull << kChunks) - 1ull));
        const unsigned long long after = tid == 63 ? 0ull : b >> (tid + 1);
        nextw[tid] = after ? (uint8_t)(tid + 1 + __builtin_ctzll(after)) : (uint8_t)kChunks;
        if (tid == 0) first = b ? (uint32_t)(__builtin_ctzll(b) * 64 + __builtin_ctzll(tm[__builtin_ctzll(b)])) : kNoTail;
        if (tid == 0) {
            const int wl = b ? 63 - __builtin_clzll(b) : 0;
            last = b ? (uint32_t)(wl * 64 + 63 - __builtin_clzll(tm[wl])) : kNoTail;
        }
    }
    __syncthreads();
    for (int b = tid; b < BINS; b += NT) hist[tile * BINS + b] = h[b];
    const rsrc_t r_d = mk_rsrc(D + t0, (uint64_t)rn * 4u);
    if (tid == 0) {
        ftail[tile] = first == kNoTail ? kNoTail : (uint32_t)(t0 + first);
        ltail[tile] = last;  // (tile-relative: the tile's open run starts after it)
    }
#pragma unroll
    for (int k = 0; k < kSortItems; ++k) {
        const uint32_t r = (uint32_t)(k * NT + tid);
        const uint32_t w = r >> 6;
        const unsigned long long m = tm[w] & (~0ull << (r & 63u));
        uint32_t d = kOpenRun;
        if (m) {
            d = (w << 6) + (uint32_t)__builtin_ctzll(m) + 1u - r;
        } else {
            const uint32_t w2 = nextw[w];
            if (w2 < (uint32_t)kChunks) d = (w2 << 6) + (uint32_t)__builtin_ctzll(tm[w2]) + 1u - r;
        }
        __builtin_amdgcn_raw_buffer_store_b32(d, r_d, (int)(r * 4u), 0, 0);
    }
}

// ntail[T] = the first run end after tile T: ftail of the next tile that
// has one (ftail grows with T; a tile without a run end lies inside a run of
// more than 4096 entries, and runs span < 2^21 entries, so a thread looks at
// no more than 513 tiles -- one, almost always)
__global__ void k_tail_suffix(const uint32_t* __restrict__ ftail, int64_t ntiles, uint32_t* __restrict__ ntail) {
    for (int64_t T = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; T < ntiles; T += (int64_t)gridDim.x * blockDim.x) {
        int64_t u = T + 1;
        while (u < ntiles && ftail[u] == kNoTail) ++u;
        ntail[T] = u < ntiles ? ftail[u] : kNoTail;
    }
}

// The open runs' distances: in tile T the entries after its last run end
// (ltail) belong to a run that ends at the first run end after the tile
// (ntail[T]).  One wave per tile.
__global__ __launch_bounds__(256) void k_fix_open(const uint32_t* __restrict__ ltail, const uint32_t* __restrict__ ntail,
                                                  int64_t ntiles, int64_t n, uint32_t* __restrict__ D) {
    const int lane = threadIdx.x & 63;
    for (int64_t T = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64; T < ntiles;
         T += (int64_t)gridDim.x * blockDim.x / 64) {
        const int64_t t0 = T * kEndsTile;
        const uint32_t lt = ltail[T];
        const int64_t b = t0 + (lt == kNoTail ? 0 : (int64_t)lt + 1), e = min(n, t0 + kEndsTile);
        const int64_t end = (int64_t)ntail[T] + 1;
        for (int64_t i = b + lane; i < e; i += 64) D[i] = (uint32_t)(end - i);
    }
}

// sum[0] += sum of part[2 k], sum[2] += sum of part[2 k + 1] (the check's
// per-tile F sums; one atomic pair per workgroup)
__global__ __launch_bounds__(256) void k_sum_pairs(const unsigned long long* __restrict__ part, int64_t n,
                                                   unsigned long long* __restrict__ sum) {
    __shared__ uint64_t ws[2 * 4];
    uint64_t a = 0, b = 0;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        a += part[2 * k];
        b += part[2 * k + 1];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        a += __shfl_down(a, o, 64);
        b += __shfl_down(b, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        ws[2 * (threadIdx.x >> 6)] = a;
        ws[2 * (threadIdx.x >> 6) + 1] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicAdd(sum, (unsigned long long)(ws[0] + ws[2] + ws[4] + ws[6]));
        atomicAdd(sum + 2, (unsigned long long)(ws[1] + ws[3] + ws[5] + ws[7]));
    }
}

// The G side of the run-end sort's check: sum over the lists (g, p), g in
// [g_lo, g_hi), of h(g * P + p, G_tet) in two lanes.  A wave takes 64
// consecutive lists -- one contiguous range of G_tet -- and streams it eight
// entries per lane in flight, each entry's list found by walking the lists'
// starts (LDS) forward from the lane's previous entry; one atomic pair per
// workgroup.  Reads nothing of F: it runs beside the whole sort.
__global__ __launch_bounds__(256) void k_hash_g(const int64_t* __restrict__ G_off, const int32_t* __restrict__ G_tet,
                                                int32_t P, int32_t g_lo, int32_t g_hi, uint64_t seed, uint64_t seed2,
                                                unsigned long long* __restrict__ sum) {
    __shared__ uint32_t pre[4][65];
    __shared__ uint64_t ws[2 * 4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t* pr = pre[wv];
    const int64_t l_lo = (int64_t)g_lo * P, l_hi = (int64_t)g_hi * P, nch = (l_hi - l_lo + 63) / 64;
    uint64_t a = 0, b = 0;
    for (int64_t ch = (int64_t)blockIdx.x * 4 + wv; ch < nch; ch += (int64_t)gridDim.x * 4) {
        const int64_t L0 = l_lo + ch * 64;
        const int nl = (int)min<int64_t>(64, l_hi - L0);
        const int64_t E0 = G_off[L0];
        pr[lane] = (uint32_t)(G_off[L0 + min(lane, nl)] - E0);  // (lanes >= nl: the range's end)
        if (lane == 0) pr[64] = (uint32_t)(G_off[L0 + nl] - E0);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t total = pr[64];
        const int32_t* gt = G_tet + E0;
        int j = 0;
        for (uint32_t f0 = 0; f0 < total; f0 += 8 * 64) {
            int32_t t[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) t[u] = __builtin_nontemporal_load(gt + min(f0 + (uint32_t)(u * 64 + lane), total - 1u));
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const uint32_t f = f0 + (uint32_t)(u * 64 + lane);
                if (f < total) {
                    while (pr[j + 1] <= f) ++j;
                    const uint32_t key = (uint32_t)(L0 + j);  // = g * P + p
                    a += member_hash(seed, key, (uint32_t)t[u]);
                    b += member_hash_b(seed2, key, (uint32_t)t[u]);
                }
            }
        }
        __builtin_amdgcn_wave_barrier();  // pr is rewritten by the next chunk
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        a += __shfl_down(a, o, 64);
        b += __shfl_down(b, o, 64);
    }
    if (lane == 0) {
        ws[2 * wv] = a;
        ws[2 * wv + 1] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicAdd(sum, (unsigned long long)(ws[0] + ws[2] + ws[4] + ws[6]));
        atomicAdd(sum + 2, (unsigned long long)(ws[1] + ws[3] + ws[5] + ws[7]));
    }
}

// F entry i -> pass 1's record, its distance to its run end from D
struct SrcFEnds {
    static constexpr bool kFilter = true;
    const int32_t* Fp;
    const int32_t* Fg;
    const uint32_t* D;
    uint32_t P;
    int kb;
    int32_t g_lo, g_hi;
    bool compact;  // few records kept: k_sort_scatter packs them before ranking
    __device__ __forceinline__ bool keep(uint64_t r) const { return !(r >> 63); }
    __device__ __forceinline__ uint64_t rec(int64_t i, int32_t g, int32_t p, uint32_t d) const {
        return (uint64_t)((uint32_t)g * P + (uint32_t)p) | ((uint64_t)(i & (kEndsTile - 1)) << kb) |
               ((uint64_t)(d & 0x1FFFFFu) << (kb + 12)) | ((uint64_t)(g < g_lo || g >= g_hi) << 63);
    }
    __device__ __forceinline__ uint64_t load(int64_t i) const { return rec(i, Fg[i], Fp[i], D[i]); }
    __device__ __forceinline__ uint64_t load_nt(int64_t i) const {
        return rec(i, __builtin_nontemporal_load(Fg + i), __builtin_nontemporal_load(Fp + i),
                   __builtin_nontemporal_load(D + i));
    }
};

// pass 1's records out: the second digit, the F index, the distance to its run end
struct DstRecsEnds {
    uint64_t* r;
    int kb, db;
    static constexpr int kWH = kSortItems;
    static constexpr bool kSum = false;
    struct Aux {};
    __device__ __forceinline__ Aux fetch(int64_t, uint64_t) const { return {}; }
    __device__ __forceinline__ uint64_t store(int64_t pos, uint64_t v, Aux, int64_t t0) const {
        const int hb = kb - db;
        const uint64_t key = v & ((1ull << kb) - 1ull);
        const uint64_t i = (uint64_t)t0 + ((v >> kb) & 0xFFFull);
        const uint64_t dist = (v >> (kb + 12)) & 0x1FFFFFull;
        r[pos] = (key >> db) | (i << hb) | (dist << (hb + 32));
        return 0;
    }
};

// pass 2 (G order): G_pe = (the F index, its run end), one 8-B store per
// entry -- a tile's digit run is one contiguous 32-B piece of one array
// instead of two 16-B pieces of G_pos and G_end (2.06 ms for the pass at 10k
// with the two arrays)
struct DstGposEnds {
    uint2* G_pe;
    int hb;
    static constexpr int kWH = kSortItems;
    static constexpr bool kSum = false;
    struct Aux {};
    __device__ __forceinline__ Aux fetch(int64_t, uint64_t) const { return {}; }
    __device__ __forceinline__ uint64_t store(int64_t pos, uint64_t v, Aux, int64_t) const {
        const uint32_t i = (uint32_t)(v >> hb), dist = (uint32_t)(v >> (hb + 32));
        G_pe[pos] = make_uint2(i, i + dist);
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
// bit 6 direct stores without the LDS reorder, bit 3 no global stores
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
    __shared__ uint32_t s_tn;  // records of the tile that pass Src::keep
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
        // Src::kFilter with few records kept (a rank's genomes, pfaai_load_rows):
        // each wave first packs its kept records, in order, into its first
        // rounds (through its own eighth of the LDS tile, free until the
        // reorder below), so the ranking ballots run over ceil(kept / 64)
        // rounds instead of kSortItems; dropped slots get the drop bit
        int kact = kSortItems;
        if constexpr (Src::kFilter) {
            if (src.compact) {
                uint64_t* ws = srt + wid * (kSortItems * 64);
                uint32_t cw = 0;
#pragma unroll
                for (int k = 0; k < kSortItems; ++k) {
                    const bool valid = t0 + (wid * kSortItems + k) * 64 + lane < n && src.keep(rec[k]);
                    const uint64_t m = __ballot(valid);
                    if (valid) ws[cw + (uint32_t)__popcll(m & lt)] = rec[k];
                    cw += (uint32_t)__popcll(m);
                }
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int k = 0; k < kSortItems; ++k) {
                    const uint32_t j = (uint32_t)(k * 64 + lane);
                    rec[k] = j < cw ? ws[j] : (1ull << 63);
                }
                kact = (int)((cw + 63u) >> 6);
            }
        }
        // ranking: peers = the valid lanes with this item's digit.  Two
        // forms.  kPairRank (the run-end sort's first pass, SrcFEnds): peers
        // accumulated as its complement, the lanes that differ in some bit --
        // per bit the bit as 0 / -1 (one v_bfe_i32), its ballot, and diff |=
        // ballot ^ bit in each half (one v_bitop3 each), 4 VALU per bit where
        // peers &= on ? m : ~m takes 8 (a 0 / -1 select, two xors, two ands,
        // the bit extracted twice); two items at a time, their bits
        // interleaved (a ballot's SGPR read by the next VALU op waits
        // otherwise).  Pass 1 of the 10k load 2.13 -> 1.85 ms; the same form
        // in pass 2 (SrcRecs -> DstGposEnds) measured 1.93 -> 2.17-2.21 ms,
        // so the other sources keep the first form.
        constexpr bool kPairRank = Src::kFilter;
        uint16_t lr[kSortItems];
        static_assert(kSortItems % 2 == 0, "items in pairs");
        if constexpr (kPairRank) {
#pragma unroll
        for (int k = 0; k < kSortItems; k += 2) {
            if (k >= kact) {  // (wave-uniform; kact is odd only when the wave packed its kept records)
                lr[k] = 0;
                lr[k + 1] = 0;
                continue;
            }
            bool valid[2];
            uint32_t d[2], dlo[2], dhi[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                valid[u] = k + u < kact && t0 + (wid * kSortItems + k + u) * 64 + lane < n && src.keep(rec[k + u]);
                d[u] = sort_digit(rec[k + u], shift, mask);
                const uint64_t vm = __ballot(valid[u]);
                dlo[u] = ~(uint32_t)vm;
                dhi[u] = ~(uint32_t)(vm >> 32);
            }
#pragma unroll
            for (int bit = 0; bit < DB; ++bit) {  // (bits above the mask are 0 in every lane: same ballot)
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    uint32_t rep = (uint32_t)__builtin_amdgcn_sbfe((int)d[u], bit, 1);
                    asm("" : "+v"(rep));  // (opaque: the ballot compares rep, not a re-shifted d)
                    const uint64_t m = __ballot(rep != 0u);
                    // dx | (m ^ rep): LUT 0xF6 over (dx, m, rep)
                    dlo[u] = __builtin_amdgcn_bitop3_b32(dlo[u], (uint32_t)m, rep, 0xF6);
                    dhi[u] = __builtin_amdgcn_bitop3_b32(dhi[u], (uint32_t)(m >> 32), rep, 0xF6);
                }
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const uint64_t peers = ~(((uint64_t)dhi[u] << 32) | dlo[u]);
                const uint32_t r = (uint32_t)__popcll(peers & lt), c = (uint32_t)__popcll(peers);
                const uint32_t base = valid[u] ? wc[d[u]] : 0u;
                lr[k + u] = (uint16_t)(base + r);
                if (valid[u] && r + 1 == c) wc[d[u]] = (uint16_t)(base + c);  // the group's last lane advances the counter
            }
        }
        } else {
#pragma unroll
        for (int k = 0; k < kSortItems; ++k) {
            if (k >= kact) {  // (wave-uniform)
                lr[k] = 0;
                continue;
            }
            const bool valid = t0 + (wid * kSortItems + k) * 64 + lane < n && src.keep(rec[k]);
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
        if constexpr ((VAR & 64) != 0) {
            // direct stores (diagnostics A/B): each record from its registers
            // to gbase[d] + (its rank among the tile's records of digit d) --
            // no digit totals scan, no LDS reorder, 8-B stores spread over
            // the tile's digit runs instead of one contiguous tile
            (void)tot;
            __syncthreads();
#pragma unroll
            for (int k = 0; k < kSortItems; ++k) {
                const uint32_t d = sort_digit(rec[k], shift, mask);
                const uint32_t pos = gbase[d] + cnt[wid * BINS + d] + lr[k];
                const bool ok = k < kact && t0 + (wid * kSortItems + k) * 64 + lane < n && src.keep(rec[k]);
                if ((VAR & 8) == 0 && ok) hsum += dst.store(pos, rec[k], dst.fetch(pos, rec[k]), t0);
            }
            __syncthreads();  // the counters and bases are rewritten by the next tile
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
            continue;
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
            if (b < BINS) {
                lstart[b] = off;
                gbase[b] -= off;  // the write phase's pos = gbase[d] + lp: one LDS read a record, not two
            }
            off += tot[q];
        }
        if (tid == NT - 1) s_tn = off;  // (the tile's records, all digits)
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
                if (t0 + (wid * kSortItems + k) * 64 + lane < n && src.keep(rec[k])) srt[slot[k]] = rec[k];
        }
        __syncthreads();
        // write the tile in digit order: each digit's run is contiguous in the output
        // (positions are < 2^32: n <= 2^32 - 64; records re-read from LDS for the stores)
        const int tn = Src::kFilter ? (int)s_tn : (int)((n - t0) < kTile ? (n - t0) : kTile);
        // (unconditional reads at positions clamped into the tile: no wait per item)
#pragma unroll
        for (int h = 0; h < kSortItems; h += kWH) {  // kWH records per thread in flight
            uint32_t pos[kWH];
            uint64_t val[kWH];
            typename Dst::Aux aux[kWH];
#pragma unroll
            for (int k = 0; k < kWH; ++k) {
                const int lp = min(tid + (h + k) * NT, max(tn - 1, 0));
                val[k] = srt[lp];
            }
#pragma unroll
            for (int k = 0; k < kWH; ++k) {
                const int lp = min(tid + (h + k) * NT, max(tn - 1, 0));
                const uint32_t d = sort_digit(val[k], shift, mask);
                pos[k] = gbase[d] + (uint32_t)lp;  // (gbase[d] >= lstart[d]: the tile's records before digit d precede it)
            }
#pragma unroll
            for (int k = 0; k < kWH; ++k) aux[k] = dst.fetch(pos[k], val[k]);
#pragma unroll
            for (int k = 0; k < kWH; ++k) {
                const int lp = tid + (h + k) * NT;
                if ((VAR & 8) == 0 && lp < tn) hsum += dst.store(pos[k], val[k], aux[k], t0);
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
                                              unsigned long long* __restrict__ sums, int32_t g_lo,
                                              int32_t g_hi) {
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
                const int64_t p = q / n_ids, g = q - p * n_ids, L = g * P + p;
                const int64_t b = G_off[L], e = G_off[L + 1];
                lb[tid] = b;
                row[tid] = p * kNTetramers;
                lid[tid] = (uint32_t)L;
                len = q0 + tid < n_lists && g >= g_lo && g < g_hi ? (uint32_t)(e - b) : 0u;
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
                        hm2 += member_hash_b(seed2, li[u], (uint32_t)t[u]);
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
