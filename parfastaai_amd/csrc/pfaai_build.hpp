// pfaai_build.hpp -- the two orientations of the SCP membership at load time.
//
// The SCP database stores every (tetramer, protein, genome) membership twice
// (scp_db.hpp:37-55): `<p>_tetras` (tetramer -> genome list: F, ordered by
// (tetramer, protein, genome), ds_helper.hpp:126-162) and `<p>_genomes`
// (genome -> tetramer list: G, (genome, protein)-major, ascending tetramers).
// The row kernels need both: G to walk a row genome's own tetramers, F for
// the run of every (tetramer, protein).  Whichever one the caller holds, the
// other is built here with the stable LSD radix sort of pfaai_kernels.hpp
// (k_rs_hist / k_rs_scatter, 8-bit digits):
//   G from F   key = genome * P + protein of each F entry, record (tetramer,
//              genome); F is sorted by tetramer, so the stable sort leaves
//              every (genome, protein) list in ascending tetramer order.
//   F from G   key = tetramer * P + protein of each G entry, record (protein,
//              genome); G is genome-major, so the stable sort leaves every
//              (tetramer, protein) run in ascending genome order -- exactly
//              the reference's F (the UNION ALL ... ORDER BY of
//              scp_db.hpp:161-216).  Lc is counted on the way in.
// When both are given, k_g_check proves that G covers F.
#pragma once
#include "pfaai_kernels.hpp"

namespace pfaai {

// G-from-F keys: one workgroup per tetramer block (grid-stride over blocks);
// record (tetramer, F index).
__global__ __launch_bounds__(256) void k_gkeys_from_f(const int64_t* __restrict__ Lp, const int32_t* __restrict__ Fp,
                                                      const int32_t* __restrict__ Fg, int32_t P,
                                                      uint32_t* __restrict__ keys, uint2* __restrict__ recs) {
    for (int t = blockIdx.x; t < kNTetramers; t += gridDim.x) {
        const int64_t e = Lp[t + 1];
        for (int64_t i = Lp[t] + threadIdx.x; i < e; i += blockDim.x) {
            const int32_t g = Fg[i];
            keys[i] = (uint32_t)g * (uint32_t)P + (uint32_t)Fp[i];
            recs[i] = make_uint2((uint32_t)t, (uint32_t)i);
        }
    }
}

// sorted (tetramer, F index) records -> G_tet and (if wanted) G_pos, the F
// index of every G entry
__global__ void k_gtet_split(const uint2* __restrict__ recs, int64_t n, int32_t* __restrict__ G_tet,
                             uint32_t* __restrict__ G_pos) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint2 r = recs[i];
        G_tet[i] = (int32_t)r.x;
        if (G_pos) G_pos[i] = r.y;
    }
}

// F from G: sorted keys (tetramer * P + protein) and (genome, G index)
// records -> the F columns, and G_pos[G index] = F index (if wanted)
__global__ void k_f_split_pos(const uint32_t* __restrict__ keys, const uint2* __restrict__ recs, int64_t n, int32_t P,
                              int32_t* __restrict__ fp, int32_t* __restrict__ fg, uint32_t* __restrict__ G_pos) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint2 r = recs[i];
        fp[i] = (int32_t)(keys[i] % (uint32_t)P);
        fg[i] = (int32_t)r.x;
        if (G_pos) G_pos[r.y] = (uint32_t)i;
    }
}

// F-from-G keys: one wave per (genome, protein) list, lanes over its entries;
// record (genome, G index).
__global__ __launch_bounds__(256) void k_fkeys_from_g(const int64_t* __restrict__ G_off, const int32_t* __restrict__ G_tet,
                                                      int64_t n_lists, int32_t P, uint32_t* __restrict__ keys,
                                                      uint2* __restrict__ recs, uint32_t* __restrict__ lc) {
    const int lane = threadIdx.x & 63;
    const int64_t waves = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t L = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); L < n_lists; L += waves) {
        const uint32_t g = (uint32_t)(L / P), p = (uint32_t)(L % P);
        const int64_t e = G_off[L + 1];
        for (int64_t k = G_off[L] + lane; k < e; k += 64) {
            const uint32_t t = (uint32_t)G_tet[k];
            keys[k] = t * (uint32_t)P + p;
            recs[k] = make_uint2(g, (uint32_t)k);
            atomicAdd(&lc[t], 1u);
        }
    }
}

// u16 protein ids of F (k_blk's run detection reads 8 per 16-B load)
__global__ void k_fp16(const int32_t* __restrict__ Fp, int64_t n, uint16_t* __restrict__ Fp16) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        Fp16[i] = (uint16_t)Fp[i];
}

// (G_pos, G_end) -> the interleaved G_pe the WK 3 walks read (the fallback
// builds, whose G_pos and G_end come from different kernels)
__global__ void k_pack_pe(const uint32_t* __restrict__ pos, const uint32_t* __restrict__ end, int64_t n,
                          uint2* __restrict__ pe) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        pe[i] = make_uint2(pos[i], end[i]);
}

// Member codes of F for k_rows_pl's WK 3 member scatter: genome b as
// (b >> 1) << 7 | (b & 1) << 4, so that the counter word's LDS byte offset
// is code >> 5 and the u16 half's increment is 1 << code (a VALU shift reads
// the low 5 bits: 0 or 16) -- one VALU op per member fewer than from b.
// n + 16 entries (the padding reads 0, like Fg's).
__global__ void k_fcode(const int32_t* __restrict__ Fg, int64_t n, uint32_t* __restrict__ code) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n + 16; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t b = i < n ? (uint32_t)Fg[i] : 0u;
        code[i] = i < n ? ((b >> 1) << 7) | ((b & 1u) << 4) : 0u;
    }
}

// Both F and G given: G must hold every membership of F, and an entry
// (genome g, protein p, tetramer t) of G that is not in F is allowed only
// where F has no run (t, p) at all (e.g. the -r path: G holds every tetramer
// of both DBs, F only those in both, scp_db.hpp:459-466; such an entry meets

// Words of a and b that differ, added to *ne (the both-given check when G and
// the G built from F must be equal: a plain streaming compare).
__global__ __launch_bounds__(256) void k_count_ne(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b,
                                                  int64_t n, unsigned long long* __restrict__ ne) {
    uint32_t k = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        k += a[i] != b[i];
    k = wave_sum_u32_fwd(k);
    if ((threadIdx.x & 63) == 0 && k) atomicAdd(ne, (unsigned long long)k);
}

// an empty run in the row kernels).  Binary search for (p, g) in F's
// tetramer block, sorted by (protein, genome); *found counts the entries F
// holds (== |F| when G covers F, lists being strictly ascending sets).  One
// wave per list.
__global__ __launch_bounds__(256) void k_g_check(const int64_t* __restrict__ Lp, const int32_t* __restrict__ Fp,
                                                 const int32_t* __restrict__ Fg, const int64_t* __restrict__ G_off,
                                                 const int32_t* __restrict__ G_tet, int64_t n_lists, int32_t P,
                                                 int* __restrict__ err, unsigned long long* __restrict__ found) {
    const int lane = threadIdx.x & 63;
    const int64_t waves = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t L = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); L < n_lists; L += waves) {
        const int32_t g = (int32_t)(L / P), p = (int32_t)(L % P);
        const uint64_t key = ((uint64_t)(uint32_t)p << 32) | (uint32_t)g;
        const int64_t e = G_off[L + 1];
        bool bad = false;
        uint32_t hit = 0;
        for (int64_t k = G_off[L] + lane; k < e; k += 64) {
            const int32_t t = G_tet[k];
            const int64_t start = Lp[t], end = Lp[t + 1];
            int64_t lo = start, hi = end;
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                const uint64_t m = ((uint64_t)(uint32_t)Fp[mid] << 32) | (uint32_t)Fg[mid];
                if (m < key) lo = mid + 1; else hi = mid;
            }
            const bool in_run = lo < end && Fp[lo] == p;
            if (in_run && Fg[lo] == g) {
                ++hit;
            } else {  // not a member: only allowed where F has no run (t, p)
                bad |= in_run || (lo > start && Fp[lo - 1] == p);
            }
        }
        if (bad) atomicOr(err, 1);
        hit = wave_sum_u32_fwd(hit);
        if (lane == 0 && hit) atomicAdd(found, (unsigned long long)hit);
    }
}

}  // namespace pfaai
