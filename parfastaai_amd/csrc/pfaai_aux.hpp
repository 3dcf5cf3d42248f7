// pfaai_aux.hpp -- the non-template kernels of the engine's support passes
// (work-list compaction counts, radix-sort histograms, the F build of
// pfaai_build_f, rowptr, the three-phase scan).  Included by pfaai_hip.hip
// only: the row-kernel translation units (pfaai_rows_m*.hip) share
// pfaai_kernels.hpp, whose kernels are all templates.
#pragma once
#include "pfaai_kernels.hpp"

namespace pfaai {

// entries of rows [row_begin, row_end) per tetramer block (compaction offsets)
__global__ __launch_bounds__(kTetraThreads) void k_count_t(Dev d, int64_t row_begin, int64_t row_end,
                                                           uint32_t* __restrict__ cnt_t) {
    __shared__ uint32_t wsum[kTetraThreads / 64];
    const int tid = threadIdx.x;
    for (int t = blockIdx.x; t < kNTetramers; t += gridDim.x) {
        const int64_t s = d.Lp[t], e = d.Lp[t + 1];
        uint32_t c = 0;
        for (int64_t i = s + tid; i < e; i += kTetraThreads) {
            const int32_t row = d.row_of[d.Fg[i]];
            c += (row >= row_begin && row < row_end) ? 1u : 0u;
        }
        c = wave_sum_u32_fwd(c);
        if ((tid & 63) == 0) wsum[tid >> 6] = c;
        __syncthreads();
        if (tid == 0) {
            uint32_t tot = 0;
            for (int w = 0; w < kTetraThreads / 64; ++w) tot += wsum[w];
            cnt_t[t] = tot;
        }
        __syncthreads();
    }
}


__global__ __launch_bounds__(kRsThreads) void k_rs_hist(const uint32_t* __restrict__ keys, int64_t n, int shift,
                                                        uint32_t* __restrict__ hist, int64_t ntiles) {
    __shared__ uint32_t h[kRsBins];
    const int tid = threadIdx.x;
    h[tid] = 0u;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * kRsTile;
#pragma unroll 4
    for (int r = 0; r < kRsRounds; ++r) {
        const int64_t j = base + r * kRsThreads + tid;
        if (j < n) atomicAdd(&h[(keys[j] >> shift) & (kRsBins - 1)], 1u);
    }
    __syncthreads();
    hist[(int64_t)tid * ntiles + blockIdx.x] = h[tid];
}


// ---------------------------------------------------------------------------
// K-F: F construction (pfaai_build_f).  The reference builds F with an SQL
// UNION ALL + ORDER BY over the `<p>_tetras` tables (scp_db.hpp:161-216,
// ds_helper.hpp:126-162) and Lc with per-protein range queries (82-122).
// Here: (protein, genome, tetramer) triples -> key t * P + p, record (p, g);
// the stable LSD radix sort above (k_rs_hist / k_rs_scatter) orders them by
// (t, p) and, being stable, keeps each protein's ascending genome order, so
// the sorted records are F by (tetramer, protein, genome).  Lc and T are
// counted on the way in.
// ---------------------------------------------------------------------------
__global__ void k_f_keys(const int32_t* __restrict__ prot, const int32_t* __restrict__ genome,
                         const int32_t* __restrict__ tetra, int64_t n, int32_t P, int32_t n_genome,
                         uint32_t* __restrict__ keys, uint2* __restrict__ recs, uint32_t* __restrict__ lc,
                         int32_t* __restrict__ T) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t p = prot[i], g = genome[i], t = tetra[i];
        keys[i] = (uint32_t)t * (uint32_t)P + (uint32_t)p;
        recs[i] = make_uint2((uint32_t)p, (uint32_t)g);
        atomicAdd(&lc[t], 1u);
        if (T) atomicAdd(&T[(int64_t)p * n_genome + g], 1);
    }
}

// sorted (p, g) records -> the two F columns
__global__ void k_f_split(const uint2* __restrict__ recs, int64_t n, int32_t* __restrict__ fp,
                          int32_t* __restrict__ fg) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint2 r = recs[i];
        fp[i] = (int32_t)r.x;
        fg[i] = (int32_t)r.y;
    }
}

// rowptr[k] = first sorted position with key >= k  (k in [0, K]).
__global__ void k_rowptr(const uint32_t* __restrict__ keys, int64_t n, int64_t K,
                         unsigned long long* __restrict__ rowptr) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const int64_t k = keys[j];
    const int64_t kq = keys[j > 0 ? j - 1 : 0];  // (unconditional: no wait at a branch)
    const int64_t kp = j > 0 ? kq : -1;
    for (int64_t x = kp + 1; x <= k; ++x) rowptr[x] = (unsigned long long)j;
    if (j == n - 1)
        for (int64_t x = k + 1; x <= K; ++x) rowptr[x] = (unsigned long long)n;
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


}  // namespace pfaai
