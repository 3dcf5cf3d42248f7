// pfaai_util.hpp -- device helpers shared by the row kernels: raw buffer
// loads, wave scans, run-line pruning, exact small-integer division.
#pragma once
#include "pfaai_kernels.hpp"

namespace pfaai {

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
__device__ __forceinline__ uint2 bld_u64(rsrc_t r, uint32_t voff, uint32_t soff) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, (int)soff, 0);
    return make_uint2((uint32_t)v[0], (uint32_t)v[1]);
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
// min_len: a full run of one member is A alone (no partner), so runs of
// length <= 1 are skipped; a column-window sub-run (k_blk<true>) may omit A,
// and one member is then a partner (min_len 0).
// split = false: the entry's splitter fields were not built (query-vs-target
// window tables: the row's column window is the table's window, nothing to prune).
__device__ __forceinline__ uint32_t run_lines(uint4 r4, int32_t wlo, int32_t whi, uint2& r, uint32_t min_len = 1u,
                                              bool split = true) {
    r = make_uint2(r4.x, r4.y);
    if (r.y - r.x <= min_len) return 0u;
    const uint32_t first = r.x & ~(uint32_t)(kGroup - 1);
    uint32_t nl = (r.y - first + kGroup - 1) / kGroup;
    if (split && nl > 1u) {
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

// (min(lo16, 1), min(hi16, 1)) of a packed u16 pair: one v_pk_min_u16 (the
// compiler turns the vector-min builtin into two compares and selects)
__device__ __forceinline__ uint32_t pk_min1_u16(uint32_t v) {
    uint32_t r;
    asm volatile("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(v), "s"(0x00010001u));
    return r;
}

// c / d for integers 1 <= c <= 65535, c <= d < 2^17 (T < 2^16 is checked at
// load), bit-identical to IEEE division: the reciprocal, Newton refinement
// and final residual correction the compiler expands '/' into (v_rcp_f64,
// fma refinement, mul, fma residual, fma correction), minus v_div_scale /
// v_div_fmas / v_div_fixup, which are the identity for operands this far
// from the exponent limits (no scaling, no inf / nan / zero / denormal
// cases), and with ONE Newton step instead of two: over this domain the
// once-refined reciprocal already makes the residual correction exact.
// Exhaustively checked against '/' on the GPU over the whole domain
// (pfaai_debug_div_check, tests/test_gpu_kernels.py; 0 mismatches for
// NS = 1 and 2, 2.9e9 of 4.3e9 quotients off for NS = 0).  S5 evaluates one
// division per nonzero counter, ~5e9 at 10k, so each fma matters.
template <int NS = 1>
__device__ __forceinline__ double exact_div_small(double c, double dd) {
    double y = __builtin_amdgcn_rcp(dd);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const double e = __builtin_fma(-dd, y, 1.0);
        y = __builtin_fma(y, e, y);
    }
    const double q = c * y;
    const double r = __builtin_fma(-dd, q, c);
    return __builtin_fma(r, y, q);
}

// c / d for any denominator the row kernels meet: the fast path on its
// verified domain (c <= d always holds for T[p][A] + T[p][B] - c with the
// true T columns), IEEE '/' otherwise -- only the reference's QT T-index
// quirk (PFAAI_FLAG_REF_COMPAT) pairs other genomes' counts
// and can give d < c, d == 0 (inf, as the reference) or d < 0.
__device__ __forceinline__ double exact_div_any(double c, double dd) {
    if (__builtin_expect(dd < c, 0)) return c / dd;
    return exact_div_small(c, dd);
}

}  // namespace pfaai
