// pfaai_hip.hip -- C-ABI implementation of libpfaai_hip.so (include/pfaai_hip.h).
//
// Owns one device per context: the problem (Lp, F, T, mode maps) stays
// resident in HBM after pfaai_load(); pfaai_run() is stream-ordered device
// work only (no host sync, no allocation): the run table (k_blk) or, for
// F-only input, the sorted work lists, then the row kernel (K-S+J).

#include <algorithm>
#include <chrono>
#include <random>
#include <atomic>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <system_error>
#include <vector>

#include "pfaai_hip.h"
#include "pfaai_aux.hpp"
#include "pfaai_build.hpp"
#include "pfaai_ctx.hpp"
#include "pfaai_sort.hpp"

using namespace pfaai;

using namespace pfaai_impl;

namespace {

// Host-side checks of pfaai_load over |F|-sized arrays: [0, n) split over up
// to 16 threads, one per 2^20 units of `work` (default n): fn(lo, hi, thread).
// If a thread cannot be started, its ranges run on the calling thread.
template <class Fn>
int par_for(int64_t n, Fn fn, int64_t work = -1) {
    const int64_t hw = std::max<int64_t>(1, (int64_t)std::thread::hardware_concurrency());
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>({hw, 16, (work < 0 ? n : work) >> 20, n}));
    if (nt == 1) {
        fn((int64_t)0, n, 0);
        return 1;
    }
    std::vector<std::thread> th;
    int started = 0;
    try {
        for (; started < nt; ++started) th.emplace_back([&, t = started] { fn(n * t / nt, n * (t + 1) / nt, t); });
    } catch (const std::system_error&) {
        for (int t = started; t < nt; ++t) fn(n * t / nt, n * (t + 1) / nt, t);
    }
    for (auto& x : th) x.join();
    return nt;
}

// exclusive scan of n u32 -> u64 out[0..n] (out[n] = total)
int scan_u32(pfaai_ctx* c, const uint32_t* in, int64_t n, unsigned long long* out, hipStream_t s);

// Device -> pinned host slot by the shader (staged_copy's D2H): 16-B loads
// from HBM, 16-B stores over the host link into the mapped pinned slot, the
// tail by bytes.  (hipMemcpyAsync into the slots: the first large D2H of a
// run stalled 8-19 ms inside the copy calls -- the C2 CLI's AJI, 16 MB --
// while a 4-KB copy just before it took 0.02 ms; round 5.)
__global__ __launch_bounds__(256) void k_stage_copy(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                   uint64_t bytes) {
    const uint64_t n16 = bytes >> 4;
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool al = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15u) == 0;
    if (al) {
        for (uint64_t i = i0; i < n16; i += step)
            reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
        for (uint64_t i = (n16 << 4) + i0; i < bytes; i += step) dst[i] = src[i];
    } else {
        for (uint64_t i = i0; i < bytes; i += step) dst[i] = src[i];
    }
}

}  // namespace

// Copies between the caller's pageable host memory and the device, both ways
// (the host-output entry points' D2H, pfaai_load's large H2D uploads).  A
// plain hipMemcpy to or from pageable memory runs through the runtime's own
// staging on one thread: ~9 GB/s up (the CLI's C2 G_tet, 230 MB: 27 ms) and
// ~2.5 GB/s down into memory nothing has touched yet (its 40 MB of outputs:
// 16 ms), round 5.  Here up to kStageThreads host threads each own a
// contiguous slice of the transfer and two kStageSlot-byte slots of the
// context's pinned buffer (allocated by pfaai_create, so the CLI's helper
// thread pays it beside the SQLite read): down, slot k is filled by the copy
// kernel k_stage_copy before slot k - 1 is copied out to dst; up, slot k is
// filled from src while slot k - 1's DMA runs.  The page faults of an
// untouched dst are taken by all threads at once.  Work ordered before on
// stream s is waited for; on return every byte has landed.  The threads all
// use stream s (spread over three streams the copies were slower, round 5).
int pfaai_impl::staged_copy(pfaai_ctx* c, void* dst, const void* src, size_t bytes, bool to_device, hipStream_t s) {
    if (bytes == 0) return PFAAI_RC_OK;
    if (!c->stage_host && hipHostMalloc(&c->stage_host, kStageBytes, hipHostMallocDefault) != hipSuccess)
        c->stage_host = nullptr;
    const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
    const int nt = (int)std::min<size_t>({(size_t)kStageThreads, (size_t)hw, bytes / (2 * kStageSlot)});
    if (nt < 2 || !c->stage_host) {  // small (< 4 MB) or no pinned buffer: the runtime's own path
        HIPCHK(c, hipMemcpyAsync(dst, src, bytes, to_device ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        return PFAAI_RC_OK;
    }
    for (int i = 0; i < 2 * nt; ++i)
        if (!c->stage_ev[i]) HIPCHK(c, hipEventCreateWithFlags(&c->stage_ev[i], hipEventDisableTiming));
    std::vector<hipError_t> err((size_t)nt, hipSuccess);
    // PFAAI_TRACE_COMPUTE (diagnostics build only): per thread, ns in the copy
    // API calls, the event waits and the host memcpy
    static const bool trace = DIAG_ENV("PFAAI_TRACE_COMPUTE") != nullptr;
    std::vector<int64_t> tr((size_t)nt * 4, 0);
    using tclk = std::chrono::steady_clock;
    const auto t_begin = tclk::now();
    auto ns_of = [](tclk::time_point a) {
        return (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(tclk::now() - a).count();
    };
    auto slice = [&](int t) {
        const auto t_slice = tclk::now();
        int64_t* T = &tr[(size_t)t * 4];
        // (all on s: spreading the threads over three streams measured
        // slower, the C2 CLI's G_tet 8.0 -> 9.6-11.5 ms, the bench's 1.15-GB
        // arrays 38 -> 42-49 ms: the DMA queue is not the limit)
        hipStream_t st = s;
        // [lo, hi) of the transfer, in slots of kStageSlot
        const size_t lo = bytes * (size_t)t / (size_t)nt, hi = bytes * (size_t)(t + 1) / (size_t)nt;
        char* pin[2] = {static_cast<char*>(c->stage_host) + (2 * (size_t)t) * kStageSlot,
                        static_cast<char*>(c->stage_host) + (2 * (size_t)t + 1) * kStageSlot};
        hipEvent_t ev[2] = {c->stage_ev[2 * t], c->stage_ev[2 * t + 1]};
        const size_t ns = (hi - lo + kStageSlot - 1) / kStageSlot;
        auto len = [&](size_t k) { return std::min(kStageSlot, hi - lo - k * kStageSlot); };
        hipError_t e = hipSuccess;
        if (to_device) {
            for (size_t k = 0; k < ns && e == hipSuccess; ++k) {
                if (k >= 2) e = hipEventSynchronize(ev[k & 1]);  // slot k & 1's previous DMA done
                if (e != hipSuccess) break;
                std::memcpy(pin[k & 1], static_cast<const char*>(src) + lo + k * kStageSlot, len(k));
                // (the slot -> device step by the copy kernel instead: no
                // change to the first step's clock and slower above 512 MB,
                // profiles/r05/ab_h2d_kernel.txt)
                e = hipMemcpyAsync(static_cast<char*>(dst) + lo + k * kStageSlot, pin[k & 1], len(k),
                                   hipMemcpyHostToDevice, st);
                if (e == hipSuccess) e = hipEventRecord(ev[k & 1], st);
            }
            for (int j = 0; j < 2 && e == hipSuccess; ++j)
                if ((size_t)j < ns) e = hipEventSynchronize(ev[j]);
        } else {
            auto out = [&](size_t k) -> hipError_t {
                auto t0 = tclk::now();
                hipError_t r = hipEventSynchronize(ev[k & 1]);
                if (trace) T[1] += ns_of(t0), t0 = tclk::now();
                if (r == hipSuccess) std::memcpy(static_cast<char*>(dst) + lo + k * kStageSlot, pin[k & 1], len(k));
                if (trace) T[2] += ns_of(t0);
                return r;
            };
            for (size_t k = 0; k < ns && e == hipSuccess; ++k) {
                const auto t0 = tclk::now();
                hipLaunchKernelGGL(k_stage_copy, dim3(128), dim3(256), 0, st,
                                   reinterpret_cast<const uint8_t*>(static_cast<const char*>(src) + lo + k * kStageSlot),
                                   reinterpret_cast<uint8_t*>(pin[k & 1]), (uint64_t)len(k));
                e = hipGetLastError();
                if (e == hipSuccess) e = hipEventRecord(ev[k & 1], st);
                if (trace) T[0] += ns_of(t0);
                if (e == hipSuccess && k >= 1) e = out(k - 1);  // slot k - 1 out while slot k's DMA runs
            }
            if (e == hipSuccess) e = out(ns - 1);
        }
        err[(size_t)t] = e;
        if (trace) T[3] = ns_of(t_slice);
    };
    std::vector<std::thread> th;
    int started = 1;
    try {
        for (; started < nt; ++started) th.emplace_back(slice, started);
    } catch (const std::system_error&) {
    }
    slice(0);
    for (auto& x : th) x.join();
    for (int t = started; t < nt; ++t) slice(t);  // threads that could not be started
    if (trace) {
        int64_t mx[4] = {0, 0, 0, 0};
        for (int t = 0; t < nt; ++t)
            for (int j = 0; j < 4; ++j) mx[j] = std::max(mx[j], tr[(size_t)t * 4 + j]);
        std::fprintf(stderr, "[pfaai_staged] %s %zu B, %d threads: wall %.2f ms; max per thread: api %.2f, wait %.2f, "
                     "memcpy %.2f, slice %.2f ms\n", to_device ? "H2D" : "D2H", bytes, nt, ns_of(t_begin) / 1e6,
                     mx[0] / 1e6, mx[1] / 1e6, mx[2] / 1e6, mx[3] / 1e6);
    }
    for (hipError_t e : err)
        if (e != hipSuccess) {
            // a failed slice may leave other slices' copy kernels or DMAs
            // writing into the shared pinned slots: drain the stream before
            // the caller reuses them
            (void)hipStreamSynchronize(s);
            return hip_fail(c, e, "staged_copy");
        }
    return PFAAI_RC_OK;
}

namespace {

// Sort space for n keys: two key and two value ping-pong buffers, the
// per-tile digit histograms and their scan (k_rs_hist / k_rs_scatter).
int ensure_sort_space(pfaai_ctx* c, int64_t n) {
    const int64_t nn = std::max<int64_t>(n, 1);
    const int64_t ntiles = ceil_div(nn, kRsTile), hist_n = kRsBins * ntiles;
    int rc;
    if ((rc = ensure(c, c->key_a, nn * 4)) || (rc = ensure(c, c->key_b, nn * 4)) || (rc = ensure(c, c->val_a, nn * 4)) ||
        (rc = ensure(c, c->val_b, nn * 4)) || (rc = ensure(c, c->hist, hist_n * 4)) ||
        (rc = ensure(c, c->hoff, (hist_n + 1) * 8)) ||
        (rc = ensure(c, c->sums, std::max<int64_t>(1, ceil_div(std::max<int64_t>(hist_n, PFAAI_NTETRAMERS), kScanTile)) * 8)))
        return rc;
    return PFAAI_RC_OK;
}

// Stable LSD radix sort (8-bit digits) of n keys with `bits` significant
// bits; keys_in is not overwritten.  The last pass writes rec_in[original
// index] to recs_out in key order; *sorted receives the sorted keys (one of
// key_a / key_b).  Used for the work lists, and for F <-> G at load.
int radix_sort_recs(pfaai_ctx* c, const uint32_t* keys_in, int64_t n, int bits, const uint2* rec_in, uint2* recs_out,
                    hipStream_t s, const uint32_t** sorted) {
    const int passes = std::max(1, (bits + 7) / 8);
    const int64_t ntiles = ceil_div(std::max<int64_t>(n, 1), kRsTile);
    auto* hist = static_cast<uint32_t*>(c->hist.p);
    auto* hoff = static_cast<unsigned long long*>(c->hoff.p);
    const uint32_t* kin = keys_in;
    const uint32_t* vin = nullptr;
    uint32_t* kout = static_cast<uint32_t*>(c->key_a.p);
    uint32_t* vout = static_cast<uint32_t*>(c->val_a.p);
    uint32_t* kalt = static_cast<uint32_t*>(c->key_b.p);
    uint32_t* valt = static_cast<uint32_t*>(c->val_b.p);
    for (int pass = 0; pass < passes; ++pass) {
        const int shift = 8 * pass;
        const bool first = pass == 0, last = pass == passes - 1;
        hipLaunchKernelGGL(k_rs_hist, dim3(ntiles), dim3(kRsThreads), 0, s, kin, n, shift, hist, ntiles);
        int rc = scan_u32(c, hist, kRsBins * ntiles, hoff, s);
        if (rc) return rc;
#define RS(F, L)                                                                                                  \
    hipLaunchKernelGGL((k_rs_scatter<F, L>), dim3(ntiles), dim3(kRsThreads), 0, s, kin, vin, n, shift, hoff, hist, \
                       ntiles, kout, vout, rec_in, recs_out)
        if (first && last) RS(true, true);
        else if (first) RS(true, false);
        else if (last) RS(false, true);
        else RS(false, false);
#undef RS
        kin = kout;  // ping-pong (never back into keys_in)
        vin = vout;
        std::swap(kout, kalt);
        std::swap(vout, valt);
    }
    if (sorted) *sorted = kin;
    HIPCHK(c, hipGetLastError());
    return PFAAI_RC_OK;
}

int bits_for(int64_t k) {  // significant bits of keys < k
    int bits = 1;
    while (bits < 32 && ((int64_t)1 << bits) < k) ++bits;
    return bits;
}

// Work-list build for rows [rb, re): entries, LSD radix sort, rowptr.
template <int MODE>
int build_records(pfaai_ctx* c, int64_t rb, int64_t re, hipStream_t s, bool first_event) {
    const int64_t P = c->prob.n_prot;
    const int64_t K = (re - rb) * P;  // keys
    const int64_t n = c->row_fprefix[re] - c->row_fprefix[rb];  // entries (exact, from F at load)
    auto* sc = static_cast<unsigned long long*>(c->scalars.p);
    int* err = reinterpret_cast<int*>(sc + SC_ERR);
    auto* rowptr = static_cast<unsigned long long*>(c->rowptr.p);
    auto* key_c = static_cast<uint32_t*>(c->key_c.p);
    auto* rec_c = static_cast<uint2*>(c->rec_c.p);
    // compaction offsets: entries per tetramer block, scanned
    auto* cnt_t = static_cast<uint32_t*>(c->cnt_t.p);
    auto* off_t = static_cast<unsigned long long*>(c->off_t.p);
    hipLaunchKernelGGL(k_count_t, dim3(kNTetramers), dim3(kTetraThreads), 0, s, c->dev, rb, re, cnt_t);
    int rc0 = scan_u32(c, cnt_t, kNTetramers, off_t, s);
    if (rc0) return rc0;
    if (first_event) HIPCHK(c, hipMemsetAsync(sc + SC_FIRST_KEY, 0xFF, sizeof(unsigned long long), s));
    if (first_event)
        hipLaunchKernelGGL((k_entries<MODE, true>), dim3(kNTetramers), dim3(kTetraThreads), 0, s, c->dev, rb, re,
                           key_c, rec_c, off_t, sc + SC_FIRST_KEY, err);
    else
        hipLaunchKernelGGL((k_entries<MODE, false>), dim3(kNTetramers), dim3(kTetraThreads), 0, s, c->dev, rb, re,
                           key_c, rec_c, off_t, sc + SC_FIRST_KEY, err);
    if (n == 0) {
        HIPCHK(c, hipMemsetAsync(rowptr, 0, (K + 1) * sizeof(unsigned long long), s));
        HIPCHK(c, hipGetLastError());
        return PFAAI_RC_OK;
    }
    const uint32_t* ksorted = nullptr;
    int rc = radix_sort_recs(c, key_c, n, bits_for(K), rec_c, static_cast<uint2*>(c->recs.p), s, &ksorted);
    if (rc) return rc;
    hipLaunchKernelGGL(k_rowptr, dim3(ceil_div(n, 256)), dim3(256), 0, s, ksorted, n, K, rowptr);
    HIPCHK(c, hipGetLastError());
    return PFAAI_RC_OK;
}

// The lexicographically first E triple of the LOADED mode (the ref-compat
// zero-overlap quirk) -- also for full-row runs, whose
// mirror cells are the loaded mode's pairs.
int launch_first_key(pfaai_ctx* c, hipStream_t s) {
    auto* sc = static_cast<unsigned long long*>(c->scalars.p);
    int* err = reinterpret_cast<int*>(sc + SC_ERR);
    HIPCHK(c, hipMemsetAsync(sc + SC_FIRST_KEY, 0xFF, sizeof(unsigned long long), s));
#define FK(M)                                                                                                       \
    hipLaunchKernelGGL((k_entries<M, true>), dim3(kNTetramers), dim3(kTetraThreads), 0, s, c->dev, (int64_t)0,       \
                       (int64_t)0, static_cast<uint32_t*>(nullptr), static_cast<uint2*>(nullptr),                  \
                       static_cast<const unsigned long long*>(nullptr), sc + SC_FIRST_KEY, err)
    switch (c->prob.mode) {
        case 0: FK(0); break;
        case 1: FK(1); break;
        default: FK(2); break;
    }
#undef FK
    HIPCHK(c, hipGetLastError());
    return PFAAI_RC_OK;
}

// Fused genome-major path: only the run table (+ the first E triple for the
// ref-compat zero-overlap quirk); k_rows walks the G lists itself.
template <int MODE>
int build_runs_g(pfaai_ctx* c, hipStream_t s, bool first_event, bool ends) {
    if (ends) {  // k_rows_pl WK 3 reads run ends only (pl_uses_ends)
        const char* et = DIAG_ENV("PFAAI_BLK_END_TILE");  // tetramers per workgroup (A/B)
        const int tile = (int)std::max<int64_t>(1, std::min<int64_t>(et ? std::min(atoi(et), kBlkEndTileMax) : kBlkEndTileMax,
                                                                     kBlkEndDynLds / (4 * c->prob.n_prot)));
        const size_t lds = (size_t)c->prob.n_prot * tile * sizeof(uint32_t);
        const char* eu = DIAG_ENV("PFAAI_BLK_END_U");  // loads in flight per lane (A/B)
        const int u = eu ? atoi(eu) : 1;
        if (u >= 4)
            hipLaunchKernelGGL((k_blk_end<1024, 4>), dim3(ceil_div(kNTetramers, tile)), dim3(1024), lds, s, c->dev, tile);
        else if (u == 2)
            hipLaunchKernelGGL((k_blk_end<1024, 2>), dim3(ceil_div(kNTetramers, tile)), dim3(1024), lds, s, c->dev, tile);
        else
            hipLaunchKernelGGL((k_blk_end<1024, 1>), dim3(ceil_div(kNTetramers, tile)), dim3(1024), lds, s, c->dev, tile);
        if (first_event) {
            const int rc = launch_first_key(c, s);
            if (rc) return rc;
        }
        HIPCHK(c, hipGetLastError());
        return PFAAI_RC_OK;
    }
    const int tile = (int)std::max<int64_t>(1, std::min<int64_t>(kBlkTileMax, kBlkDynLds / (16 * c->prob.n_prot)));
    const int dbg = DIAG_ENV("PFAAI_BLK_ABLATE") ? atoi(DIAG_ENV("PFAAI_BLK_ABLATE")) : 0;
    const size_t lds = (size_t)c->prob.n_prot * tile * sizeof(uint4);
    // 1024 threads (0.649 vs 0.666 ms at 10k; the window form gains 2x, see
    // run_mode); PFAAI_BLK_THREADS=256 for A/B
    const char* bt = DIAG_ENV("PFAAI_BLK_THREADS");
    if (bt && atoi(bt) == 256)
        hipLaunchKernelGGL((k_blk<false, kTetraThreads>), dim3(ceil_div(kNTetramers, tile)), dim3(kTetraThreads), lds, s,
                           c->dev, tile, dbg, 0, 1);
    else
        hipLaunchKernelGGL((k_blk<false, 1024>), dim3(ceil_div(kNTetramers, tile)), dim3(1024), lds, s, c->dev, tile,
                           dbg, 0, 1);
    if (first_event) {
        const int rc = launch_first_key(c, s);
        if (rc) return rc;
    }
    HIPCHK(c, hipGetLastError());
    return PFAAI_RC_OK;
}

int scan_u32(pfaai_ctx* c, const uint32_t* in, int64_t n, unsigned long long* out, hipStream_t s) {
    auto* sums = static_cast<unsigned long long*>(c->sums.p);
    auto* sc = static_cast<unsigned long long*>(c->scalars.p);
    const int64_t tiles = std::max<int64_t>(1, ceil_div(n, kScanTile));
    hipLaunchKernelGGL(k_scan_tiles, dim3(tiles), dim3(kScanThreads), 0, s, in, n, out, sums);
    hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(kScanThreads), 0, s, sums, tiles, sc + SC_GRAND);
    hipLaunchKernelGGL(k_scan_add, dim3(tiles), dim3(kScanThreads), 0, s, out, n, sums, sc + SC_GRAND,
                       static_cast<unsigned long long*>(nullptr));
    return PFAAI_RC_OK;
}

// Work-list space for the sorted (F-only) path, sized for all rows: ~36 B per
// F entry of the row genomes.  The genome-major kernels need none of it, so
// it is allocated at load only for F-only input (and on first use by
// pfaai_debug_row_counts).
int ensure_worklists(pfaai_ctx* c) {
    if (c->wl_ready) return PFAAI_RC_OK;
    const auto& p = c->prob;
    int rc;
    const int64_t nmax = std::max<int64_t>(1, c->row_fprefix[c->n_rows]);
    const int64_t K = c->n_rows * p.n_prot;
    const int64_t ntiles = ceil_div(nmax, kRsTile);
    const int64_t hist_n = kRsBins * ntiles;
    if ((rc = ensure(c, c->rowptr, (K + 1) * sizeof(unsigned long long)))) return rc;
    if ((rc = ensure(c, c->lens, std::max<int64_t>(K, 1) * sizeof(uint32_t)))) return rc;
    if ((rc = ensure(c, c->cnt_t, PFAAI_NTETRAMERS * sizeof(uint32_t)))) return rc;
    if ((rc = ensure(c, c->off_t, (PFAAI_NTETRAMERS + 1) * sizeof(unsigned long long)))) return rc;
    if ((rc = ensure(c, c->key_c, nmax * sizeof(uint32_t)))) return rc;
    if ((rc = ensure(c, c->rec_c, nmax * sizeof(uint2)))) return rc;
    if ((rc = ensure(c, c->key_a, nmax * sizeof(uint32_t)))) return rc;
    if ((rc = ensure(c, c->key_b, nmax * sizeof(uint32_t)))) return rc;
    if ((rc = ensure(c, c->val_a, nmax * sizeof(uint32_t)))) return rc;
    if ((rc = ensure(c, c->val_b, nmax * sizeof(uint32_t)))) return rc;
    if ((rc = ensure(c, c->recs, nmax * sizeof(uint2)))) return rc;
    if ((rc = ensure(c, c->hist, hist_n * sizeof(uint32_t)))) return rc;
    if ((rc = ensure(c, c->hoff, (hist_n + 1) * sizeof(unsigned long long)))) return rc;
    if ((rc = ensure(c, c->sums, std::max<int64_t>(1, ceil_div(std::max({hist_n, K, (int64_t)PFAAI_NTETRAMERS}), kScanTile)) *
                                     sizeof(unsigned long long))))
        return rc;
    c->wl_ready = true;
    return PFAAI_RC_OK;
}

template <int MODE>
int run_mode(pfaai_ctx* c, int64_t rb, int64_t re, uint32_t flags, double* aji, double* S, int32_t* N,
             hipStream_t s) {
    const bool compat = flags & PFAAI_FLAG_REF_COMPAT;
    auto* sc = static_cast<unsigned long long*>(c->scalars.p);
    HIPCHK(c, hipMemsetAsync(sc + SC_EVENTS, 0, sizeof(unsigned long long), s));
    const bool wl = c->rows_kernel == RK_WORKLIST;
    if (c->prob.mode == PFAAI_MODE_ALL && (c->order_n ? re > c->order_n : (rb < c->chk_lo || re > c->chk_hi)))
        return fail(c, PFAAI_RC_INVALID,
                    c->order_n ? "rows past the genome list of pfaai_set_row_order"
                               : "rows outside the block whose G lists pfaai_load_rows verified");
    c->run_rb = rb;  // (pl_uses_ends: the rows' G_pos / G_end must have been built)
    c->run_re = re;
    c->last_walk = PFAAI_WALK_NONE;  // (set by launch_pl / launch_narrow)
    c->last_narrow = false;
    // rows wider than one k_rows_pl chunk: absolute column windows, each with
    // its own run table (launch_pl); PFAAI_PL_WINDOWS=0 keeps the per-row
    // chunks over one table (A/B)
    int win_tile = 0, nwin = 1;
    const int64_t wcols = pl_chunk_cols(c);
    {
        const char* wv = DIAG_ENV("PFAAI_PL_WINDOWS");
        c->windows = (c->rows_kernel == RK_PL || c->rows_kernel == RK_PL512) &&
                     !(wv && wv[0] == '0') &&
                     (int64_t)c->cols_run + 1 > wcols;
        if (c->windows) {  // all windows' tables staged in one k_blk workgroup's LDS (nwin * P <= 5104)
            nwin = (int)ceil_div(MODE == 2 ? c->prob.n_tgt : c->prob.n_ids, wcols);
            win_tile = (int)std::min<int64_t>(kBlkTileMax, kBlkDynLds / (16 * (int64_t)c->prob.n_prot * nwin));
            c->windows = win_tile >= 1 &&
                         ensure(c, c->blkw, (size_t)nwin * c->prob.n_prot * kNTetramers * sizeof(uint4)) == PFAAI_RC_OK;
        }
    }
    if (c->windows) {
        if (!c->take_events()) return fail(c, PFAAI_RC_HIP, "hipEventCreate failed");
        HIPCHK(c, hipEventRecord(c->ev0, s));
        // the window tables depend only on the loaded F and the window width:
        // built by the first windowed run after a load, then kept by every
        // later run of that load (a load product, like G_pe; round 6 -- the
        // query-vs-target and streamed steps rebuilt them every run before)
        const bool keep = c->win_valid && c->win_cols == wcols && (c->win_key || !compat);
        // the WK 4 spans' member codes (pl_win_spans): k_fcode once per load
        if (pl_win_spans(c, MODE) && !c->dev.Fcode) {
            if (int rcf = ensure(c, c->Fcode, (size_t)(c->prob.n_f + 16) * sizeof(uint32_t))) return rcf;
            hipLaunchKernelGGL(k_fcode, dim3((int)std::min<int64_t>(ceil_div(c->prob.n_f + 16, 256), 1 << 16)),
                               dim3(256), 0, s, c->dev.Fg, c->prob.n_f, static_cast<uint32_t*>(c->Fcode.p));
            HIPCHK(c, hipGetLastError());
            c->dev.Fcode = static_cast<const uint32_t*>(c->Fcode.p);
        }
        if (!keep) {
            Dev dw = c->dev;
            dw.blk = static_cast<uint4*>(c->blkw.p);
            // 1024 threads: the 80 KB of LDS staging allows two workgroups per
            // CU, so a 256-thread form ran 8 waves per CU (PFAAI_BLK_THREADS=256
            // A/B: 6.0 -> 2.9 ms at QT 50 000 x 1 000)
            const size_t lds = (size_t)nwin * c->prob.n_prot * win_tile * sizeof(uint4);
            const char* bt = DIAG_ENV("PFAAI_BLK_THREADS");
            // query-vs-target rows' column window IS the table's window: the
            // row kernel never prunes by splitters there, so they are not built
            // (k_blk phase 2 off; PFAAI_BLK_QT_SPLIT=1 builds them, A/B)
            const char* qs = DIAG_ENV("PFAAI_BLK_QT_SPLIT");
            const int ph = MODE == 2 && !(qs && qs[0] == '1') ? 2 : 0;
            // query vs target: the tables stop at n_tgt (targets only, WK 4)
            const int32_t gmax = MODE == 2 ? c->prob.n_tgt : c->prob.n_ids;
            if (bt && atoi(bt) == 256)
                hipLaunchKernelGGL((k_blk<true, 256>), dim3(ceil_div(kNTetramers, win_tile)), dim3(256), lds, s, dw,
                                   win_tile, ph, (int32_t)wcols, nwin, gmax);
            else
                hipLaunchKernelGGL((k_blk<true, 1024>), dim3(ceil_div(kNTetramers, win_tile)), dim3(1024), lds, s, dw,
                                   win_tile, ph, (int32_t)wcols, nwin, gmax);
            if (compat) {  // the zero-overlap quirk's first E triple (build_runs_g's second half)
                const int rcf = launch_first_key(c, s);
                if (rcf) return rcf;
            }
            HIPCHK(c, hipGetLastError());
            c->win_valid = true;
            c->win_key = compat;
            c->win_cols = wcols;
        }
        HIPCHK(c, hipEventRecord(c->ev1, s));
        launch_rows<MODE>(c, rb, re, flags, aji, S, N, s);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipEventRecord(c->ev2, s));
        return PFAAI_RC_OK;
    }
    // three events per run: start, after work-list build, after row kernel
    if (!c->take_events()) return fail(c, PFAAI_RC_HIP, "hipEventCreate failed");
    HIPCHK(c, hipEventRecord(c->ev0, s));
    if (wl) {
        const int rcw = ensure_worklists(c);
        if (rcw) return rcw;
    }
    // PFAAI_FLAG_KEEP_RUNS: the run table depends only on the loaded F, so a
    // run over further rows of the same problem may reuse it (stream-ordered
    // after the run that built it)
    const bool ends = !wl && pl_uses_ends(c, MODE);  // which table launch_rows will read
    const bool keep = !wl && (flags & PFAAI_FLAG_KEEP_RUNS) && c->runs_valid && (c->runs_key || !compat) &&
                      c->runs_ends == ends;
    int rc = PFAAI_RC_OK;
    if constexpr (MODE == kModeFull) {
        if (wl) return fail(c, PFAAI_RC_INVALID, "full rows need the genome-major path");
    } else if (wl) {
        rc = build_records<MODE>(c, rb, re, s, compat);
    }
    if (!wl && ends && c->dev.G_pe) {
        // WK 3 reads G_pe (built at load): no run table; only the ref-compat
        // zero-overlap quirk's first E triple
        if (compat) rc = launch_first_key(c, s);
    } else if (!wl && !keep) {
        rc = build_runs_g<MODE>(c, s, compat, ends);
        c->runs_valid = rc == PFAAI_RC_OK;
        c->runs_key = compat;
        c->runs_ends = ends;
    }
    if (rc) return rc;
    HIPCHK(c, hipEventRecord(c->ev1, s));
    launch_rows<MODE>(c, rb, re, flags, aji, S, N, s);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(c->ev2, s));
    return PFAAI_RC_OK;
}

// Run fn() and map a C++ exception to an error code: nothing may unwind
// through the C ABI (a std::bad_alloc of a host vector, a std::system_error
// of a checking thread).
template <class Fn>
int guarded(pfaai_ctx* c, Fn fn) {
    try {
        return fn();
    } catch (const std::bad_alloc&) {
        return fail(c, PFAAI_RC_OOM, "host allocation failed");
    } catch (const std::exception& e) {
        return fail(c, PFAAI_RC_INVALID, std::string("internal error: ") + e.what());
    } catch (...) {
        return fail(c, PFAAI_RC_INVALID, "internal error");
    }
}

// F from G on the device (the CLI's `<p>_genomes` read; F never exists on
// the host): keys t * P + p, stable radix sort, split into Fp / Fg, Lp by a
// scan of the tetramer counts.
int build_f_from_g(pfaai_ctx* c, int64_t n_lists, int64_t n, hipStream_t s) {
    const int32_t P = c->prob.n_prot;
    int rc;
    if ((rc = ensure(c, c->key_c, std::max<int64_t>(n, 1) * 4)) || (rc = ensure(c, c->rec_c, std::max<int64_t>(n, 1) * 8)) ||
        (rc = ensure(c, c->recs, std::max<int64_t>(n, 1) * 8)) || (rc = ensure(c, c->cnt_t, PFAAI_NTETRAMERS * 4)) ||
        (rc = ensure_sort_space(c, n)))
        return rc;
    auto* lc = static_cast<uint32_t*>(c->cnt_t.p);
    HIPCHK(c, hipMemsetAsync(lc, 0, PFAAI_NTETRAMERS * 4, s));
    const int grid = (int)std::min<int64_t>(std::max<int64_t>(ceil_div(n_lists, 4), 1), 1 << 16);
    hipLaunchKernelGGL(k_fkeys_from_g, dim3(grid), dim3(256), 0, s, static_cast<const int64_t*>(c->G_off.p),
                       static_cast<const int32_t*>(c->G_tet.p), n_lists, P, static_cast<uint32_t*>(c->key_c.p),
                       static_cast<uint2*>(c->rec_c.p), lc);
    HIPCHK(c, hipGetLastError());
    if ((rc = scan_u32(c, lc, PFAAI_NTETRAMERS, static_cast<unsigned long long*>(c->Lp.p), s))) return rc;
    if (n) {
        auto* recs = static_cast<uint2*>(c->recs.p);
        const uint32_t* ksorted = nullptr;
        if ((rc = radix_sort_recs(c, static_cast<const uint32_t*>(c->key_c.p), n, bits_for((int64_t)PFAAI_NTETRAMERS * P),
                                  static_cast<const uint2*>(c->rec_c.p), recs, s, &ksorted)))
            return rc;
        const int g2 = (int)std::min<int64_t>(ceil_div(n, 256), 1 << 16);
        hipLaunchKernelGGL(k_f_split_pos, dim3(g2), dim3(256), 0, s, ksorted, recs, n, P, static_cast<int32_t*>(c->Fp.p),
                           static_cast<int32_t*>(c->Fg.p), static_cast<uint32_t*>(c->G_pos.p));
        HIPCHK(c, hipGetLastError());
    }
    return PFAAI_RC_OK;
}

// G from F on the device (F-only callers, e.g. the reference's own
// DataStructInterface classes): keys g * P + p, stable radix sort, G_tet from
// the sorted (tetramer, genome) records, G_off = first sorted key >= k.
int build_g_from_f(pfaai_ctx* c, int64_t n_lists, int64_t n, hipStream_t s) {
    const int32_t P = c->prob.n_prot;
    int rc;
    if ((rc = ensure(c, c->key_c, std::max<int64_t>(n, 1) * 4)) || (rc = ensure(c, c->rec_c, std::max<int64_t>(n, 1) * 8)) ||
        (rc = ensure(c, c->recs, std::max<int64_t>(n, 1) * 8)) || (rc = ensure_sort_space(c, n)) ||
        (rc = ensure(c, c->G_off, (n_lists + 1) * 8)) || (rc = ensure(c, c->G_tet, std::max<int64_t>(n, 1) * 4)))
        return rc;
    auto* goff = static_cast<unsigned long long*>(c->G_off.p);
    if (n == 0) {
        HIPCHK(c, hipMemsetAsync(goff, 0, (n_lists + 1) * 8, s));
        return PFAAI_RC_OK;
    }
    hipLaunchKernelGGL(k_gkeys_from_f, dim3(8192), dim3(256), 0, s, static_cast<const int64_t*>(c->Lp.p),
                       static_cast<const int32_t*>(c->Fp.p), static_cast<const int32_t*>(c->Fg.p), P,
                       static_cast<uint32_t*>(c->key_c.p), static_cast<uint2*>(c->rec_c.p));
    HIPCHK(c, hipGetLastError());
    auto* recs = static_cast<uint2*>(c->recs.p);
    const uint32_t* ksorted = nullptr;
    if ((rc = radix_sort_recs(c, static_cast<const uint32_t*>(c->key_c.p), n, bits_for(n_lists),
                              static_cast<const uint2*>(c->rec_c.p), recs, s, &ksorted)))
        return rc;
    const int g2 = (int)std::min<int64_t>(ceil_div(n, 256), 1 << 16);
    hipLaunchKernelGGL(k_gtet_split, dim3(g2), dim3(256), 0, s, recs, n, static_cast<int32_t*>(c->G_tet.p),
                       static_cast<uint32_t*>(c->G_pos.p));
    hipLaunchKernelGGL(k_rowptr, dim3(ceil_div(n, 256)), dim3(256), 0, s, ksorted, n, n_lists, goff);
    HIPCHK(c, hipGetLastError());
    return PFAAI_RC_OK;
}

// The load-time sort space is also the work-list space: release it when the
// genome-major kernels (which need none of it) will run.
void release_sort_space(pfaai_ctx* c) {
    for (DevBuf* b : {&c->key_c, &c->rec_c, &c->recs, &c->key_a, &c->key_b, &c->val_a, &c->val_b, &c->hist, &c->hoff})
        release(*b);
    c->wl_ready = false;
}

// ---- the load-time transposition sort (pfaai_sort.hpp) ---------------------
// passes and digit width for kb-bit keys: one pass up to 11 bits, two up to
// 22 (10-bit digits for the 20-bit keys g * P + p at 10k x 100), three above
int tsort_db(int kb, int* passes) {
    if (const char* v = DIAG_ENV("PFAAI_TSORT_DB")) {  // diagnostics: digit width (A/B)
        const int db = std::max(8, std::min(kSortMaxDB, atoi(v)));
        *passes = (kb + db - 1) / db;
        return db;
    }
    *passes = kb <= kSortMaxDB ? 1 : kb <= 2 * kSortMaxDB ? 2 : 3;
    return std::max(8, (kb + *passes - 1) / *passes);
}

// records ping-pong (srec_b only for keygen sources or three passes), the
// tile histograms, the group sums, the digit bases
int ensure_tsort(pfaai_ctx* c, int64_t n, int kb, bool keygen) {
    int passes;
    const int db = tsort_db(kb, &passes);
    const int64_t nn = std::max<int64_t>(n, 1);
    const int64_t ntiles = ceil_div(nn, kSortTileMin), ngroups = ceil_div(ntiles, kSortGroup);
    int rc;
    if ((rc = ensure(c, c->srec_a, nn * 8)) || ((keygen || passes > 2) && (rc = ensure(c, c->srec_b, nn * 8))) ||
        (rc = ensure(c, c->shist, (size_t)ntiles * (4u << db))) ||
        (rc = ensure(c, c->sgsum, (size_t)ngroups * (4u << db))) || (rc = ensure(c, c->sbase, (4u << db) + 64)))
        return rc;
    return PFAAI_RC_OK;
}

// exclusive-scan workspace (k_scan_tiles' tile sums) for n values
int ensure_scan(pfaai_ctx* c, int64_t n) {
    return ensure(c, c->sums, std::max<int64_t>(1, ceil_div(std::max<int64_t>(n, PFAAI_NTETRAMERS), kScanTile)) * 8);
}

template <int DB, int NT, bool PF, class S0, class DN, int VAR = 0>
void tsort_launch(pfaai_ctx* c, const S0& src0, const DN& dstN, int64_t n, int kb, int passes, hipStream_t s) {
    const int64_t ntiles = ceil_div(n, sort_tile<NT>()), ngroups = ceil_div(ntiles, kSortGroup);
    auto* hist = static_cast<uint32_t*>(c->shist.p);
    auto* gsum = static_cast<uint32_t*>(c->sgsum.p);
    auto* base = static_cast<uint32_t*>(c->sbase.p);
    uint32_t* tctr = base + (1 << DB);  // the scatter's per-XCD tile counters (zeroed by k_sort_top)
    uint64_t* buf[2] = {static_cast<uint64_t*>(c->srec_a.p), static_cast<uint64_t*>(c->srec_b.p)};
    const size_t lds = sort_scatter_lds<DB, NT>();
    // persistent scatter: as many workgroups as fit the CUs (two 512-thread
    // ones per CU at DB <= 10), each walking ntiles / grid tiles
    int cus = 256, per_cu = 1;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per_cu, reinterpret_cast<const void*>(&k_sort_scatter<DB, NT, PF, SrcRecs, DstRecs>), NT, lds);
    const int grid = (int)std::min<int64_t>(ntiles, (int64_t)cus * std::max(1, per_cu));
    for (int pass = 0; pass < passes; ++pass) {
        const int shift = pass * DB;
        const bool last = pass == passes - 1;
        // the digit covers only key bits: the records carry other fields right above the key
        const uint32_t mask = (1u << std::min(DB, kb - shift)) - 1u;
        const SrcRecs prev{buf[(pass + 1) & 1]};  // pass p reads what pass p - 1 wrote
        const DstRecs next{buf[pass & 1]};
        if (pass == 0)
            hipLaunchKernelGGL((k_sort_hist<DB, NT, S0>), dim3(ntiles), dim3(NT), 0, s, src0, n, shift, mask, hist);
        else
            hipLaunchKernelGGL((k_sort_hist<DB, NT, SrcRecs>), dim3(ntiles), dim3(NT), 0, s, prev, n, shift, mask,
                               hist);
        hipLaunchKernelGGL((k_sort_grp<DB>), dim3(ngroups), dim3(kSortThreads), 0, s, hist, ntiles, gsum);
        hipLaunchKernelGGL((k_sort_top<DB>), dim3(1), dim3(kSortThreads), 0, s, gsum, ngroups, base, tctr);
#define SC(SRC_T, SRC, DST_T, DST)                                                                        \
    hipLaunchKernelGGL((k_sort_scatter<DB, NT, PF, SRC_T, DST_T, VAR>), dim3(grid), dim3(NT), lds, s, SRC, DST, n, ntiles, \
                       shift, mask, hist, gsum, base, tctr)
        if (pass == 0 && last) SC(S0, src0, DN, dstN);
        else if (pass == 0) SC(S0, src0, DstRecs, next);
        else if (last) SC(SrcRecs, prev, DN, dstN);
        else SC(SrcRecs, prev, DstRecs, next);
#undef SC
    }
}

// Stable sort of n records by their low kb bits, src0 -> ... -> dstN.  A
// keygen source (SrcRecs) must read srec_b: the first pass writes srec_a.
template <class S0, class DN>
int tsort(pfaai_ctx* c, const S0& src0, const DN& dstN, int64_t n, int kb, hipStream_t s) {
    if (n == 0) return PFAAI_RC_OK;
    int passes;
    const int db = tsort_db(kb, &passes);
    // the ping-pong buffers this pass count writes (ensure_tsort sized them
    // from the same tsort_db): pass p writes srec[p & 1] except the last
    const size_t need = (size_t)n * 8;
    if (c->srec_a.bytes < need || c->shist.bytes < (size_t)ceil_div(n, kSortTileMin) * (4u << db) ||
        (passes > 2 && c->srec_b.bytes < need))
        return fail(c, PFAAI_RC_INVALID, "internal: transposition sort buffers not sized for this pass count");
#ifdef PFAAI_DIAGNOSTICS
    // diagnostics (A/B): PFAAI_TSORT_NT=1024 the one-per-CU form (with the
    // next-tile prefetch), PFAAI_TSORT_PF=0|1 the prefetch of the 512 form
    const char* nt = DIAG_ENV("PFAAI_TSORT_NT");
    const char* pf = DIAG_ENV("PFAAI_TSORT_PF");
    if (const char* vr = DIAG_ENV("PFAAI_TSORT_VAR"); vr && (db == 10 || db == 8)) {  // scatter variants / ablations (A/B)
#define TV(D, V) tsort_launch<D, kSortNT, kSortPF, S0, DN, V>(c, src0, dstN, n, kb, passes, s)
#define TVS(D)                                    \
    switch (atoi(vr)) {                           \
        case 1: TV(D, 1); break;                  \
        case 16: TV(D, 16); break;                \
        case 32: TV(D, 32); break;                \
        case 48: TV(D, 48); break;                \
        default: TV(D, 0); break;                 \
    }
        if (db == 8) { TVS(8) } else { TVS(10) }
#undef TVS
#undef TV
        HIPCHK(c, hipGetLastError());
        return PFAAI_RC_OK;
    }
    if ((nt && atoi(nt) == 1024) || (pf && (atoi(pf) != 0) != kSortPF)) {
        const bool big = nt && atoi(nt) == 1024;
        switch (db) {
            case 8: big ? tsort_launch<8, 1024, true>(c, src0, dstN, n, kb, passes, s) : tsort_launch<8, kSortNT, !kSortPF>(c, src0, dstN, n, kb, passes, s); break;
            case 9: big ? tsort_launch<9, 1024, true>(c, src0, dstN, n, kb, passes, s) : tsort_launch<9, kSortNT, !kSortPF>(c, src0, dstN, n, kb, passes, s); break;
            case 10: big ? tsort_launch<10, 1024, true>(c, src0, dstN, n, kb, passes, s) : tsort_launch<10, kSortNT, !kSortPF>(c, src0, dstN, n, kb, passes, s); break;
            default: big ? tsort_launch<11, 1024, true>(c, src0, dstN, n, kb, passes, s) : tsort_launch<11, kSortNT, !kSortPF>(c, src0, dstN, n, kb, passes, s); break;
        }
        HIPCHK(c, hipGetLastError());
        return PFAAI_RC_OK;
    }
#endif
    switch (db) {
        case 8: tsort_launch<8, kSortNT, kSortPF>(c, src0, dstN, n, kb, passes, s); break;
        case 9: tsort_launch<9, kSortNT, kSortPF>(c, src0, dstN, n, kb, passes, s); break;
        case 10: tsort_launch<10, kSortNT, kSortPF>(c, src0, dstN, n, kb, passes, s); break;
        default: tsort_launch<11, kSortNT, kSortPF>(c, src0, dstN, n, kb, passes, s); break;
    }
    HIPCHK(c, hipGetLastError());
    return PFAAI_RC_OK;
}

void release_tsort(pfaai_ctx* c) {
    for (DevBuf* b : {&c->srec_a, &c->srec_b, &c->shist, &c->sgsum, &c->sbase, &c->tails, &c->ranks}) release(*b);
}

// F only: G_off from T, records (k_fkeys_rec: key, tetramer, block offset)
// -> the sort -> DstGFromRecs builds G_tet / G_pos.  Returns -1 if the
// records do not fit 64 bits or T disagrees with F: the caller takes
// build_g_from_f.
int build_g_from_f_sorted(pfaai_ctx* c, int64_t ng, int64_t n_f, int jb, bool want_pos, hipStream_t s) {
    const int32_t P = c->prob.n_prot, ni = c->prob.n_ids;
    const int kb = bits_for(ng);
    if (kb + 18 + jb > 64) return -1;
    int rc;
    if ((rc = ensure_tsort(c, n_f, kb, true)) || (rc = ensure(c, c->G_off, (ng + 1) * 8)) ||
        (rc = ensure(c, c->G_tet, std::max<int64_t>(n_f, 1) * 4)) || (rc = ensure(c, c->cnt_t, std::max<int64_t>(ng, 1) * 4)) ||
        (rc = ensure_scan(c, ng)))
        return rc;
    auto* sc = static_cast<unsigned long long*>(c->scalars.p);
    int* err = reinterpret_cast<int*>(sc + SC_ERR);
    HIPCHK(c, hipMemsetAsync(err, 0, sizeof(int), s));
    auto* len = static_cast<uint32_t*>(c->cnt_t.p);
    hipLaunchKernelGGL(k_len_from_t, dim3((int)std::min<int64_t>(ceil_div(ng, 256), 8192)), dim3(256), 0, s,
                       static_cast<const int32_t*>(c->T.p), P, ni, c->prob.t_cols, len);
    if ((rc = scan_u32(c, len, ng, static_cast<unsigned long long*>(c->G_off.p), s))) return rc;
    hipLaunchKernelGGL(k_fkeys_rec, dim3(8192), dim3(256), 0, s, static_cast<const int64_t*>(c->Lp.p),
                       static_cast<const int32_t*>(c->Fp.p), static_cast<const int32_t*>(c->Fg.p), (uint32_t)P, kb,
                       static_cast<uint64_t*>(c->srec_b.p), static_cast<uint16_t*>(c->Fp16.p));
    HIPCHK(c, hipGetLastError());
    const SrcRecs src{static_cast<const uint64_t*>(c->srec_b.p)};
    const DstGFromRecs dst{want_pos ? static_cast<uint32_t*>(c->G_pos.p) : nullptr, static_cast<int32_t*>(c->G_tet.p),
                           static_cast<const int64_t*>(c->G_off.p), static_cast<const int64_t*>(c->Lp.p), kb, err};
    if ((rc = tsort(c, src, dst, n_f, kb, s))) return rc;
    int bad = 0;
    HIPCHK(c, hipMemcpyAsync(&bad, err, sizeof(int), hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    return bad ? -1 : PFAAI_RC_OK;
}

// Both F and G given with |G| = |F|: G must be F's genome-major transpose.
// One two-pass sort of F by (genome, protein) -- records (key, F index),
// read straight from F -- yields G_pos (into gpos); k_hash_f sums the F side
// of the membership check (pfaai_sort.hpp, DstGpos) on the second stream
// beside the sort.  The G side comes from k_gend (HASH), launched by
// load_impl, which then compares the two (finish_g_check).
int check_g_transpose(pfaai_ctx* c, int64_t n_f, uint32_t* gpos, uint64_t seed, uint64_t seed2, hipStream_t s) {
    const int kb = bits_for((int64_t)c->prob.n_ids * c->prob.n_prot);
    int rc;
    if ((rc = ensure_tsort(c, n_f, kb, false))) return rc;
    auto* sc = static_cast<unsigned long long*>(c->scalars.p);
    HIPCHK(c, hipMemsetAsync(sc + SC_HF, 0, 4 * sizeof(unsigned long long), s));  // SC_HF, SC_HG, SC_HF2, SC_HG2
    const SrcFKeys src{static_cast<const int32_t*>(c->Fp.p), static_cast<const int32_t*>(c->Fg.p),
                       (uint32_t)c->prob.n_prot, static_cast<uint16_t*>(c->Fp16.p)};
    const DstGpos dst{gpos};
    // the F side runs on the second stream beside the sort (its VALU work
    // beside HBM-bound passes); the load's stream waits for it after the sort
    if (!c->copy_stream) HIPCHK(c, hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
    hipEvent_t* ev = c->side_ev;
    for (int k = 0; k < 2; ++k)
        if (!ev[k]) HIPCHK(c, hipEventCreateWithFlags(&ev[k], hipEventDisableTiming));
    HIPCHK(c, hipEventRecord(ev[0], s));  // (after the sums were cleared)
    HIPCHK(c, hipStreamWaitEvent(c->copy_stream, ev[0], 0));
    hipLaunchKernelGGL(k_hash_f, dim3(8192), dim3(256), 0, c->copy_stream, static_cast<const int64_t*>(c->Lp.p),
                       static_cast<const int32_t*>(c->Fp.p), static_cast<const int32_t*>(c->Fg.p),
                       (uint32_t)c->prob.n_prot, seed, seed2, sc + SC_HF, 0, c->prob.n_ids);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(ev[1], c->copy_stream));
    rc = tsort(c, src, dst, n_f, kb, s);
    // the join also on failure: a later load clears SC_HF on s, which must
    // not overtake k_hash_f still adding into it on copy_stream
    const hipError_t we = hipStreamWaitEvent(s, ev[1], 0);
    if (rc) return rc;
    HIPCHK(c, we);
    return PFAAI_RC_OK;
}

// G only, all-vs-all (the CLI's `<p>_genomes` load): G_pos, the F index of
// every G entry, by the sort the both-given load runs (F by genome * P +
// protein, records read straight from F, DstGpos) over the F that
// build_f_from_g_sorted just built from G.  F is G's transpose by
// construction, so the sorted positions are G's and nothing is checked; the
// row kernels then take the benchmarked WK 3 form (G_pos + G_end) on this
// path too.
int build_gpos_from_f(pfaai_ctx* c, int64_t n_f, hipStream_t s) {
    const int kb = bits_for((int64_t)c->prob.n_ids * c->prob.n_prot);
    int rc;
    if ((rc = ensure_tsort(c, n_f, kb, false))) return rc;
    const SrcFKeys src{static_cast<const int32_t*>(c->Fp.p), static_cast<const int32_t*>(c->Fg.p),
                       (uint32_t)c->prob.n_prot, nullptr};
    const DstGpos dst{static_cast<uint32_t*>(c->G_pos.p)};
    return tsort(c, src, dst, n_f, kb, s);
}

// All-vs-all G_pos and G_end of the lists of genomes [g_lo, g_hi) (G index
// gbase.., n_kept entries) by the F -> G sort that carries run ends
// (pfaai_sort.hpp: k_block_ends, k_fends_hist writes each entry's distance to
// its run end, SrcFEnds / DstRecsEnds / DstGposEnds): two passes over F and no
// run-end table or per-entry lookup.  check (seeds): the both-given
// membership sums of those genomes -- the F side in k_fends_hist (per tile,
// added up by k_sum_pairs), the G side (k_hash_g) on the second stream
// beside the whole sort.  Returns -1 where the records do
// not fit two passes (the caller takes check_g_transpose / the plain G_pos
// sort + k_blk_end + k_gend).
template <int DB>
int gpos_ends_passes(pfaai_ctx* c, int64_t n_f, int kb, int32_t g_lo, int32_t g_hi, int64_t gbase, int64_t n_kept,
                     const uint64_t* seeds, hipStream_t s) {
    constexpr int NT = kSortNT;
    static_assert(sort_tile<NT>() == kEndsTile, "the run-end tiles are the sort's tiles");
    const int32_t P = c->prob.n_prot;
    const int hb = kb - DB;
    const int64_t kT = sort_tile<NT>(), ntiles = ceil_div(n_f, kT), ngroups = ceil_div(ntiles, kSortGroup);
    auto* hist = static_cast<uint32_t*>(c->shist.p);
    auto* gsum = static_cast<uint32_t*>(c->sgsum.p);
    auto* base = static_cast<uint32_t*>(c->sbase.p);
    uint32_t* tctr = base + (1 << DB);
    auto* bend = static_cast<uint32_t*>(c->tails.p);
    const int64_t nwords = ceil_div(n_f, 32);
    uint32_t* tcnt = bend + nwords;    // block ends per tile (the check's ranks; zeroed with bend)
    uint32_t* ftail = tcnt + ntiles;
    uint32_t* ntail = ftail + ntiles;
    uint32_t* ltail = ntail + ntiles;
    uint32_t* flag = ltail + ntiles;   // non-empty tetramer blocks, then the list of them (tnz)
    auto* trank = static_cast<unsigned long long*>(c->ranks.p);  // [ntiles + 1]
    unsigned long long* rho = trank + ntiles + 1;                // [160001]
    unsigned long long* hpart = rho + kNTetramers + 1;           // [2 * ntiles]: the F side's per-tile sums
    auto* D = static_cast<uint32_t*>(c->srec_b.p);
    auto* sc = static_cast<unsigned long long*>(c->scalars.p);
    const auto* Lp = static_cast<const int64_t*>(c->Lp.p);
    const auto* Fp = static_cast<const int32_t*>(c->Fp.p);
    const auto* Fg = static_cast<const int32_t*>(c->Fg.p);
    HIPCHK(c, hipMemsetAsync(bend, 0, (nwords + (seeds ? ntiles : 0)) * 4, s));
    if (seeds) {  // the G side of the check (reads G only) beside the whole sort: 0.34 ms alone at 10k
        HIPCHK(c, hipMemsetAsync(sc + SC_HF, 0, 4 * sizeof(unsigned long long), s));
        HIPCHK(c, hipEventRecord(c->side_ev[0], s));
        HIPCHK(c, hipStreamWaitEvent(c->copy_stream, c->side_ev[0], 0));
        const int64_t nch = ceil_div((int64_t)(g_hi - g_lo) * P, 64);
        hipLaunchKernelGGL(k_hash_g, dim3((int)std::clamp<int64_t>(ceil_div(nch, 4), 1, 2048)), dim3(256), 0,
                           c->copy_stream, static_cast<const int64_t*>(c->G_off.p),
                           static_cast<const int32_t*>(c->G_tet.p), P, g_lo, g_hi, seeds[0], seeds[1], sc + SC_HG);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipEventRecord(c->side_ev[1], c->copy_stream));
    }
    hipLaunchKernelGGL(k_block_ends, dim3(ceil_div(kNTetramers, 256)), dim3(256), 0, s, Lp, bend,
                       seeds ? tcnt : nullptr, flag);
    if (seeds) {  // the F side's tetramers: block ranks per tile, the non-empty blocks (k_tnz)
        int rc;
        if ((rc = scan_u32(c, tcnt, ntiles, trank, s)) || (rc = scan_u32(c, flag, kNTetramers, rho, s))) return rc;
        hipLaunchKernelGGL(k_tnz, dim3(ceil_div(kNTetramers, 256)), dim3(256), 0, s, rho, flag);
    }
    const uint32_t mask1 = (1u << DB) - 1u, mask2 = (1u << hb) - 1u;
    // the WK 3 member codes (k_fcode's), written by the histogram pass
    if (int rc = ensure(c, c->Fcode, (size_t)(n_f + 16) * sizeof(uint32_t))) return rc;
    HIPCHK(c, hipMemsetAsync(static_cast<uint32_t*>(c->Fcode.p) + n_f, 0, 16 * sizeof(uint32_t), s));
    hipLaunchKernelGGL((k_fends_hist<DB, NT>), dim3(ntiles), dim3(NT), 0, s, Fp, Fg, bend, n_f, (uint32_t)P, g_lo, g_hi,
                       mask1, static_cast<uint16_t*>(c->Fp16.p), D, hist, ftail, ltail, trank, flag,
                       seeds ? seeds[0] : 0ull, seeds ? seeds[1] : 0ull, seeds ? hpart : nullptr,
                       static_cast<uint32_t*>(c->Fcode.p));
    HIPCHK(c, hipGetLastError());
    hipLaunchKernelGGL(k_tail_suffix, dim3((int)std::min<int64_t>(ceil_div(ntiles, 256), 4096)), dim3(256), 0, s, ftail,
                       ntiles, ntail);
    hipLaunchKernelGGL(k_fix_open, dim3((int)std::min<int64_t>(ceil_div(ntiles, 4), 65536)), dim3(256), 0, s, ltail, ntail,
                       ntiles, n_f, D);
    hipLaunchKernelGGL((k_sort_grp<DB>), dim3(ngroups), dim3(kSortThreads), 0, s, hist, ntiles, gsum);
    hipLaunchKernelGGL((k_sort_top<DB>), dim3(1), dim3(kSortThreads), 0, s, gsum, ngroups, base, tctr);
    if (seeds) hipLaunchKernelGGL(k_sum_pairs, dim3(256), dim3(256), 0, s, hpart, ntiles, sc + SC_HF);
    const size_t lds = sort_scatter_lds<DB, NT>();
    int cus = 256, per1 = 1, per2 = 1;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per1, reinterpret_cast<const void*>(&k_sort_scatter<DB, NT, kSortPF, SrcFEnds, DstRecsEnds>), NT, lds);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per2, reinterpret_cast<const void*>(&k_sort_scatter<DB, NT, kSortPF, SrcRecs, DstGposEnds>), NT, lds);
    auto* rec = static_cast<uint64_t*>(c->srec_a.p);
    const SrcFEnds src{Fp, Fg, D, (uint32_t)P, kb, g_lo, g_hi, 2 * n_kept < n_f};
    // (PFAAI_SORT_DIRECT, diagnostics: both passes store each record from its
    // registers, k_sort_scatter VAR bit 6, A/B of the LDS reorder)
#ifdef PFAAI_DIAGNOSTICS
    const bool sdirect = DIAG_ENV("PFAAI_SORT_DIRECT") != nullptr;
    if (sdirect)
        hipLaunchKernelGGL((k_sort_scatter<DB, NT, kSortPF, SrcFEnds, DstRecsEnds, 64>),
                           dim3((int)std::min<int64_t>(ntiles, (int64_t)cus * std::max(1, per1))), dim3(NT), lds, s,
                           src, DstRecsEnds{rec, kb, DB}, n_f, ntiles, 0, mask1, hist, gsum, base, tctr);
    else
#endif
    hipLaunchKernelGGL((k_sort_scatter<DB, NT, kSortPF, SrcFEnds, DstRecsEnds>),
                       dim3((int)std::min<int64_t>(ntiles, (int64_t)cus * std::max(1, per1))), dim3(NT), lds, s, src,
                       DstRecsEnds{rec, kb, DB}, n_f, ntiles, 0, mask1, hist, gsum, base, tctr);
    HIPCHK(c, hipGetLastError());
    if (n_kept > 0) {
        const int64_t nt2 = ceil_div(n_kept, kT), ng2 = ceil_div(nt2, kSortGroup);
        const SrcRecs src2{rec};
        hipLaunchKernelGGL((k_sort_hist<DB, NT, SrcRecs>), dim3(nt2), dim3(NT), 0, s, src2, n_kept, 0, mask2, hist);
        hipLaunchKernelGGL((k_sort_grp<DB>), dim3(ng2), dim3(kSortThreads), 0, s, hist, nt2, gsum);
        hipLaunchKernelGGL((k_sort_top<DB>), dim3(1), dim3(kSortThreads), 0, s, gsum, ng2, base, tctr);
#ifdef PFAAI_DIAGNOSTICS
        if (sdirect)
            hipLaunchKernelGGL((k_sort_scatter<DB, NT, kSortPF, SrcRecs, DstGposEnds, 64>),
                               dim3((int)std::min<int64_t>(nt2, (int64_t)cus * std::max(1, per2))), dim3(NT), lds, s,
                               src2, DstGposEnds{static_cast<uint2*>(c->G_pe.p) + gbase, hb}, n_kept, nt2, 0, mask2,
                               hist, gsum, base, tctr);
        else
#endif
        hipLaunchKernelGGL((k_sort_scatter<DB, NT, kSortPF, SrcRecs, DstGposEnds>),
                           dim3((int)std::min<int64_t>(nt2, (int64_t)cus * std::max(1, per2))), dim3(NT), lds, s, src2,
                           DstGposEnds{static_cast<uint2*>(c->G_pe.p) + gbase, hb},
                           n_kept, nt2, 0, mask2, hist, gsum, base, tctr);
        HIPCHK(c, hipGetLastError());
    }
    return PFAAI_RC_OK;
}

// the run-end sort's buffers: records (srec_a), run-end distances (srec_b,
// u32), the block-end bitmap + per-tile run ends (tails), tile histograms
int ensure_gpos_ends(pfaai_ctx* c, int64_t n_f, int64_t n_kept, int db) {
    const int64_t ntiles = ceil_div(std::max<int64_t>(n_f, 1), sort_tile<kSortNT>());
    int rc;
    if ((rc = ensure(c, c->srec_a, (size_t)std::max<int64_t>(n_kept, 1) * 8)) ||
        (rc = ensure(c, c->srec_b, (size_t)std::max<int64_t>(n_f, 1) * 4)) ||
        (rc = ensure(c, c->shist, (size_t)ntiles * (4u << db))) ||
        (rc = ensure(c, c->sgsum, (size_t)ceil_div(ntiles, kSortGroup) * (4u << db))) ||
        (rc = ensure(c, c->sbase, (4u << db) + 64)) ||
        (rc = ensure(c, c->tails, (size_t)(ceil_div(std::max<int64_t>(n_f, 1), 32) + 4 * ntiles + kNTetramers) * 4)) ||
        (rc = ensure(c, c->ranks, (size_t)(ntiles + 1 + kNTetramers + 1 + 2 * ntiles) * 8)) ||
        (rc = ensure_scan(c, std::max<int64_t>(ntiles, kNTetramers))))
        return rc;
    return PFAAI_RC_OK;
}

int build_gpos_ends(pfaai_ctx* c, int64_t n_f, int32_t g_lo, int32_t g_hi, int64_t gbase, int64_t n_kept,
                    const uint64_t* seeds, hipStream_t s) {
    const int32_t P = c->prob.n_prot;
    const int kb = bits_for((int64_t)c->prob.n_ids * P);
    int passes;
    const int db = tsort_db(kb, &passes);
    if (passes != 2 || kb + 33 > 63 || db < 8 || db > 11 || n_f == 0) return -1;
    int rc;
    if ((rc = ensure_gpos_ends(c, n_f, n_kept, db))) return rc;
    if (seeds && !c->copy_stream) HIPCHK(c, hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
    switch (db) {
        case 8: rc = gpos_ends_passes<8>(c, n_f, kb, g_lo, g_hi, gbase, n_kept, seeds, s); break;
        case 9: rc = gpos_ends_passes<9>(c, n_f, kb, g_lo, g_hi, gbase, n_kept, seeds, s); break;
        case 10: rc = gpos_ends_passes<10>(c, n_f, kb, g_lo, g_hi, gbase, n_kept, seeds, s); break;
        default: rc = gpos_ends_passes<11>(c, n_f, kb, g_lo, g_hi, gbase, n_kept, seeds, s); break;
    }
    if (seeds) {  // join (also on failure: nothing may overtake the sums on copy_stream)
        const hipError_t we = hipStreamWaitEvent(s, c->side_ev[1], 0);
        if (!rc && we != hipSuccess) return hip_fail(c, we, "hipStreamWaitEvent");
    }
    return rc;
}

// (before the load's device span: allocation inside it leaves the stream idle)
int ensure_gpos_ends_pre(pfaai_ctx* c, int64_t n_f, int64_t n_kept, int64_t ng) {
    int passes;
    const int db = tsort_db(bits_for(ng), &passes);
    return passes == 2 && db >= 8 && db <= 11 ? ensure_gpos_ends(c, n_f, n_kept, db) : PFAAI_RC_OK;
}

// After k_gend<*, true>: -1 unless the F and G membership sums agree.
int finish_g_check(pfaai_ctx* c, hipStream_t s) {
    unsigned long long h[4] = {0, 0, 0, 0};
    HIPCHK(c, hipMemcpyAsync(h, static_cast<unsigned long long*>(c->scalars.p) + SC_HF, sizeof(h), hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    return h[0] != h[1] || h[2] != h[3] ? -1 : PFAAI_RC_OK;  // [HF, HG, HF2, HG2]
}

// G only (the CLI's `<p>_genomes` ingest): the G entries enumerated
// protein-major (k_gkeys_pm), one two-pass sort by tetramer (18-bit keys,
// 9-bit digits) -> F (t, p, g) and Fp16 (DstFFromG), Lp from the sorted
// tetramers (k_rowptr).  Needs P < 4096 and n_ids < 2^21 (the record
// fields); else the caller takes build_f_from_g.  G_pos, where the row
// kernels use it, comes from a second sort (build_gpos_from_f).
int build_f_from_g_sorted(pfaai_ctx* c, int64_t n_lists, int64_t n, hipStream_t s) {
    const int32_t P = c->prob.n_prot, ni = c->prob.n_ids;
    int rc;
    if ((rc = ensure_tsort(c, n, 18, true)) || (rc = ensure(c, c->cnt_t, std::max<int64_t>(n_lists, PFAAI_NTETRAMERS) * 4)) ||
        (rc = ensure(c, c->off_t, (n_lists + 1) * 8)) || (rc = ensure_scan(c, n_lists)))
        return rc;
    auto* len = static_cast<uint32_t*>(c->cnt_t.p);
    auto* pm_off = static_cast<unsigned long long*>(c->off_t.p);
    hipLaunchKernelGGL(k_len_pm, dim3((int)std::min<int64_t>(ceil_div(n_lists, 256), 8192)), dim3(256), 0, s,
                       static_cast<const int64_t*>(c->G_off.p), P, ni, len);
    if ((rc = scan_u32(c, len, n_lists, pm_off, s))) return rc;
    const int grid = (int)std::min<int64_t>(std::max<int64_t>(ceil_div(n_lists, 4), 1), 1 << 16);
    hipLaunchKernelGGL(k_gkeys_pm, dim3(grid), dim3(256), 0, s, static_cast<const int64_t*>(c->G_off.p),
                       static_cast<const int32_t*>(c->G_tet.p), n_lists, P, ni, pm_off,
                       static_cast<uint64_t*>(c->srec_b.p));
    HIPCHK(c, hipGetLastError());
    if (n == 0) {
        HIPCHK(c, hipMemsetAsync(c->Lp.p, 0, (PFAAI_NTETRAMERS + 1) * 8, s));
        return PFAAI_RC_OK;
    }
    // the last pass reads srec_a (two passes) or srec_b (three, diagnostics):
    // the tetramer column goes to the one it does not read
    int passes;
    (void)tsort_db(18, &passes);
    auto* ft = static_cast<uint32_t*>(passes == 2 ? c->srec_b.p : c->srec_a.p);
    const SrcRecs src{static_cast<const uint64_t*>(c->srec_b.p)};
    const DstFFromG dst{static_cast<int32_t*>(c->Fp.p), static_cast<int32_t*>(c->Fg.p),
                        static_cast<uint16_t*>(c->Fp16.p), ft};
    if ((rc = tsort(c, src, dst, n, 18, s))) return rc;
    hipLaunchKernelGGL(k_rowptr, dim3(ceil_div(n, 256)), dim3(256), 0, s, ft, n, (int64_t)PFAAI_NTETRAMERS,
                       static_cast<unsigned long long*>(c->Lp.p));
    HIPCHK(c, hipGetLastError());
    return PFAAI_RC_OK;
}

// rows_lo / rows_hi: the all-vs-all rows (genomes) whose walk data (G_pos,
// G_end) the load builds, [0, n_ids) by default (pfaai_load_rows).
int load_impl(pfaai_ctx* c, const pfaai_problem* pb, int64_t rows_lo = 0, int64_t rows_hi = -1) {
    HIPCHK(c, hipSetDevice(c->device));
    c->loaded = false;
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    double ms_upload = 0.0;
    const pfaai_problem& p = *pb;
    if (p.mode < 0 || p.mode > 2) return fail(c, PFAAI_RC_INVALID, "mode must be 0, 1 or 2");
    if (p.n_ids < 2 || p.n_prot < 1 || p.n_prot >= kMaxRuns || p.t_cols < 1)
        return fail(c, PFAAI_RC_INVALID, "bad sizes (n_ids >= 2, 1 <= n_prot < 4096)");
    // 21-bit genome ids (run-table splitters, first-key packing); F indices
    // are u32 in the run table / work lists (and 16-B records in k_rows_pl)
    if (p.n_ids >= (1 << 21)) return fail(c, PFAAI_RC_INVALID, "n_ids must be < 2^21");
    const bool in_f = p.Lp || p.F_prot || p.F_genome;
    const bool in_g = p.G_off || p.G_tet;
    if (in_f && !(p.Lp && p.F_prot && p.F_genome))
        return fail(c, PFAAI_RC_INVALID, "Lp, F_prot and F_genome are required together");
    if (in_g && !(p.G_off && p.G_tet)) return fail(c, PFAAI_RC_INVALID, "G_off and G_tet are required together");
    if (!in_f && !in_g) return fail(c, PFAAI_RC_INVALID, "F (Lp, F_prot, F_genome) or G (G_off, G_tet) is required");
    if (!p.T) return fail(c, PFAAI_RC_INVALID, "T is required");
    if (p.mode != PFAAI_MODE_ALL && !p.is_q) return fail(c, PFAAI_RC_INVALID, "is_q is required for QSUB/QT");
    if (p.mode == PFAAI_MODE_QSUB && (!p.q_index || !p.t_rank))
        return fail(c, PFAAI_RC_INVALID, "q_index and t_rank are required for QSUB");
    if (p.mode == PFAAI_MODE_QT && p.n_ids != p.n_tgt + p.n_qry)
        return fail(c, PFAAI_RC_INVALID, "QT: n_ids must equal n_tgt + n_qry");
    if (p.t_cols < p.n_ids) return fail(c, PFAAI_RC_INVALID, "T needs a column per genome id");
    const int32_t ni = p.n_ids, P = p.n_prot;
    // T must hold every count < 2^16 (packed u16 LDS counters; c <= min T)
    const int64_t tn = (int64_t)P * p.t_cols;
    {
        std::atomic<int> bad{0};
        par_for(tn, [&](int64_t lo, int64_t hi, int) {
            for (int64_t i = lo; i < hi; ++i)
                if (p.T[i] < 0 || p.T[i] > 65535) { bad = 1; return; }
        });
        if (bad) return fail(c, PFAAI_RC_INVALID, "T entries must lie in [0, 65535]");
    }

    // G: offsets first (they bound every G_tet access), then the entries:
    // tetramer ids in range, each (genome, protein) list strictly ascending
    const int64_t ng = (int64_t)ni * P;
    int64_t n_g = 0;
    c->max_glen = 0;
    c->t_exact = false;
    if (in_g) {
        if (p.G_off[0] != 0) return fail(c, PFAAI_RC_INVALID, "G_off must start at 0");
        std::atomic<int> bad_off{0};
        par_for(ng, [&](int64_t lo, int64_t hi, int) {
            for (int64_t k = lo; k < hi; ++k)
                if (p.G_off[k + 1] < p.G_off[k]) { bad_off = 1; return; }
        });
        if (bad_off) return fail(c, PFAAI_RC_INVALID, "G_off must be non-decreasing");
        n_g = p.G_off[ng];
        if (n_g > kMaxF) return fail(c, PFAAI_RC_INVALID, "|G| must be <= 2^32 - 64");
        std::atomic<int> bad_t{0}, bad_ord{0}, t_diff{0};
        std::vector<int64_t> mx(16, 0);
        par_for(
            ng,
            [&](int64_t lo, int64_t hi, int th) {
                int64_t m = 0;
                bool td = false;
                for (int64_t k = lo; k < hi; ++k) {
                    const int64_t b = p.G_off[k], e = p.G_off[k + 1];
                    m = std::max(m, e - b);
                    const int64_t g = k / P, q = k - g * P;  // list k = (genome g, protein q)
                    td = td || g >= p.t_cols || (int64_t)p.T[q * p.t_cols + g] != e - b;
                    for (int64_t i = b; i < e; ++i) {
                        if (p.G_tet[i] < 0 || p.G_tet[i] >= PFAAI_NTETRAMERS) { bad_t = 1; return; }
                        if (i > b && p.G_tet[i] <= p.G_tet[i - 1]) { bad_ord = 1; return; }
                    }
                }
                mx[th] = m;
                if (td) t_diff = 1;
            },
            n_g);
        c->t_exact = !t_diff;
        if (bad_t) return fail(c, PFAAI_RC_INVALID, "G_tet holds a tetramer id outside [0, 160000)");
        if (bad_ord) return fail(c, PFAAI_RC_INVALID, "every G list must be strictly ascending");
        for (int64_t m : mx) c->max_glen = std::max(c->max_glen, m);
    }

    // F: Lp first (it bounds every F access): starts at 0, ends at n_f,
    // non-decreasing; then ids in range and the (tetramer, protein, genome)
    // order of ds_helper.hpp:126-162 that the run table relies on
    const int64_t n_f = in_f ? p.n_f : n_g;
    if (n_f < 0 || n_f > kMaxF) return fail(c, PFAAI_RC_INVALID, "|F| must be <= 2^32 - 64");
    std::vector<int64_t> fcount(ni, 0);  // F entries per genome (work-list sizes)
    int64_t max_lc = 0;                  // largest tetramer block of F
    if (in_f) {
        if (p.Lp[0] != 0 || p.Lp[PFAAI_NTETRAMERS] != p.n_f)
            return fail(c, PFAAI_RC_INVALID, "Lp must start at 0 and end at n_f");
        for (int t = 0; t < PFAAI_NTETRAMERS; ++t) {
            if (p.Lp[t + 1] < p.Lp[t]) return fail(c, PFAAI_RC_INVALID, "Lp must be non-decreasing");
            max_lc = std::max<int64_t>(max_lc, p.Lp[t + 1] - p.Lp[t]);
        }
        if (in_g && n_g < n_f) return fail(c, PFAAI_RC_INVALID, "G must hold every membership of F (|G| < |F|)");
        std::vector<std::vector<int64_t>> fc(16);
        std::atomic<int> bad_id{0}, bad_p{0}, bad_sort{0};
        const int nth = par_for(p.n_f, [&](int64_t lo, int64_t hi, int t) {
            std::vector<int64_t>& cnt = fc[t];
            cnt.assign(ni, 0);
            for (int64_t i = lo; i < hi; ++i) {
                const int32_t g = p.F_genome[i];
                if (g < 0 || g >= ni) { bad_id = 1; return; }
                if (p.F_prot[i] < 0 || p.F_prot[i] >= P) { bad_p = 1; return; }
                cnt[g]++;
            }
        });
        if (bad_id) return fail(c, PFAAI_RC_INVALID, "F holds a genome id outside [0, n_ids)");
        if (bad_p) return fail(c, PFAAI_RC_INVALID, "F holds a protein id outside [0, n_prot)");
        for (int t = 0; t < nth; ++t)
            for (int32_t g = 0; g < ni; ++g) fcount[g] += fc[t][g];
        par_for(
            PFAAI_NTETRAMERS,
            [&](int64_t lo, int64_t hi, int) {
                for (int64_t t = lo; t < hi; ++t)
                    for (int64_t i = p.Lp[t] + 1; i < p.Lp[t + 1]; ++i)
                        if (p.F_prot[i] < p.F_prot[i - 1] ||
                            (p.F_prot[i] == p.F_prot[i - 1] && p.F_genome[i] <= p.F_genome[i - 1])) {
                            bad_sort = 1;
                            return;
                        }
            },
            p.n_f);
        if (bad_sort) return fail(c, PFAAI_RC_INVALID, "F must be sorted by (tetramer, protein, genome)");
    } else {
        for (int32_t g = 0; g < ni; ++g) fcount[g] = p.G_off[(int64_t)(g + 1) * P] - p.G_off[(int64_t)g * P];
    }

    c->prob = p;
    c->prob.n_f = n_f;
    // borrowed host arrays are not kept past this call
    c->prob.Lp = nullptr;
    c->prob.F_prot = c->prob.F_genome = c->prob.T = nullptr;
    c->prob.is_q = nullptr;
    c->prob.q_index = c->prob.t_rank = nullptr;
    c->prob.G_off = nullptr;
    c->prob.G_tet = nullptr;
    c->runs_valid = c->runs_key = false;
    c->win_valid = c->win_key = false;
    // output rows and derived maps
    std::vector<int32_t> row_of(ni, -1), tcol_row(ni), tcol_col(ni);
    c->row_genome_h.clear();
    c->q_index_h.clear();
    c->order_n = 0;
    c->order_in_pos = false;
    if (p.mode == PFAAI_MODE_ALL) {
        for (int32_t g = 0; g < ni; ++g) { row_of[g] = g; c->row_genome_h.push_back(g); }
        c->n_rows = ni;
        c->n_pairs = (int64_t)ni * (ni - 1) / 2;
        c->max_cols = ni - 1;
        c->prob.n_qry = ni;
        c->prob.n_tgt = 0;
    } else if (p.mode == PFAAI_MODE_QSUB) {
        c->row_genome_h.assign(p.n_qry, -1);
        c->q_index_h.assign(p.q_index, p.q_index + ni);
        for (int32_t g = 0; g < ni; ++g) {
            if (!p.is_q[g]) continue;
            const int32_t qi = p.q_index[g];
            if (qi < 0 || qi >= p.n_qry) return fail(c, PFAAI_RC_INVALID, "q_index out of range");
            row_of[g] = qi;
            c->row_genome_h[qi] = g;
        }
        for (int32_t x : c->row_genome_h)
            if (x < 0) return fail(c, PFAAI_RC_INVALID, "query list has holes");
        c->n_rows = p.n_qry;
        c->n_pairs = (int64_t)p.n_qry * p.n_tgt + (int64_t)p.n_qry * (p.n_qry - 1) / 2;
        c->max_cols = ni;
    } else {
        for (int32_t q = 0; q < p.n_qry; ++q) {
            row_of[p.n_tgt + q] = q;
            c->row_genome_h.push_back(p.n_tgt + q);
        }
        c->n_rows = p.n_qry;
        c->n_pairs = (int64_t)p.n_qry * p.n_tgt;
        c->max_cols = p.n_tgt;
    }
    c->cols_run = c->max_cols;
    for (int32_t g = 0; g < ni; ++g) { tcol_row[g] = g; tcol_col[g] = g; }
    // QT reference T-index quirk: the reference reads
    // T[p][i / nT] and T[p][nQ + i % nT] for JAC index i = q*nT + t.  Both
    // are per-genome remaps, applied only under PFAAI_FLAG_REF_COMPAT.
    if (p.mode == PFAAI_MODE_QT) {
        for (int32_t q = 0; q < p.n_qry; ++q) tcol_row[p.n_tgt + q] = q;
        for (int32_t t = 0; t < p.n_tgt; ++t) tcol_col[t] = p.n_qry + t;
        for (int32_t g = 0; g < ni; ++g)
            if (tcol_row[g] >= p.t_cols || tcol_col[g] >= p.t_cols) {
                // compat maps out of T: clamp to identity (compat is then undefined, as in the reference)
                tcol_row[g] = std::min(tcol_row[g], p.t_cols - 1);
                tcol_col[g] = std::min(tcol_col[g], p.t_cols - 1);
            }
    }

    int rc;
    hipStream_t s = c->stream;
    const auto t1 = clk::now();  // host checks done
    if ((rc = upload(c, c->T, p.T, tn))) return rc;
    std::vector<uint8_t> isq(ni, 1);
    if (p.is_q) isq.assign(p.is_q, p.is_q + ni);
    if ((rc = upload(c, c->is_q, isq.data(), ni))) return rc;
    std::vector<int32_t> qidx(ni, -1), trank(ni, -1);
    if (p.q_index) qidx.assign(p.q_index, p.q_index + ni);
    if (p.t_rank) trank.assign(p.t_rank, p.t_rank + ni);
    if ((rc = upload(c, c->q_index, qidx.data(), ni))) return rc;
    if ((rc = upload(c, c->t_rank, trank.data(), ni))) return rc;
    if ((rc = upload(c, c->row_of, row_of.data(), ni))) return rc;
    if ((rc = upload(c, c->row_genome, c->row_genome_h.data(), c->row_genome_h.size()))) return rc;
    if ((rc = upload(c, c->tcol_row, tcol_row.data(), ni))) return rc;
    if ((rc = upload(c, c->tcol_col, tcol_col.data(), ni))) return rc;

    // u16 T by column genome id (and through tcol_col for the QT quirk), rows
    // of an even number of columns so one u32 holds a counter word's pair
    c->dev.t16_cols = ((int64_t)ni + 15) & ~(int64_t)7;  // 16-B rows, >= n_ids + 8 (uint4 reads past chi)
    {
        const int64_t tc = c->dev.t16_cols;
        std::vector<uint16_t> t16((size_t)P * tc, 0);
        for (int64_t q = 0; q < P; ++q)
            for (int32_t g = 0; g < ni; ++g) t16[q * tc + g] = (uint16_t)p.T[q * p.t_cols + g];
        if ((rc = upload(c, c->T16, t16.data(), t16.size()))) return rc;
        if (p.mode == PFAAI_MODE_QT) {
            for (int64_t q = 0; q < P; ++q)
                for (int32_t g = 0; g < ni; ++g) t16[q * tc + g] = (uint16_t)p.T[q * p.t_cols + tcol_col[g]];
            if ((rc = upload(c, c->T16c, t16.data(), t16.size()))) return rc;
        } else {
            release(c->T16c);
        }
    }

    // F and G on the device, whichever the caller did not give built from
    // the other (pfaai_build.hpp)
    if ((rc = ensure(c, c->Lp, (PFAAI_NTETRAMERS + 1) * sizeof(int64_t)))) return rc;
    if ((rc = ensure(c, c->Fp, std::max<int64_t>(n_f, 1) * sizeof(int32_t)))) return rc;
    if ((rc = ensure(c, c->Fg, (n_f + 16) * sizeof(int32_t)))) return rc;  // int4 reads may pass the end
    if (in_g) {
        if ((rc = upload(c, c->G_off, p.G_off, ng + 1))) return rc;
        if ((rc = upload(c, c->G_tet, p.G_tet, std::max<int64_t>(n_g, 1)))) return rc;
    }
    if (in_f) {
        if ((rc = upload(c, c->Lp, p.Lp, PFAAI_NTETRAMERS + 1))) return rc;
        if ((rc = upload(c, c->Fp, p.F_prot, n_f))) return rc;
        if ((rc = upload(c, c->Fg, p.F_genome, n_f))) return rc;
    }
    const auto t2 = clk::now();  // uploads done (hipMemcpy is synchronous)
    ms_upload = ms(t1, t2);
    // G_pos, the F index of every G entry, falls out of either transpose: the
    // all-vs-all row kernel starts each run walk just past the row genome
    // (k_rows_pl WK 3); not built for QSUB / QT or rows wider than two chunks
    bool pos_ok = false;
    if (p.mode == PFAAI_MODE_ALL && ni <= kGposMaxIds && n_f > 0) {
        if ((rc = ensure(c, c->G_pos, n_f * sizeof(uint32_t)))) return rc;
    } else {
        release(c->G_pos);
    }
    const bool want_pos = c->G_pos.p != nullptr;
    // the rows (genomes) whose G_pos / G_end are built: a rank's block (pfaai_load_rows)
    if (rows_hi < 0 || rows_hi > ni) rows_hi = ni;
    rows_lo = std::max<int64_t>(0, std::min<int64_t>(rows_lo, rows_hi));
    const int32_t g_lo = (int32_t)rows_lo, g_hi = (int32_t)rows_hi;
    const int64_t gbase = in_g ? p.G_off[(int64_t)g_lo * P] : 0, n_kept = in_g ? p.G_off[(int64_t)g_hi * P] - gbase : 0;
    bool ends_built = false;  // G_pos and G_end of [g_lo, g_hi) by the run-end sort (build_gpos_ends)
    // the u16 protein column (k_blk's run detection): written by the
    // transposition sorts on the way, else by k_fp16 below
    if ((rc = ensure(c, c->Fp16, (n_f + 16) * sizeof(uint16_t)))) return rc;  // 16-B reads may pass the end
    HIPCHK(c, hipMemsetAsync(c->Fp16.p, 0, (n_f + 16) * sizeof(uint16_t), s));
    // the both-given path's device buffers, allocated before the device span
    // starts (hipMalloc inside it left the stream idle: 8.5-9.0 ms measured
    // for 7.8 ms of kernels at 10k)
    if (in_g && in_f && n_f && n_g == n_f && ng < ((int64_t)1 << 32)) {
        if (want_pos && (rc = ensure_tsort(c, n_f, bits_for(ng), false))) return rc;
        if (want_pos && (rc = ensure(c, c->G_pe, n_f * sizeof(uint2)))) return rc;
        if (want_pos && (rc = ensure_gpos_ends_pre(c, n_f, n_kept, ng))) return rc;
        if ((rc = ensure(c, c->blk, (size_t)P * PFAAI_NTETRAMERS * sizeof(uint4)))) return rc;
    } else if (in_g && !in_f && n_f && P < kMaxRuns && ng < ((int64_t)1 << 32)) {  // G only: both sorts' buffers
        if ((rc = ensure_tsort(c, n_f, 18, true))) return rc;
        if (want_pos && (rc = ensure_tsort(c, n_f, bits_for(ng), false))) return rc;
        if (want_pos && (rc = ensure(c, c->G_pe, n_f * sizeof(uint2)))) return rc;
        if (want_pos && (rc = ensure_gpos_ends_pre(c, n_f, n_kept, ng))) return rc;
        if ((rc = ensure(c, c->blk, (size_t)P * PFAAI_NTETRAMERS * sizeof(uint4)))) return rc;
    }
    for (hipEvent_t& e : c->load_ev)
        if (!e) HIPCHK(c, hipEventCreate(&e));
    HIPCHK(c, hipEventRecord(c->load_ev[0], s));
    bool fp16_done = false;
    c->load_path = PFAAI_LOAD_AS_GIVEN;
    if (!in_f) {  // G only: F by the transposition sort (record fields permitting)
        if (P < kMaxRuns && ni < (1 << 21)) {
            if ((rc = build_f_from_g_sorted(c, ng, n_f, s))) return rc;
            fp16_done = true;
            c->load_path = PFAAI_LOAD_F_FROM_G;
            if (want_pos && ng < ((int64_t)1 << 32)) {  // the WK 3 walks' G_pos and G_end
                if (!(c->G_pe.p) && (rc = ensure(c, c->G_pe, n_f * sizeof(uint2)))) return rc;
                rc = build_gpos_ends(c, n_f, g_lo, g_hi, gbase, n_kept, nullptr, s);
                ends_built = rc == PFAAI_RC_OK;
                if (rc == -1 && (rc = build_gpos_from_f(c, n_f, s))) return rc;  // (G_end from k_gend below)
                if (rc) return rc;
                pos_ok = true;
            }
        } else {
            if ((rc = build_f_from_g(c, ng, n_f, s))) return rc;
            c->load_path = PFAAI_LOAD_LEGACY;
            pos_ok = true;  // (the general sort writes G_pos on the way)
        }
    }
    bool has_g = in_g;
    bool g_check = false;  // both given: the membership sums, completed by k_gend's G side
    uint64_t check_seed = 0, check_seed2 = 0;
    if (in_g && in_f && n_f && n_g == n_f && ng < ((int64_t)1 << 32)) {
        // both given, same size (ALL / QSUB, and QT with F's own G): G must BE
        // the transpose of F, proven by the membership sums over F (k_hash_f)
        // and over G (k_gend); G_pos, where the row kernels use it, from one
        // sort of F by (genome, protein).  Without G_pos no sort runs.
        check_seed = ((uint64_t)std::random_device{}() << 32) ^ (uint64_t)std::random_device{}() ^
                     (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
        check_seed2 = ((uint64_t)std::random_device{}() << 32) ^ (uint64_t)std::random_device{}();
        g_check = true;
        if (want_pos) {
            const uint64_t seeds[2] = {check_seed, check_seed2};
            rc = build_gpos_ends(c, n_f, g_lo, g_hi, gbase, n_kept, seeds, s);
            ends_built = rc == PFAAI_RC_OK;
            if (rc == -1 &&
                (rc = check_g_transpose(c, n_f, static_cast<uint32_t*>(c->G_pos.p), check_seed, check_seed2, s)))
                return rc;
            if (rc) return rc;
            fp16_done = true;
        } else {
            auto* sc = static_cast<unsigned long long*>(c->scalars.p);
            HIPCHK(c, hipMemsetAsync(sc + SC_HF, 0, 4 * sizeof(unsigned long long), s));
            hipLaunchKernelGGL(k_hash_f, dim3(8192), dim3(256), 0, s, static_cast<const int64_t*>(c->Lp.p),
                               static_cast<const int32_t*>(c->Fp.p), static_cast<const int32_t*>(c->Fg.p), (uint32_t)P,
                               check_seed, check_seed2, sc + SC_HF, 0, ni);
            HIPCHK(c, hipGetLastError());
        }
        pos_ok = true;
        c->load_path = PFAAI_LOAD_G_CHECKED;
    } else if (in_g && in_f && n_f) {  // both given, G larger (QT: both DBs' lists): G must hold F (k_g_check)
        auto* sc = static_cast<unsigned long long*>(c->scalars.p);
        int* err = reinterpret_cast<int*>(sc + SC_ERR);
        HIPCHK(c, hipMemsetAsync(err, 0, sizeof(int), s));
        HIPCHK(c, hipMemsetAsync(sc + SC_GRAND, 0, sizeof(unsigned long long), s));
        hipLaunchKernelGGL(k_g_check, dim3((int)std::min<int64_t>(ceil_div(ng, 4), 1 << 16)), dim3(256), 0, s,
                           static_cast<const int64_t*>(c->Lp.p), static_cast<const int32_t*>(c->Fp.p),
                           static_cast<const int32_t*>(c->Fg.p), static_cast<const int64_t*>(c->G_off.p),
                           static_cast<const int32_t*>(c->G_tet.p), ng, P, err, sc + SC_GRAND);
        HIPCHK(c, hipGetLastError());
        int bad = 0;
        unsigned long long found = 0;
        HIPCHK(c, hipMemcpyAsync(&bad, err, sizeof(int), hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(&found, sc + SC_GRAND, sizeof(found), hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        if (bad) return fail(c, PFAAI_RC_INVALID, "G lists a membership that F does not hold");
        if ((int64_t)found != n_f) return fail(c, PFAAI_RC_INVALID, "G does not hold every membership of F");
    } else if (!in_g && ng < ((int64_t)1 << 32)) {  // G from F (keys g * P + p fit 32 bits)
        // G_off from T when T counts exactly F's memberships per (genome,
        // protein) -- then one sort; else (or if any list bound disagrees) the
        // general radix sort with G_off from the sorted keys
        int64_t tsum = 0, tmax = 0;
        for (int64_t q = 0; q < P; ++q)
            for (int32_t g = 0; g < ni; ++g) {
                tsum += p.T[q * p.t_cols + g];
                tmax = std::max<int64_t>(tmax, p.T[q * p.t_cols + g]);
            }
        rc = tsum == n_f ? build_g_from_f_sorted(c, ng, n_f, bits_for(max_lc + 1), want_pos, s) : -1;
        if (rc == -1) {
            if ((rc = build_g_from_f(c, ng, n_f, s))) return rc;
            std::vector<int64_t> goff(ng + 1);
            HIPCHK(c, hipMemcpyAsync(goff.data(), c->G_off.p, (ng + 1) * sizeof(int64_t), hipMemcpyDeviceToHost, s));
            HIPCHK(c, hipStreamSynchronize(s));
            for (int64_t k = 0; k < ng; ++k) c->max_glen = std::max<int64_t>(c->max_glen, goff[k + 1] - goff[k]);
            c->load_path = PFAAI_LOAD_LEGACY;
        } else if (rc) {
            return rc;
        } else {
            c->max_glen = tmax;
            c->t_exact = true;  // G_off from T, every list bound verified against the sorted keys
            fp16_done = true;
            c->load_path = PFAAI_LOAD_G_FROM_F;
        }
        has_g = true;
        pos_ok = true;
    }
    c->has_g = has_g;
    if (!has_g) {
        release(c->G_off);
        release(c->G_tet);
    }
    if (!has_g || !pos_ok) release(c->G_pos);
    if (n_f && !fp16_done)
        hipLaunchKernelGGL(k_fp16, dim3((int)std::min<int64_t>(ceil_div(n_f, 256), 1 << 16)), dim3(256), 0, s,
                           static_cast<const int32_t*>(c->Fp.p), n_f, static_cast<uint16_t*>(c->Fp16.p));
    HIPCHK(c, hipGetLastError());
    if (has_g && (rc = ensure(c, c->blk, (size_t)P * PFAAI_NTETRAMERS * sizeof(uint4)))) return rc;

    Dev& d = c->dev;
    d.mode = p.mode;
    d.n_ids = ni;
    d.n_prot = P;
    d.t_cols = p.t_cols;
    d.n_qry = c->prob.n_qry;
    d.n_tgt = c->prob.n_tgt;
    d.n_f = n_f;
    d.Lp = static_cast<const int64_t*>(c->Lp.p);
    d.Fp = static_cast<const int32_t*>(c->Fp.p);
    d.Fg = static_cast<const int32_t*>(c->Fg.p);
    d.T = static_cast<const int32_t*>(c->T.p);
    d.is_q = static_cast<const uint8_t*>(c->is_q.p);
    d.q_index = static_cast<const int32_t*>(c->q_index.p);
    d.t_rank = static_cast<const int32_t*>(c->t_rank.p);
    d.row_of = static_cast<const int32_t*>(c->row_of.p);
    d.row_genome = static_cast<const int32_t*>(c->row_genome.p);
    d.tcol_row = static_cast<const int32_t*>(c->tcol_row.p);
    d.tcol_col = static_cast<const int32_t*>(c->tcol_col.p);
    d.G_off = has_g ? static_cast<const int64_t*>(c->G_off.p) : nullptr;
    d.G_tet = has_g ? static_cast<const int32_t*>(c->G_tet.p) : nullptr;
    const bool have_pos = c->G_pos.p != nullptr;
    d.blk = has_g ? static_cast<uint4*>(c->blk.p) : nullptr;
    d.Fp16 = static_cast<const uint16_t*>(c->Fp16.p);
    d.T16 = static_cast<const uint16_t*>(c->T16.p);
    d.T16c = c->T16c.p ? static_cast<const uint16_t*>(c->T16c.p) : d.T16;
    // G_end with G_pos: the end of the F run of every G entry -- carried by
    // the run-end sort (build_gpos_ends), else from the run-end table looked
    // up once here (k_blk_end + k_gend).  The WK 3 row kernel then reads
    // (G_pos, G_end) of its G entries with coalesced loads instead of one
    // run-table lookup per entry and step, and its steps build no run table.
    d.G_pe = nullptr;
    c->runs_valid = false;
    {
        // k_gend: G_end (with G_pos) and / or the G sides of the both-given check
        const int ggrid = (int)std::min<int64_t>(std::max<int64_t>(ceil_div(ng, kGendLists), 1), 1 << 16);
        auto* sums = static_cast<unsigned long long*>(c->scalars.p) + SC_HG;
        if (have_pos && ends_built) {  // G_pe came from the run-end sort; the G side of the check ran beside it
            d.G_pe = static_cast<const uint2*>(c->G_pe.p);
            release(c->G_pos);  // (not written on this path)
            release(c->G_end);
        } else if (have_pos) {
            if ((rc = ensure(c, c->G_end, std::max<int64_t>(n_f, 1) * sizeof(uint32_t)))) return rc;
            if ((rc = build_runs_g<0>(c, s, false, true))) return rc;  // the u32 run-end table, into blk
            const auto* ends = reinterpret_cast<const uint32_t*>(c->blk.p);
            auto* gend = static_cast<uint32_t*>(c->G_end.p);
            if (g_check)
                hipLaunchKernelGGL((k_gend<true, true>), dim3(ggrid), dim3(256), 0, s, d.G_off, d.G_tet, ng, P, ends,
                                   gend, check_seed, check_seed2, sums, 0, ni);
            else
                hipLaunchKernelGGL((k_gend<true, false>), dim3(ggrid), dim3(256), 0, s, d.G_off, d.G_tet, ng, P, ends,
                                   gend, 0ull, 0ull, nullptr, 0, ni);
            HIPCHK(c, hipGetLastError());
            if ((rc = ensure(c, c->G_pe, std::max<int64_t>(n_f, 1) * sizeof(uint2)))) return rc;
            hipLaunchKernelGGL(k_pack_pe, dim3((int)std::min<int64_t>(ceil_div(n_f, 256), 1 << 16)), dim3(256), 0, s,
                               static_cast<const uint32_t*>(c->G_pos.p), gend, n_f, static_cast<uint2*>(c->G_pe.p));
            HIPCHK(c, hipGetLastError());
            d.G_pe = static_cast<const uint2*>(c->G_pe.p);
        } else {
            release(c->G_end);
            release(c->G_pe);
            if (g_check) {
                hipLaunchKernelGGL((k_gend<false, true>), dim3(ggrid), dim3(256), 0, s, d.G_off, d.G_tet, ng, P,
                                   nullptr, nullptr, check_seed, check_seed2, sums, 0, ni);
                HIPCHK(c, hipGetLastError());
            }
        }
        // member codes for the WK 3 walks (all-vs-all with G_pos / G_end):
        // the run-end sort's histogram pass wrote them; else k_fcode
        d.Fcode = nullptr;
        if (d.G_pe && p.mode == PFAAI_MODE_ALL) {
            if (!ends_built) {
                if ((rc = ensure(c, c->Fcode, (size_t)(n_f + 16) * sizeof(uint32_t)))) return rc;
                hipLaunchKernelGGL(k_fcode, dim3((int)std::min<int64_t>(ceil_div(n_f + 16, 256), 1 << 16)), dim3(256), 0,
                                   s, d.Fg, n_f, static_cast<uint32_t*>(c->Fcode.p));
                HIPCHK(c, hipGetLastError());
            }
            d.Fcode = static_cast<const uint32_t*>(c->Fcode.p);
        } else {
            release(c->Fcode);
        }
        if (g_check && (rc = finish_g_check(c, s))) {
            if (rc == -1)
                return fail(c, PFAAI_RC_INVALID,
                            "G does not hold exactly the memberships of F (it must be F's genome-major transpose)");
            return rc;
        }
    }
    HIPCHK(c, hipEventRecord(c->load_ev[1], s));
    // the rows whose G_pos / G_end exist (the WK 3 walks; others take the run table)
    c->pos_lo = ends_built ? g_lo : 0;
    c->pos_hi = ends_built ? g_hi : ni;
    c->chk_lo = ends_built && g_check ? g_lo : 0;
    c->chk_hi = ends_built && g_check ? g_hi : ni;

    // work-list sizes (exact: one record per F entry of a row genome)
    c->row_fprefix.assign(c->n_rows + 1, 0);
    for (int64_t r = 0; r < c->n_rows; ++r) c->row_fprefix[r + 1] = c->row_fprefix[r] + fcount[c->row_genome_h[r]];
    HIPCHK(c, hipMemsetAsync(c->scalars.p, 0, SC_N * sizeof(unsigned long long), s));
    HIPCHK(c, hipStreamSynchronize(s));
    const auto t3 = clk::now();
    c->load_ms[0] = ms(t0, t1);
    c->load_ms[1] = ms_upload;
    {
        float dev_ms = 0.f;
        HIPCHK(c, hipEventElapsedTime(&dev_ms, c->load_ev[0], c->load_ev[1]));
        c->load_ms[2] = dev_ms;
    }
    (void)t3;
    release_sort_space(c);  // pfaai_run never allocates; the work-list path re-allocates below
    release_tsort(c);
    if (!has_g && (rc = ensure_worklists(c))) return rc;
    c->loaded = true;
    return PFAAI_RC_OK;
}

}  // namespace

extern "C" {

int pfaai_version(void) { return PFAAI_ABI_VERSION; }

int pfaai_create(pfaai_ctx** out, int device_id) {
    if (!out) return PFAAI_RC_INVALID;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return PFAAI_RC_HIP;
    if (device_id < 0 || device_id >= ndev) return PFAAI_RC_INVALID;
    auto* c = new pfaai_ctx();
    c->device = device_id;
    // the context stream at the highest priority: the load's side work (the
    // both-given check's hash sums on copy_stream) fills what the sort leaves
    int pri_least = 0, pri_greatest = 0;
    if (hipSetDevice(device_id) != hipSuccess ||
        hipDeviceGetStreamPriorityRange(&pri_least, &pri_greatest) != hipSuccess ||
        hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, pri_greatest) != hipSuccess) {
        delete c;
        return PFAAI_RC_HIP;
    }
    int rc = ensure(c, c->scalars, SC_N * sizeof(unsigned long long));
    if (rc) {
        release(c->scalars);
        (void)hipStreamDestroy(c->stream);
        delete c;
        return rc;
    }
    (void)hipMemset(c->scalars.p, 0, SC_N * sizeof(unsigned long long));
    // the second stream (the load's k_hash_f beside the sort, the streamed
    // outputs' copies) and the load's fork / join events: created here, since
    // a stream's first creation costs milliseconds (a load that created it
    // measured 13.6 ms of device span instead of 8.0 at 10k)
    if (hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking) != hipSuccess) c->copy_stream = nullptr;
    for (hipEvent_t& e : c->side_ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) e = nullptr;
    // the narrow rows' stream (launch_narrow; without it they run on the caller's stream)
    if (hipStreamCreateWithFlags(&c->side_stream, hipStreamNonBlocking) != hipSuccess) c->side_stream = nullptr;
    for (hipEvent_t& e : c->narrow_ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) e = nullptr;
    for (hipEvent_t& e : c->load_ev)
        if (hipEventCreate(&e) != hipSuccess) e = nullptr;
    // the code objects of this file and of the all-vs-all row kernels loaded
    // now rather than at the first launch of one of their kernels (HIP's
    // deferred loading), so no all-vs-all caller's first run pays it (the CLI
    // creates its context on a thread during the SQLite read).  The -q, -r
    // and full-row translation units (pfaai_rows_m{1,2,3}, 20 MB) load at
    // their first launch: preloading all four kept the C2 CLI waiting 129 ms
    // for its helper thread after the load (round 5)
    {
        hipFuncAttributes a;
        (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&k_blk_end<1024, 1>));
        preload_rows<0>();
    }
    if (hipHostMalloc(&c->stage_host, kStageBytes, hipHostMallocDefault) != hipSuccess) c->stage_host = nullptr;
    for (hipEvent_t& e : c->stage_ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) e = nullptr;
    // one slot-sized DMA copy each way now, on the creating thread: the first
    // host-to-device DMA of a process costs ~8 ms of setup (without this the
    // C2 CLI's load H2D went 8.6 -> 16.4 ms: its small uploads take the
    // runtime's path, round 5)
    void* warm = nullptr;
    if (c->stage_host && hipMalloc(&warm, kStageSlot) == hipSuccess) {
        if (hipMemcpyAsync(warm, c->stage_host, kStageSlot, hipMemcpyHostToDevice, c->stream) == hipSuccess)
            (void)hipMemcpyAsync(c->stage_host, warm, kStageSlot, hipMemcpyDeviceToHost, c->stream);
        (void)hipStreamSynchronize(c->stream);
        (void)hipFree(warm);
    }
    *out = c;
    return PFAAI_RC_OK;
}

int pfaai_destroy(pfaai_ctx* c) {
    if (!c) return PFAAI_RC_OK;
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();
    for (DevBuf* b : {&c->T16, &c->T16c, &c->Fp16, &c->Lp, &c->Fp, &c->Fg, &c->T, &c->is_q, &c->q_index, &c->t_rank, &c->row_of,
                      &c->row_genome, &c->tcol_row, &c->tcol_col, &c->G_off, &c->G_tet, &c->G_pos, &c->G_end, &c->G_pe, &c->Fcode, &c->blk, &c->rowptr, &c->lens, &c->cnt_t, &c->off_t, &c->key_c, &c->rec_c, &c->key_a,
                      &c->key_b, &c->val_a, &c->val_b, &c->hist, &c->hoff, &c->recs, &c->sums, &c->scalars,
                      &c->out_aji, &c->out_S, &c->out_N, &c->dbg, &c->blkw, &c->srec_a, &c->srec_b, &c->shist,
                      &c->sgsum, &c->sbase, &c->tails, &c->ranks})
        release(*b);
    for (hipEvent_t e : c->pool) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->load_ev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->side_ev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->narrow_ev)
        if (e) (void)hipEventDestroy(e);
    release(c->st_dev);
    if (c->st_host) (void)hipHostFree(c->st_host);
    if (c->stage_host) (void)hipHostFree(c->stage_host);
    for (hipEvent_t e : c->stage_ev)
        if (e) (void)hipEventDestroy(e);
    for (int i = 0; i < 2; ++i) {
        if (c->st_done[i]) (void)hipEventDestroy(c->st_done[i]);
        if (c->st_copied[i]) (void)hipEventDestroy(c->st_copied[i]);
    }
    if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
    if (c->side_stream) (void)hipStreamDestroy(c->side_stream);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return PFAAI_RC_OK;
}

const char* pfaai_last_error(const pfaai_ctx* c) { return c ? c->err.c_str() : "null context"; }

int pfaai_load(pfaai_ctx* c, const pfaai_problem* pb) {
    if (!c || !pb) return PFAAI_RC_INVALID;
    return guarded(c, [&] { return load_impl(c, pb); });
}

int pfaai_load_rows(pfaai_ctx* c, const pfaai_problem* pb, int64_t row_begin, int64_t row_end) {
    if (!c || !pb) return PFAAI_RC_INVALID;
    if (row_begin < 0 || row_end < row_begin || row_end > pb->n_ids) return fail(c, PFAAI_RC_INVALID, "bad row range");
    return guarded(c, [&] { return load_impl(c, pb, row_begin, row_end); });
}

int pfaai_shape(const pfaai_ctx* c, int64_t* n_rows, int64_t* n_pairs) {
    if (!c || !c->loaded) return PFAAI_RC_INVALID;
    if (n_rows) *n_rows = c->n_rows;
    if (n_pairs) *n_pairs = c->n_pairs;
    return PFAAI_RC_OK;
}

int pfaai_row_span(const pfaai_ctx* c, int64_t rb, int64_t re, int64_t* first, int64_t* count) {
    if (!c || !c->loaded || rb < 0 || re > c->n_rows || rb > re || c->order_n) return PFAAI_RC_INVALID;
    const auto& p = c->prob;
    int64_t f = 0, l = 0;  // [f, l)
    if (rb == re) {
        f = l = 0;
    } else if (p.mode == PFAAI_MODE_ALL) {
        const int64_t n = p.n_ids;
        auto base = [n](int64_t a) { return n * a - a * (a + 1) / 2; };  // JAC index of (a, a+1)
        f = base(rb);
        l = base(re);
    } else if (p.mode == PFAAI_MODE_QT) {
        f = rb * p.n_tgt;
        l = re * p.n_tgt;
    } else {
        f = rb * (int64_t)p.n_tgt;
        l = c->n_pairs;  // triangle rows follow all cross rows: hull to the end
        if (re == c->n_rows && rb == 0) f = 0;
    }
    if (first) *first = f;
    if (count) *count = l - f;
    return PFAAI_RC_OK;
}

int pfaai_run(pfaai_ctx* c, int64_t rb, int64_t re, uint32_t flags, double* aji, double* S, int32_t* N,
              void* stream) {
    if (!c) return PFAAI_RC_INVALID;
    if (!c->loaded) return fail(c, PFAAI_RC_INVALID, "no problem loaded");
    if (rb < 0 || re > c->n_rows || rb > re) return fail(c, PFAAI_RC_INVALID, "row range out of bounds");
    if ((flags & PFAAI_FLAG_EMIT_JAC) && (!S || !N)) return fail(c, PFAAI_RC_INVALID, "EMIT_JAC needs S and N");
    if (!aji && !S && !N) return fail(c, PFAAI_RC_INVALID, "no output");
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->stream;
    // row kernel: default by input, PFAAI_ROWS_KERNEL overrides (A/B runs)
    {
        int k = !c->has_g ? RK_WORKLIST : c->max_glen > kPlEntries ? RK_FUSED : RK_PL;
        if (const char* v = DIAG_ENV("PFAAI_ROWS_KERNEL")) {
            const std::string x(v);
            if (x == "pl") k = RK_PL;
            else if (x == "pl512") k = RK_PL512;
            else if (x == "fused") k = RK_FUSED;
            else if (x == "worklist") k = RK_WORKLIST;
            else return fail(c, PFAAI_RC_INVALID, "PFAAI_ROWS_KERNEL must be pl, pl512, fused or worklist");
        }
        if (!c->has_g && k != RK_WORKLIST) k = RK_WORKLIST;       // the others walk the G lists
        if (c->max_glen > kPlEntries && k != RK_WORKLIST) k = RK_FUSED;  // lists too long
        // k_rows_pl addresses the run table with 32-bit buffer offsets
        if ((uint64_t)c->prob.n_prot * PFAAI_NTETRAMERS * 16u >= (1ull << 32) && (k == RK_PL || k == RK_PL512))
            k = RK_FUSED;
        c->rows_kernel = k;
    }
    {  // consecutive rows per XCD (L2 sharing of a clade's runs); PFAAI_XCD_CHUNK for A/B
        const char* xc = DIAG_ENV("PFAAI_XCD_CHUNK");
        c->dev.xcd_chunk = xc ? std::max(1, atoi(xc)) : kXcdChunk;
    }
    if (const char* abl = DIAG_ENV("PFAAI_ABLATE")) flags |= (uint32_t)atoi(abl) << 8;  // diagnostics only
    {  // k_rows_pl's S5 entry order (flags bits 18-20; pfaai_rows_pl.hpp): default 2, PFAAI_PL_STAG overrides (A/B)
        const char* sg = DIAG_ENV("PFAAI_PL_STAG");
        flags = (flags & ~(7u << 18)) | (uint32_t)((sg ? atoi(sg) : kPlStag) & 7) << 18;
    }
    {  // k_rows_pl's further member rounds from the last lane pair (flags bit 21): default kPlRev, PFAAI_PL_REV overrides (A/B)
        const char* rv = DIAG_ENV("PFAAI_PL_REV");
        flags = (flags & ~(1u << 21)) | (uint32_t)((rv ? atoi(rv) : kPlRev) & 1) << 21;
    }
    // k_rows_pl wave priorities: bit 0 raises the load-issue stages above other
    // waves' fp64 normalisation, bit 1 the scatter rounds (3: 11.52 -> 11.33
    // ms at 10k, tools/gpu/ab_rows.py); PFAAI_PL_PRIO=0..3 overrides (A/B)
    {
        const char* pr = DIAG_ENV("PFAAI_PL_PRIO");
        flags = (flags & ~(3u << 16)) | (uint32_t)((pr ? atoi(pr) : kPlPrio) & 3) << 16;
    }
    if (c->pool_used >= 3 * 4096) {  // nobody reads the window: recycle it
        HIPCHK(c, hipStreamSynchronize(s));
        c->pool_used = 0;
    }
    c->timed = true;
    // full rows (pfaai_stream_matrix): every column of the loaded mode's
    // target set; QT rows already are full rows
    const bool full = (flags & PFAAI_FLAG_FULL_ROWS) && c->prob.mode != PFAAI_MODE_QT;
    c->cols_run = full ? c->prob.n_ids : c->max_cols;
    // all-vs-all row a has n - 1 - a columns, so a launch is as wide as its
    // first row: row blocks past the first (a multi-GPU rank's shard, a
    // stream tile) get the counter words per thread (KW) and column chunks
    // their own rows need -- fewer T loads and S5 words per protein (the last
    // 10k/8 shard: 1.36 -> 1.22 ms at KW 1).  Only with G_pos (<= 20 480
    // genomes), whose run walks start at the row genome: without it a narrow
    // launch would leave the column windows for whole-run walks pruned by
    // three splitters (100k streamed: 613 -> 689 ms).  PFAAI_PL_LAUNCH_COLS=0
    // keeps the problem's widest row (A/B; results identical)
    if (!full && c->prob.mode == PFAAI_MODE_ALL && c->dev.G_pe) {
        const char* lc = DIAG_ENV("PFAAI_PL_LAUNCH_COLS");
        if (!(lc && lc[0] == '0') && rb < re)  // (rows ascend by genome: the first is the widest)
            c->cols_run = (int32_t)std::max<int64_t>(1, c->prob.n_ids - 1 - c->row_genome_h[rb]);
    }
    if (rb == re) return PFAAI_RC_OK;
    if (full) return run_mode<kModeFull>(c, rb, re, flags, aji, S, N, s);
    switch (c->prob.mode) {
        case 0: return run_mode<0>(c, rb, re, flags, aji, S, N, s);
        case 1: return run_mode<1>(c, rb, re, flags, aji, S, N, s);
        default: return run_mode<2>(c, rb, re, flags, aji, S, N, s);
    }
}

int pfaai_compute(pfaai_ctx* c, uint32_t flags, double* h_aji, double* h_S, int32_t* h_N) {
    if (!c) return PFAAI_RC_INVALID;
    if (!c->loaded) return fail(c, PFAAI_RC_INVALID, "no problem loaded");
    if (c->order_n) return fail(c, PFAAI_RC_INVALID, "a row order is set (pfaai_set_row_order): only pfaai_run");
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t np = c->n_pairs;
    int rc;
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    // (trace) the job's CPU-quota throttling over this call: cgroup v2 cpu.stat
    auto throttled_us = []() -> long long {
        FILE* f = std::fopen("/sys/fs/cgroup/cpu.stat", "r");
        if (!f) return -1;
        char key[64];
        long long v = 0, r = -1;
        while (std::fscanf(f, "%63s %lld", key, &v) == 2)
            if (std::strcmp(key, "throttled_usec") == 0) r = v;
        std::fclose(f);
        return r;
    };
    const bool trace0 = DIAG_ENV("PFAAI_TRACE_COMPUTE") != nullptr;
    const long long thr0 = trace0 ? throttled_us() : 0;
    if ((rc = ensure(c, c->out_aji, np * sizeof(double)))) return rc;
    if ((rc = ensure(c, c->out_S, np * sizeof(double)))) return rc;
    if ((rc = ensure(c, c->out_N, np * sizeof(int32_t)))) return rc;
    auto* aji = static_cast<double*>(c->out_aji.p);
    auto* S = static_cast<double*>(c->out_S.p);
    auto* N = static_cast<int32_t*>(c->out_N.p);
    HIPCHK(c, hipMemsetAsync(aji, 0, np * sizeof(double), c->stream));
    HIPCHK(c, hipMemsetAsync(S, 0, np * sizeof(double), c->stream));
    HIPCHK(c, hipMemsetAsync(N, 0, np * sizeof(int32_t), c->stream));
    const auto t1 = clk::now();
    rc = pfaai_run(c, 0, c->n_rows, flags | PFAAI_FLAG_EMIT_JAC, aji, S, N, c->stream);
    if (rc) return rc;
    const auto t2 = clk::now();
    const bool trace = DIAG_ENV("PFAAI_TRACE_COMPUTE") != nullptr;
    if (trace) HIPCHK(c, hipStreamSynchronize(c->stream));
    double probe_ms = 0.0;
    if (trace && c->stage_host) {  // one 4-KB copy alone: is the first D2H after the run slow whatever its size?
        const auto tp = clk::now();
        HIPCHK(c, hipMemcpyAsync(c->stage_host, aji, 4096, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        probe_ms = std::chrono::duration<double, std::milli>(clk::now() - tp).count();
    }
    const auto t3 = clk::now();
    if (h_aji && (rc = staged_copy(c, h_aji, aji, np * sizeof(double), false, c->stream))) return rc;
    const auto t4 = clk::now();
    if (h_S && (rc = staged_copy(c, h_S, S, np * sizeof(double), false, c->stream))) return rc;
    if (h_N && (rc = staged_copy(c, h_N, N, np * sizeof(int32_t), false, c->stream))) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const auto t5 = clk::now();
    if (trace) {
        auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        const long long thr1 = throttled_us();
        std::fprintf(stderr, "[pfaai_compute] alloc+memset %.2f, run submit %.2f, run wait %.2f (4-KB D2H probe %.2f), "
                     "D2H aji %.2f, S+N %.2f ms; cgroup CPU throttling during the call %.2f ms\n", ms(t0, t1), ms(t1, t2),
                     ms(t2, t3) - probe_ms, probe_ms, ms(t3, t4), ms(t4, t5),
                     thr0 >= 0 && thr1 >= 0 ? (thr1 - thr0) / 1e3 : -1.0);
    }
    return PFAAI_RC_OK;
}

int pfaai_load_info(const pfaai_ctx* c, int32_t* path) {
    if (!c || !c->loaded) return PFAAI_RC_INVALID;
    if (path) *path = c->load_path;
    return PFAAI_RC_OK;
}

int pfaai_load_timing(const pfaai_ctx* c, double* ms_checks, double* ms_upload, double* ms_device) {
    if (!c || !c->loaded) return PFAAI_RC_INVALID;
    if (ms_checks) *ms_checks = c->load_ms[0];
    if (ms_upload) *ms_upload = c->load_ms[1];
    if (ms_device) *ms_device = c->load_ms[2];
    return PFAAI_RC_OK;
}

int pfaai_run_info(const pfaai_ctx* c, int32_t* rows_kernel, int32_t* column_windows) {
    if (!c) return PFAAI_RC_INVALID;
    if (rows_kernel) *rows_kernel = c->rows_kernel;
    if (column_windows) *column_windows = c->windows ? 1 : 0;
    return PFAAI_RC_OK;
}

int pfaai_set_row_order(pfaai_ctx* c, const int32_t* genomes, int64_t n) {
    if (!c) return PFAAI_RC_INVALID;
    if (!c->loaded) return fail(c, PFAAI_RC_INVALID, "no problem loaded");
    if (c->prob.mode != PFAAI_MODE_ALL) return fail(c, PFAAI_RC_INVALID, "pfaai_set_row_order: all-vs-all only");
    if (!c->has_g) return fail(c, PFAAI_RC_INVALID, "pfaai_set_row_order: needs a genome-major load");
    const int32_t ni = c->prob.n_ids;
    if (n < 0 || n > ni || (n > 0 && !genomes)) return fail(c, PFAAI_RC_INVALID, "pfaai_set_row_order: bad list");
    std::vector<int32_t> order;
    order.reserve((size_t)ni);
    bool in_pos = true;
    for (int64_t i = 0; i < n; ++i) {
        const int32_t g = genomes[i];
        if (g < 0 || g >= ni || (i && g <= genomes[i - 1]))
            return fail(c, PFAAI_RC_INVALID, "pfaai_set_row_order: genome ids must ascend strictly within [0, n_ids)");
        if (g < c->chk_lo || g >= c->chk_hi)
            return fail(c, PFAAI_RC_INVALID, "pfaai_set_row_order: a genome outside the block pfaai_load_rows verified");
        in_pos = in_pos && g >= c->pos_lo && g < c->pos_hi;
        order.push_back(g);
    }
    {  // the other genomes follow in id order (rows past n are refused while the list is set)
        std::vector<char> listed((size_t)ni, 0);
        for (int32_t g : order) listed[(size_t)g] = 1;
        for (int32_t g = 0; g < ni; ++g)
            if (!listed[(size_t)g]) order.push_back(g);
    }
    std::vector<int32_t> row_of((size_t)ni);
    for (int32_t r = 0; r < ni; ++r) row_of[(size_t)order[(size_t)r]] = r;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipDeviceSynchronize());  // no launch in flight still reads the old order
    HIPCHK(c, hipMemcpy(c->row_genome.p, order.data(), (size_t)ni * sizeof(int32_t), hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->row_of.p, row_of.data(), (size_t)ni * sizeof(int32_t), hipMemcpyHostToDevice));
    {  // the work-list sizes follow the rows (pfaai_debug_row_counts' sorted path)
        std::vector<int64_t> fcount((size_t)ni, 0);
        for (int64_t r = 0; r < c->n_rows; ++r)
            fcount[(size_t)c->row_genome_h[(size_t)r]] = c->row_fprefix[r + 1] - c->row_fprefix[r];
        for (int64_t r = 0; r < c->n_rows; ++r) c->row_fprefix[r + 1] = c->row_fprefix[r] + fcount[(size_t)order[(size_t)r]];
    }
    c->row_genome_h.swap(order);
    c->order_n = n;
    c->order_in_pos = in_pos;
    return PFAAI_RC_OK;
}

int pfaai_run_walk(const pfaai_ctx* c, int32_t* walk, int32_t* narrow_launch) {
    if (!c) return PFAAI_RC_INVALID;
    if (walk) *walk = c->last_walk;
    if (narrow_launch) *narrow_launch = c->last_narrow ? 1 : 0;
    return PFAAI_RC_OK;
}

int pfaai_last_stats(pfaai_ctx* c, int64_t* n_events, float* ms_build, float* ms_rows) {
    if (!c) return PFAAI_RC_INVALID;
    HIPCHK(c, hipSetDevice(c->device));
    unsigned long long ev = 0;
    HIPCHK(c, hipMemcpy(&ev, static_cast<unsigned long long*>(c->scalars.p) + SC_EVENTS, sizeof(ev),
                        hipMemcpyDeviceToHost));
    if (n_events) *n_events = (int64_t)ev;
    if (c->timed) {
        HIPCHK(c, hipEventSynchronize(c->ev2));
        float a = 0.f, b = 0.f;
        HIPCHK(c, hipEventElapsedTime(&a, c->ev0, c->ev1));
        HIPCHK(c, hipEventElapsedTime(&b, c->ev1, c->ev2));
        if (ms_build) *ms_build = a;
        if (ms_rows) *ms_rows = b;
    }
    return PFAAI_RC_OK;
}

int pfaai_timing(pfaai_ctx* c, int reset, int32_t* n_runs, double* ms_build, double* ms_rows) {
    if (!c) return PFAAI_RC_INVALID;
    HIPCHK(c, hipSetDevice(c->device));
    double b = 0.0, r = 0.0;
    const size_t n = c->pool_used / 3;
    for (size_t i = 0; i < n; ++i) {
        hipEvent_t* ev = &c->pool[3 * i];
        HIPCHK(c, hipEventSynchronize(ev[2]));
        float x = 0.f, y = 0.f;
        HIPCHK(c, hipEventElapsedTime(&x, ev[0], ev[1]));
        HIPCHK(c, hipEventElapsedTime(&y, ev[1], ev[2]));
        b += x;
        r += y;
    }
    if (n_runs) *n_runs = (int32_t)n;
    if (ms_build) *ms_build = b;
    if (ms_rows) *ms_rows = r;
    if (reset) {
        c->pool_used = 0;
        c->timed = false;
    }
    return PFAAI_RC_OK;
}

int pfaai_debug_row_counts(pfaai_ctx* c, int64_t row, int32_t* h_counts) {
    if (!c || !h_counts) return PFAAI_RC_INVALID;
    if (!c->loaded) return fail(c, PFAAI_RC_INVALID, "no problem loaded");
    if (row < 0 || row >= c->n_rows) return fail(c, PFAAI_RC_INVALID, "row out of range");
    HIPCHK(c, hipSetDevice(c->device));
    const auto& p = c->prob;
    const int64_t cells = (int64_t)p.n_prot * p.n_ids;
    int rc;
    if ((rc = ensure(c, c->dbg, cells * sizeof(int32_t)))) return rc;
    if ((rc = ensure_worklists(c))) return rc;
    HIPCHK(c, hipMemsetAsync(c->dbg.p, 0, cells * sizeof(int32_t), c->stream));
    const int32_t chunk = 2 * 10 * kRowThreads;
    const int32_t nchunks = (int32_t)ceil_div(std::max<int32_t>(c->max_cols, 1), chunk);
    const size_t lds = 10 * kRowThreads * sizeof(uint32_t);
    auto* rowptr = static_cast<const unsigned long long*>(c->rowptr.p);
    auto* recs = static_cast<const uint2*>(c->recs.p);
    auto* out = static_cast<int32_t*>(c->dbg.p);
    switch (p.mode) {
        case 0:
            if ((rc = build_records<0>(c, row, row + 1, c->stream, false)))
                return rc;
            hipLaunchKernelGGL(k_row_counts<0>, dim3(1, nchunks), dim3(kRowThreads), lds, c->stream, c->dev, row, rowptr, recs, chunk, out);
            break;
        case 1:
            if ((rc = build_records<1>(c, row, row + 1, c->stream, false)))
                return rc;
            hipLaunchKernelGGL(k_row_counts<1>, dim3(1, nchunks), dim3(kRowThreads), lds, c->stream, c->dev, row, rowptr, recs, chunk, out);
            break;
        default:
            if ((rc = build_records<2>(c, row, row + 1, c->stream, false)))
                return rc;
            hipLaunchKernelGGL(k_row_counts<2>, dim3(1, nchunks), dim3(kRowThreads), lds, c->stream, c->dev, row, rowptr, recs, chunk, out);
            break;
    }
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(h_counts, out, cells * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return PFAAI_RC_OK;
}

}  // extern "C"

namespace {
template <int NS>
__global__ void k_div_check(int32_t c_max, int32_t d_max, unsigned long long* bad) {
    const int32_t c = 1 + (int32_t)blockIdx.y;  // c <= c_max by the grid
    unsigned long long nb = 0;
    for (int64_t d = c + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; d <= d_max; d += (int64_t)gridDim.x * blockDim.x) {
        const double q0 = (double)c / (double)d;
        const double q1 = exact_div_small<NS>((double)c, (double)d);
        nb += __double_as_longlong(q0) != __double_as_longlong(q1);
        // k_rows_pl's paired form (exact_div_pair: one reciprocal of d * d1
        // for both columns of a counter word) against partners d1 across
        // the range, both columns checked
        const int32_t d1s[6] = {1, (int32_t)d, (int32_t)d + 1, 2 * (int32_t)d - 1,
                                (int32_t)((d * 7919) % 131071) + 1, 131071};
#pragma unroll
        for (int u = 0; u < 6; ++u) {
            const int32_t d1 = d1s[u], c1 = (int32_t)min<int64_t>(c, d1);
            double s0 = 0.0, s1 = 0.0;
            exact_div_pair(c, (int32_t)d, c1, d1, s0, s1);
            nb += (__double_as_longlong(s0) != __double_as_longlong(q0)) +
                  (__double_as_longlong(s1) != __double_as_longlong((double)c1 / (double)d1));
        }
    }
    if (nb) atomicAdd(bad, nb);
    (void)c_max;
}
}  // namespace

extern "C" {

int pfaai_debug_div_check(pfaai_ctx* c, int32_t c_max, int32_t d_max, int64_t* mismatches) {
    if (!c || !mismatches || c_max < 1 || d_max < c_max || d_max >= (1 << 24) || c_max > 65535)
        return PFAAI_RC_INVALID;
    HIPCHK(c, hipSetDevice(c->device));
    int rc = ensure(c, c->dbg, sizeof(unsigned long long));
    if (rc) return rc;
    auto* bad = static_cast<unsigned long long*>(c->dbg.p);
    HIPCHK(c, hipMemsetAsync(bad, 0, sizeof(unsigned long long), c->stream));
    const char* ns = DIAG_ENV("PFAAI_DIV_NEWTON");  // diagnostics: check a shorter refinement
    if (ns && atoi(ns) == 0)
        hipLaunchKernelGGL(k_div_check<0>, dim3(64, c_max), dim3(256), 0, c->stream, c_max, d_max, bad);
    else if (ns && atoi(ns) == 2)
        hipLaunchKernelGGL(k_div_check<2>, dim3(64, c_max), dim3(256), 0, c->stream, c_max, d_max, bad);
    else  // the kernels' form
        hipLaunchKernelGGL(k_div_check<1>, dim3(64, c_max), dim3(256), 0, c->stream, c_max, d_max, bad);
    HIPCHK(c, hipGetLastError());
    unsigned long long h = 0;
    HIPCHK(c, hipMemcpyAsync(&h, bad, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    *mismatches = (int64_t)h;
    return PFAAI_RC_OK;
}

int pfaai_debug_clocks(pfaai_ctx* c, uint64_t* out, int64_t n) {
    if (!c || n < 0 || (n > 0 && !out)) return PFAAI_RC_INVALID;
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t cap = (int64_t)kClkBlocks * 16 * 8;
    if (n == 0) {  // arm: allocate and clear the clock buffer
        int rc = ensure(c, c->dbg, cap * sizeof(uint64_t));
        if (rc) return rc;
        HIPCHK(c, hipMemset(c->dbg.p, 0, cap * sizeof(uint64_t)));
        return PFAAI_RC_OK;
    }
    if (c->dbg.bytes < (size_t)cap * sizeof(uint64_t)) return fail(c, PFAAI_RC_INVALID, "clocks not armed");
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(out, c->dbg.p, std::min(n, cap) * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return PFAAI_RC_OK;
}

int pfaai_device_alloc(pfaai_ctx* c, void** ptr, int64_t bytes) {
    if (!c || !ptr || bytes < 0) return PFAAI_RC_INVALID;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMalloc(ptr, bytes > 0 ? bytes : 8));
    return PFAAI_RC_OK;
}

int pfaai_device_free(pfaai_ctx* c, void* ptr) {
    if (!c) return PFAAI_RC_INVALID;
    HIPCHK(c, hipSetDevice(c->device));
    if (ptr) HIPCHK(c, hipFree(ptr));
    return PFAAI_RC_OK;
}

int pfaai_memcpy_d2h(pfaai_ctx* c, void* dst, const void* src, int64_t bytes) {
    if (!c || bytes < 0) return PFAAI_RC_INVALID;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return PFAAI_RC_OK;
}

int pfaai_synchronize(pfaai_ctx* c) {
    if (!c) return PFAAI_RC_INVALID;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipDeviceSynchronize());
    return PFAAI_RC_OK;
}


// Output-tile streaming (config C5, a matrix too large to
// hold whole on the host or the device).  Rows are cut into tiles of at most
// tile_pairs JAC entries; tile k is computed into device buffer k & 1 on the
// context stream while tile k - 1 is copied to pinned host buffer (k-1) & 1
// on the copy stream and tile k - 2 is handed to the sink on this thread.
// The run table is built by the first tile only (PFAAI_FLAG_KEEP_RUNS).
static int stream_impl(pfaai_ctx* c, int64_t rb, int64_t re, int64_t tile_pairs, uint32_t flags, pfaai_sink_fn sink,
                       void* user) {
    if (!c) return PFAAI_RC_INVALID;
    if (!c->loaded) return fail(c, PFAAI_RC_INVALID, "no problem loaded");
    if (!sink) return fail(c, PFAAI_RC_INVALID, "sink is required");
    if (rb < 0 || re > c->n_rows || rb > re) return fail(c, PFAAI_RC_INVALID, "row range out of bounds");
    if (c->prob.mode == PFAAI_MODE_QSUB)
        return fail(c, PFAAI_RC_INVALID, "pfaai_stream: QSUB rows have no contiguous JAC span (use pfaai_run)");
    HIPCHK(c, hipSetDevice(c->device));
    const bool jac = flags & PFAAI_FLAG_EMIT_JAC;
    c->st_events = 0;
    if (rb == re) return PFAAI_RC_OK;
    // row tiles: maximal row ranges whose span fits tile_pairs (>= one row)
    std::vector<int64_t> cut{rb};
    int64_t cap = 1;
    for (int64_t r = rb; r < re;) {
        int64_t f0, n0, r2 = r + 1;
        pfaai_row_span(c, r, r2, &f0, &n0);
        while (r2 < re) {
            int64_t f1, n1;
            pfaai_row_span(c, r, r2 + 1, &f1, &n1);
            if (n1 > tile_pairs) break;
            n0 = n1;
            ++r2;
        }
        cap = std::max(cap, n0);
        cut.push_back(r2);
        r = r2;
    }
    const int64_t ntiles = (int64_t)cut.size() - 1;
    const size_t per = (size_t)cap * (sizeof(double) + (jac ? sizeof(double) + sizeof(int32_t) : 0));
    int rc;
    if ((rc = ensure(c, c->st_dev, 2 * per))) return rc;
    const size_t host_bytes = 2 * per + (size_t)ntiles * sizeof(unsigned long long);
    if (c->st_host_bytes < host_bytes) {
        if (c->st_host) (void)hipHostFree(c->st_host);
        c->st_host = nullptr;
        c->st_host_bytes = 0;
        HIPCHK(c, hipHostMalloc(&c->st_host, host_bytes, hipHostMallocDefault));
        c->st_host_bytes = host_bytes;
    }
    if (!c->copy_stream) HIPCHK(c, hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
    for (int i = 0; i < 2; ++i) {
        if (!c->st_done[i]) HIPCHK(c, hipEventCreateWithFlags(&c->st_done[i], hipEventDisableTiming));
        if (!c->st_copied[i]) HIPCHK(c, hipEventCreateWithFlags(&c->st_copied[i], hipEventDisableTiming));
    }
    auto dptr = [&](int b, int which) -> char* {  // 0 aji, 1 S, 2 N of device buffer b
        char* base = static_cast<char*>(c->st_dev.p) + b * per;
        return base + (which == 0 ? 0 : which == 1 ? cap * sizeof(double) : 2 * cap * sizeof(double));
    };
    auto hptr = [&](int b, int which) -> char* {
        char* base = static_cast<char*>(c->st_host) + b * per;
        return base + (which == 0 ? 0 : which == 1 ? cap * sizeof(double) : 2 * cap * sizeof(double));
    };
    auto* evs = reinterpret_cast<unsigned long long*>(static_cast<char*>(c->st_host) + 2 * per);
    const auto* sc_ev = static_cast<unsigned long long*>(c->scalars.p) + SC_EVENTS;
    auto drain = [&]() {  // error exit: nothing may still write the buffers
        (void)hipStreamSynchronize(c->stream);
        (void)hipStreamSynchronize(c->copy_stream);
    };
    auto deliver = [&](int64_t k) -> int {
        const int b = (int)(k & 1);
        HIPCHK(c, hipEventSynchronize(c->st_copied[b]));
        int64_t f, n;
        pfaai_row_span(c, cut[k], cut[k + 1], &f, &n);
        c->st_events += (int64_t)evs[k];
        const int src = sink(user, cut[k], cut[k + 1], f, n, reinterpret_cast<const double*>(hptr(b, 0)),
                             jac ? reinterpret_cast<const double*>(hptr(b, 1)) : nullptr,
                             jac ? reinterpret_cast<const int32_t*>(hptr(b, 2)) : nullptr);
        return src ? fail(c, src, "pfaai_stream: the sink stopped the stream") : PFAAI_RC_OK;
    };
    for (int64_t k = 0; k < ntiles; ++k) {
        const int b = (int)(k & 1);
        int64_t f, n;
        pfaai_row_span(c, cut[k], cut[k + 1], &f, &n);
        if (k >= 2) {  // host buffer b is reused below: hand tile k - 2 over first
            if ((rc = deliver(k - 2))) { drain(); return rc; }
        }
        // device buffer b was last read by the copy of tile k - 2
        if (k >= 2) HIPCHK(c, hipStreamWaitEvent(c->stream, c->st_copied[b], 0));
        auto* aji = reinterpret_cast<double*>(dptr(b, 0)) - f;  // kernels index by the global JAC index
        auto* S = jac ? reinterpret_cast<double*>(dptr(b, 1)) - f : nullptr;
        auto* N = jac ? reinterpret_cast<int32_t*>(dptr(b, 2)) - f : nullptr;
        rc = pfaai_run(c, cut[k], cut[k + 1], flags | (k ? PFAAI_FLAG_KEEP_RUNS : 0u), aji, S, N, c->stream);
        if (rc) { drain(); return rc; }
        HIPCHK(c, hipMemcpyAsync(&evs[k], sc_ev, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipEventRecord(c->st_done[b], c->stream));
        HIPCHK(c, hipStreamWaitEvent(c->copy_stream, c->st_done[b], 0));
        HIPCHK(c, hipMemcpyAsync(hptr(b, 0), dptr(b, 0), n * sizeof(double), hipMemcpyDeviceToHost, c->copy_stream));
        if (jac) {
            HIPCHK(c, hipMemcpyAsync(hptr(b, 1), dptr(b, 1), n * sizeof(double), hipMemcpyDeviceToHost, c->copy_stream));
            HIPCHK(c, hipMemcpyAsync(hptr(b, 2), dptr(b, 2), n * sizeof(int32_t), hipMemcpyDeviceToHost, c->copy_stream));
        }
        HIPCHK(c, hipEventRecord(c->st_copied[b], c->copy_stream));
    }
    for (int64_t k = std::max<int64_t>(0, ntiles - 2); k < ntiles; ++k)
        if ((rc = deliver(k))) { drain(); return rc; }
    return PFAAI_RC_OK;
}

// Dense output rows (pfaai_stream_matrix): row tiles of printOutput's
// matrix, each computed whole with PFAAI_FLAG_FULL_ROWS (no tile depends on
// another), double-buffered like stream_impl: tile k computes into device
// buffer k & 1 while tile k - 1 is copied to pinned buffer (k - 1) & 1 and
// tile k - 2 is handed to the sink.  The run table is built by tile 0 only.
static int stream_matrix_impl(pfaai_ctx* c, int64_t rb, int64_t re, int64_t tile_rows, uint32_t flags,
                              pfaai_matrix_sink_fn sink, void* user) {
    if (!c->loaded) return fail(c, PFAAI_RC_INVALID, "no problem loaded");
    if (!sink) return fail(c, PFAAI_RC_INVALID, "sink is required");
    if (rb < 0 || re > c->n_rows || rb > re) return fail(c, PFAAI_RC_INVALID, "row range out of bounds");
    if (flags & PFAAI_FLAG_EMIT_JAC) return fail(c, PFAAI_RC_INVALID, "pfaai_stream_matrix writes AJI only");
    HIPCHK(c, hipSetDevice(c->device));
    c->st_events = 0;
    if (rb == re) return PFAAI_RC_OK;
    const bool qt = c->prob.mode == PFAAI_MODE_QT;
    const int64_t n_cols = qt ? c->prob.n_tgt : c->prob.n_ids;
    // QT under REF_COMPAT: the reference prints pair (q, t) at column
    // mapTargetId(nQ + t) (its JAC ids, ds_impl.hpp:434-436 + main.cpp:149), i.e.
    // each row rotated right by nQ; with nQ > nT its rows collide instead.
    const bool rot = qt && (flags & PFAAI_FLAG_REF_COMPAT);
    if (rot && c->prob.n_qry > c->prob.n_tgt)
        return fail(c, PFAAI_RC_INVALID,
                    "pfaai_stream_matrix: the reference's QT ids overlap rows when nQ > nT; run without "
                    "PFAAI_FLAG_REF_COMPAT (CLI: --corrected)");
    const int64_t shift = rot ? c->prob.n_qry % n_cols : 0;
    tile_rows = std::max<int64_t>(1, std::min<int64_t>(tile_rows, re - rb));
    const int64_t ntiles = ceil_div(re - rb, tile_rows);
    const size_t per = (size_t)tile_rows * n_cols * sizeof(double);
    int rc;
    if ((rc = ensure(c, c->st_dev, 2 * per))) return rc;
    const size_t host_bytes = 2 * per + (size_t)ntiles * sizeof(unsigned long long);
    if (c->st_host_bytes < host_bytes) {
        if (c->st_host) (void)hipHostFree(c->st_host);
        c->st_host = nullptr;
        c->st_host_bytes = 0;
        HIPCHK(c, hipHostMalloc(&c->st_host, host_bytes, hipHostMallocDefault));
        c->st_host_bytes = host_bytes;
    }
    if (!c->copy_stream) HIPCHK(c, hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
    for (int i = 0; i < 2; ++i) {
        if (!c->st_done[i]) HIPCHK(c, hipEventCreateWithFlags(&c->st_done[i], hipEventDisableTiming));
        if (!c->st_copied[i]) HIPCHK(c, hipEventCreateWithFlags(&c->st_copied[i], hipEventDisableTiming));
    }
    auto dptr = [&](int b) { return reinterpret_cast<double*>(static_cast<char*>(c->st_dev.p) + b * per); };
    auto hptr = [&](int b) { return reinterpret_cast<double*>(static_cast<char*>(c->st_host) + b * per); };
    auto* evs = reinterpret_cast<unsigned long long*>(static_cast<char*>(c->st_host) + 2 * per);
    const auto* sc_ev = static_cast<unsigned long long*>(c->scalars.p) + SC_EVENTS;
    auto tile = [&](int64_t k, int64_t& r0, int64_t& r1) {
        r0 = rb + k * tile_rows;
        r1 = std::min(re, r0 + tile_rows);
    };
    auto drain = [&]() {
        (void)hipStreamSynchronize(c->stream);
        (void)hipStreamSynchronize(c->copy_stream);
    };
    auto deliver = [&](int64_t k) -> int {
        const int b = (int)(k & 1);
        HIPCHK(c, hipEventSynchronize(c->st_copied[b]));
        int64_t r0, r1;
        tile(k, r0, r1);
        c->st_events += (int64_t)evs[k];
        if (shift) {
            double* h = hptr(b);
            par_for(r1 - r0, [&](int64_t lo, int64_t hi, int) {
                for (int64_t r = lo; r < hi; ++r)
                    std::rotate(h + r * n_cols, h + r * n_cols + (n_cols - shift), h + (r + 1) * n_cols);
            }, (r1 - r0) * n_cols);
        }
        const int src = sink(user, r0, r1, n_cols, hptr(b));
        return src ? fail(c, src, "pfaai_stream_matrix: the sink stopped the stream") : PFAAI_RC_OK;
    };
    for (int64_t k = 0; k < ntiles; ++k) {
        const int b = (int)(k & 1);
        int64_t r0, r1;
        tile(k, r0, r1);
        const size_t bytes = (size_t)(r1 - r0) * n_cols * sizeof(double);
        if (k >= 2 && (rc = deliver(k - 2))) { drain(); return rc; }
        if (k >= 2) HIPCHK(c, hipStreamWaitEvent(c->stream, c->st_copied[b], 0));
        if (!qt) HIPCHK(c, hipMemsetAsync(dptr(b), 0, bytes, c->stream));  // the diagonal stays 0 (main.cpp:143)
        rc = pfaai_run(c, r0, r1, flags | PFAAI_FLAG_FULL_ROWS | (k ? PFAAI_FLAG_KEEP_RUNS : 0u), dptr(b) - r0 * n_cols,
                       nullptr, nullptr, c->stream);
        if (rc) { drain(); return rc; }
        HIPCHK(c, hipMemcpyAsync(&evs[k], sc_ev, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipEventRecord(c->st_done[b], c->stream));
        HIPCHK(c, hipStreamWaitEvent(c->copy_stream, c->st_done[b], 0));
        HIPCHK(c, hipMemcpyAsync(hptr(b), dptr(b), bytes, hipMemcpyDeviceToHost, c->copy_stream));
        HIPCHK(c, hipEventRecord(c->st_copied[b], c->copy_stream));
    }
    for (int64_t k = std::max<int64_t>(0, ntiles - 2); k < ntiles; ++k)
        if ((rc = deliver(k))) { drain(); return rc; }
    return PFAAI_RC_OK;
}

int pfaai_stream_matrix(pfaai_ctx* c, int64_t rb, int64_t re, int64_t tile_rows, uint32_t flags,
                        pfaai_matrix_sink_fn sink, void* user) {
    if (!c) return PFAAI_RC_INVALID;
    if (c->order_n) return fail(c, PFAAI_RC_INVALID, "a row order is set (pfaai_set_row_order): only pfaai_run");
    return guarded(c, [&] { return stream_matrix_impl(c, rb, re, tile_rows, flags, sink, user); });
}

int pfaai_stream(pfaai_ctx* c, int64_t rb, int64_t re, int64_t tile_pairs, uint32_t flags, pfaai_sink_fn sink,
                 void* user) {
    if (!c) return PFAAI_RC_INVALID;
    if (c->order_n) return fail(c, PFAAI_RC_INVALID, "a row order is set (pfaai_set_row_order): only pfaai_run");
    return guarded(c, [&] { return stream_impl(c, rb, re, tile_pairs, flags, sink, user); });
}

int pfaai_stream_events(const pfaai_ctx* c, int64_t* n_events) {
    if (!c || !n_events) return PFAAI_RC_INVALID;
    *n_events = c->st_events;
    return PFAAI_RC_OK;
}


// F construction on the device (SURVEY 8b pfaai_build_f; ds_helper.hpp:82-162,
// scp_db.hpp:161-262): count Lc / T, stable LSD radix sort of the triples by
// tetramer * P + protein (8-bit digits, the work-list sort's kernels), split
// the sorted (protein, genome) records into the F columns.
static int build_f_impl(pfaai_ctx* c, const int32_t* prot, const int32_t* genome, const int32_t* tetra, int64_t n,
                        int32_t n_prot, int32_t n_genome, int32_t* Lc_out, int64_t* Lp_out, int32_t* F_prot_out,
                        int32_t* F_genome_out, int32_t* T_out) {
    if (!c) return PFAAI_RC_INVALID;
    if (n < 0 || n > kMaxF || n_prot < 1 || n_prot >= kMaxRuns || n_genome < 1)
        return fail(c, PFAAI_RC_INVALID, "pfaai_build_f: bad sizes (|F| <= 2^32 - 64, 1 <= n_prot < 4096)");
    if ((n && (!prot || !genome || !tetra || !F_prot_out || !F_genome_out)) || !Lc_out || !Lp_out)
        return fail(c, PFAAI_RC_INVALID, "pfaai_build_f: null array");
    {  // ranges, and every protein's triples in non-decreasing genome order (the stable sort keeps it)
        std::vector<int32_t> last(n_prot, -1);
        for (int64_t i = 0; i < n; ++i) {
            const int32_t p = prot[i], g = genome[i], t = tetra[i];
            if (p < 0 || p >= n_prot || g < 0 || g >= n_genome || t < 0 || t >= PFAAI_NTETRAMERS)
                return fail(c, PFAAI_RC_INVALID, "pfaai_build_f: protein, genome or tetramer id out of range");
            if (g < last[p])
                return fail(c, PFAAI_RC_INVALID,
                            "pfaai_build_f: triples of a protein must come in non-decreasing genome order");
            last[p] = g;
        }
    }
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t s = c->stream;
    int rc;
    const int64_t nn = std::max<int64_t>(n, 1);
    DevBuf in_p, in_g, in_t, Tdev;
    auto cleanup = [&]() { release(in_p); release(in_g); release(in_t); release(Tdev); release_sort_space(c); };
    if ((rc = upload(c, in_p, prot, n)) || (rc = upload(c, in_g, genome, n)) || (rc = upload(c, in_t, tetra, n))) {
        cleanup();
        return rc;
    }
    if ((rc = ensure(c, c->key_c, nn * 4)) || (rc = ensure(c, c->rec_c, nn * 8)) || (rc = ensure(c, c->recs, nn * 8)) ||
        (rc = ensure(c, c->cnt_t, PFAAI_NTETRAMERS * 4)) || (rc = ensure_sort_space(c, n))) {
        cleanup();
        return rc;
    }
    const size_t tbytes = (size_t)n_prot * n_genome * sizeof(int32_t);
    if (T_out && (rc = ensure(c, Tdev, tbytes))) { cleanup(); return rc; }
    auto* cnt = static_cast<uint32_t*>(c->cnt_t.p);
    HIPCHK(c, hipMemsetAsync(cnt, 0, PFAAI_NTETRAMERS * 4, s));
    if (T_out) HIPCHK(c, hipMemsetAsync(Tdev.p, 0, tbytes, s));
    auto* keys0 = static_cast<uint32_t*>(c->key_c.p);
    auto* rec0 = static_cast<uint2*>(c->rec_c.p);
    const int grid = (int)std::min<int64_t>(ceil_div(nn, 256), 8192);
    if (n)
        hipLaunchKernelGGL(k_f_keys, dim3(grid), dim3(256), 0, s, static_cast<const int32_t*>(in_p.p),
                           static_cast<const int32_t*>(in_g.p), static_cast<const int32_t*>(in_t.p), n, n_prot,
                           n_genome, keys0, rec0, cnt, static_cast<int32_t*>(T_out ? Tdev.p : nullptr));
    HIPCHK(c, hipGetLastError());
    auto* recs = static_cast<uint2*>(c->recs.p);
    if (n) {
        if ((rc = radix_sort_recs(c, keys0, n, bits_for((int64_t)PFAAI_NTETRAMERS * n_prot), rec0, recs, s, nullptr))) {
            cleanup();
            return rc;
        }
        // the F columns into two free key-sized buffers
        int32_t* fp = static_cast<int32_t*>(c->key_a.p);
        int32_t* fg = static_cast<int32_t*>(c->key_b.p);
        hipLaunchKernelGGL(k_f_split, dim3(grid), dim3(256), 0, s, recs, n, fp, fg);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipMemcpyAsync(F_prot_out, fp, n * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(F_genome_out, fg, n * 4, hipMemcpyDeviceToHost, s));
    }
    std::vector<uint32_t> lc(PFAAI_NTETRAMERS);
    HIPCHK(c, hipMemcpyAsync(lc.data(), cnt, PFAAI_NTETRAMERS * 4, hipMemcpyDeviceToHost, s));
    if (T_out) HIPCHK(c, hipMemcpyAsync(T_out, Tdev.p, tbytes, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    cleanup();  // also the work-list buffers: a later work-list run re-allocates them
    Lp_out[0] = 0;
    for (int t = 0; t < PFAAI_NTETRAMERS; ++t) {
        Lc_out[t] = (int32_t)lc[t];
        Lp_out[t + 1] = Lp_out[t] + lc[t];
    }
    return PFAAI_RC_OK;
}


int pfaai_build_f(pfaai_ctx* c, const int32_t* prot, const int32_t* genome, const int32_t* tetra, int64_t n,
                  int32_t n_prot, int32_t n_genome, int32_t* Lc_out, int64_t* Lp_out, int32_t* F_prot_out,
                  int32_t* F_genome_out, int32_t* T_out) {
    if (!c) return PFAAI_RC_INVALID;
    return guarded(c, [&] {
        return build_f_impl(c, prot, genome, tetra, n, n_prot, n_genome, Lc_out, Lp_out, F_prot_out, F_genome_out, T_out);
    });
}

// Rows into host arrays at their JAC span: one thread per context (device)
// runs its own row block; the spans of disjoint row blocks are disjoint in
// ALL and QT, so several devices fill one host JAC array without a gather.
// A query-subset row block (ds_impl.hpp:251-305): rows [rb, re) are query
// file indices.  Their nQ x nT cross cells are the contiguous span [rb * nT,
// re * nT); their query-query cells lie in the triangle after all cross
// rows, each pair owned by the row of its smaller genome id (isValidPair,
// ds_impl.hpp:270-273) but placed by query file index -- not contiguous, and
// not even confined to the block's rows when the -q list is not in id order
// (SURVEY 8a row U).  So the block runs into a device copy of its hull with
// the triangle's N preset to -1, the cross span is copied out directly, and
// the triangle's written cells (N >= 0: every owned pair is written, zero
// overlaps included) are merged into the caller's arrays -- the blocks of a
// split own disjoint cells, so per-device threads may fill one output.
static int compute_rows_qsub(pfaai_ctx* c, int64_t rb, int64_t re, uint32_t flags, double* h_aji, double* h_S,
                             int32_t* h_N) {
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t nT = c->prob.n_tgt, f = rb * nT, tri0 = (int64_t)c->prob.n_qry * nT;
    const int64_t n = c->n_pairs - f, ncross = (re - rb) * nT, ntri = c->n_pairs - tri0;
    int rc;
    if ((rc = ensure(c, c->out_aji, std::max<int64_t>(n, 1) * sizeof(double)))) return rc;
    if ((rc = ensure(c, c->out_S, std::max<int64_t>(n, 1) * sizeof(double)))) return rc;
    if ((rc = ensure(c, c->out_N, std::max<int64_t>(n, 1) * sizeof(int32_t)))) return rc;
    auto* aji = static_cast<double*>(c->out_aji.p);
    auto* S = static_cast<double*>(c->out_S.p);
    auto* N = static_cast<int32_t*>(c->out_N.p);
    HIPCHK(c, hipMemsetAsync(N + (tri0 - f), 0xFF, ntri * sizeof(int32_t), c->stream));
    rc = pfaai_run(c, rb, re, flags | PFAAI_FLAG_EMIT_JAC, aji - f, S - f, N - f, c->stream);
    if (rc) return rc;
    if (h_aji && (rc = staged_copy(c, h_aji + f, aji, ncross * sizeof(double), false, c->stream))) return rc;
    if (h_S && (rc = staged_copy(c, h_S + f, S, ncross * sizeof(double), false, c->stream))) return rc;
    if (h_N && (rc = staged_copy(c, h_N + f, N, ncross * sizeof(int32_t), false, c->stream))) return rc;
    if (ntri > 0) {
        std::vector<double> ta((size_t)ntri), ts((size_t)ntri);
        std::vector<int32_t> tn((size_t)ntri);
        if ((rc = staged_copy(c, tn.data(), N + (tri0 - f), ntri * sizeof(int32_t), false, c->stream))) return rc;
        if ((rc = staged_copy(c, ta.data(), aji + (tri0 - f), ntri * sizeof(double), false, c->stream))) return rc;
        if ((rc = staged_copy(c, ts.data(), S + (tri0 - f), ntri * sizeof(double), false, c->stream))) return rc;
        HIPCHK(c, hipStreamSynchronize(c->stream));
        par_for(ntri, [&](int64_t lo, int64_t hi, int) {
            for (int64_t i = lo; i < hi; ++i) {
                if (tn[(size_t)i] < 0) continue;  // another block's cell
                if (h_aji) h_aji[tri0 + i] = ta[(size_t)i];
                if (h_S) h_S[tri0 + i] = ts[(size_t)i];
                if (h_N) h_N[tri0 + i] = tn[(size_t)i];
            }
        });
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return PFAAI_RC_OK;
}

int pfaai_compute_rows(pfaai_ctx* c, int64_t rb, int64_t re, uint32_t flags, double* h_aji, double* h_S,
                       int32_t* h_N) {
    if (!c) return PFAAI_RC_INVALID;
    if (!c->loaded) return fail(c, PFAAI_RC_INVALID, "no problem loaded");
    if (rb < 0 || re > c->n_rows || rb > re) return fail(c, PFAAI_RC_INVALID, "row range out of bounds");
    if (c->order_n) return fail(c, PFAAI_RC_INVALID, "a row order is set (pfaai_set_row_order): only pfaai_run");
    if (rb == re) return PFAAI_RC_OK;
    if (c->prob.mode == PFAAI_MODE_QSUB && !(rb == 0 && re == c->n_rows)) return compute_rows_qsub(c, rb, re, flags, h_aji, h_S, h_N);
    HIPCHK(c, hipSetDevice(c->device));
    int64_t f = 0, n = 0;
    pfaai_row_span(c, rb, re, &f, &n);
    int rc;
    if ((rc = ensure(c, c->out_aji, n * sizeof(double)))) return rc;
    if ((rc = ensure(c, c->out_S, n * sizeof(double)))) return rc;
    if ((rc = ensure(c, c->out_N, n * sizeof(int32_t)))) return rc;
    auto* aji = static_cast<double*>(c->out_aji.p);
    auto* S = static_cast<double*>(c->out_S.p);
    auto* N = static_cast<int32_t*>(c->out_N.p);
    if (c->prob.mode == PFAAI_MODE_QSUB) {  // the hull holds every pair; the kernel writes them all
        HIPCHK(c, hipMemsetAsync(aji, 0, n * sizeof(double), c->stream));
        HIPCHK(c, hipMemsetAsync(S, 0, n * sizeof(double), c->stream));
        HIPCHK(c, hipMemsetAsync(N, 0, n * sizeof(int32_t), c->stream));
    }
    rc = pfaai_run(c, rb, re, flags | PFAAI_FLAG_EMIT_JAC, aji - f, S - f, N - f, c->stream);
    if (rc) return rc;
    if (h_aji && (rc = staged_copy(c, h_aji + f, aji, n * sizeof(double), false, c->stream))) return rc;
    if (h_S && (rc = staged_copy(c, h_S + f, S, n * sizeof(double), false, c->stream))) return rc;
    if (h_N && (rc = staged_copy(c, h_N + f, N, n * sizeof(int32_t), false, c->stream))) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return PFAAI_RC_OK;
}

}  // extern "C"
