// pfaai_ctx.hpp -- the engine context (pfaai_ctx) and the host helpers
// shared by the C-ABI translation unit (pfaai_hip.hip) and the row-kernel
// translation units (pfaai_rows_m{0,1,2}.hip, one per mode, compiled in
// parallel: each instantiates launch_rows<MODE> of pfaai_launch.hpp).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "pfaai_hip.h"
#include "pfaai_kernels.hpp"
#include "pfaai_rows_pl.hpp"  // kernel constants (kPlEntries, kClkBlocks); templates only

// Diagnostic switches that change results or instrument the kernels
// (PFAAI_ABLATE, PFAAI_BLK_ABLATE: skip kernel phases; PFAAI_PL_CLK: stage
// clocks; PFAAI_DIV_NEWTON: the division self-test's refinement count) exist
// only in a library built with -DPFAAI_DIAGNOSTICS (tools/build_native.py
// --diag -> libpfaai_hip_diag.so).  The release library never reads them.
#ifdef PFAAI_DIAGNOSTICS
#define DIAG_ENV(name) getenv(name)
#else
#define DIAG_ENV(name) (static_cast<const char*>(nullptr))
#endif

namespace pfaai_impl {

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

// staged_copy's pinned buffer: kStageThreads host threads x two slots
constexpr int kStageThreads = 16;
constexpr size_t kStageSlot = (size_t)1 << 20;
constexpr size_t kStageBytes = 2 * (size_t)kStageThreads * kStageSlot;

}  // namespace pfaai_impl

struct pfaai_ctx {
    using DevBuf = pfaai_impl::DevBuf;
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    bool loaded = false;
    double load_ms[3] = {0, 0, 0};  // last pfaai_load: host checks, H2D uploads, device F/G build (HIP events)
    int32_t load_path = 0;          // PFAAI_LOAD_*: which transposition the last load ran (pfaai_load_info)

    // problem (host copies of scalars + small maps)
    pfaai_problem prob{};
    int64_t n_rows = 0, n_pairs = 0;
    std::vector<int32_t> row_genome_h;
    std::vector<int32_t> q_index_h;
    int32_t max_cols = 0;  // widest output row of the loaded mode
    int32_t cols_run = 0;  // widest row of the current run (max_cols; n_ids for full rows)

    // device-resident problem
    DevBuf T16, T16c;      // u16 T by column genome (k_rows_pl)
    int64_t max_glen = 0;  // longest (genome, protein) G list
    // T[p][g] is the length of every list (g, p) (checked at load): then
    // every denominator T[p][A] + T[p][B] - c of a row with entries in p is
    // >= 1, which the WK 3 row kernel relies on (it divides without a clamp)
    bool t_exact = false;
    DevBuf Fp16;
    DevBuf Lp, Fp, Fg, T, is_q, q_index, t_rank, row_of, row_genome, tcol_row, tcol_col, G_off, G_tet, G_pos, blk;
    DevBuf G_end;  // end of the F run of every G entry (the fallback builds, packed into G_pe)
    DevBuf G_pe;   // (G_pos, G_end) of every G entry, interleaved: what k_rows_pl WK 3 reads
    DevBuf Fcode;  // member codes of F (k_fcode; with G_end, the WK 3 member scatter)
    bool has_g = false;
    bool runs_valid = false;  // run table (and, if runs_key, the first E key) built for the loaded problem
    bool runs_key = false;
    bool runs_ends = false;  // the run table holds u32 run ends only (k_blk_end, k_rows_pl WK 3)
    bool wl_ready = false;  // work-list buffers allocated (ensure_worklists)
    pfaai::Dev dev{};

    // work space (sized at load for all rows, so runs never allocate)
    DevBuf cnt_t, off_t;
    DevBuf rowptr, lens, key_c, rec_c, key_a, key_b, val_a, val_b, hist, hoff, recs, sums, scalars;
    DevBuf out_aji, out_S, out_N, dbg;
    DevBuf srec_a, srec_b, shist, sgsum, sbase;  // the load-time transposition sort (pfaai_sort.hpp)
    DevBuf tails;  // the run-end sort's block-end bitmap and per-tile tables
    DevBuf ranks;  // the run-end sort's check: block ends before each tile, tetramer ranks (u64)
    // all-vs-all rows whose walk data (G_pos, G_end) the last load built:
    // genomes [pos_lo, pos_hi) (pfaai_load_rows; pfaai_load: all)
    int32_t pos_lo = 0, pos_hi = 0;
    // the genomes whose caller-given G lists the load verified against F (a
    // both-given pfaai_load_rows checks its block only): rows beyond them
    // are refused, since every walk reads the row genome's G lists
    int32_t chk_lo = 0, chk_hi = 0;
    // pfaai_set_row_order (all-vs-all): rows [0, order_n) are the caller's
    // ascending genome list (0: rows are the genomes in id order), whose
    // genomes all lie in the walk-data block when order_in_pos
    int64_t order_n = 0;
    bool order_in_pos = false;
    int64_t run_rb = 0, run_re = 0;  // rows of the current pfaai_run (pl_uses_ends)
    hipEvent_t load_ev[2] = {nullptr, nullptr};  // device span of the last load's F / G build
    hipEvent_t side_ev[2] = {nullptr, nullptr};  // the load's fork to / join from copy_stream (k_hash_f)
    // the narrow all-vs-all rows' launch beside the wide rows (launch_narrow):
    // its own stream and fork / join events, so the streamed outputs' D2H
    // copies on copy_stream never queue it
    hipStream_t side_stream = nullptr;
    hipEvent_t narrow_ev[2] = {nullptr, nullptr};
    std::vector<int64_t> row_fprefix;  // F entries of rows [0, r): exact work-list sizes

    // staged copies to / from the caller's pageable memory (staged_copy):
    // kStageThreads pairs of kStageSlot-byte pinned slots and their events
    void* stage_host = nullptr;
    hipEvent_t stage_ev[2 * pfaai_impl::kStageThreads] = {};
    // output-tile streaming (pfaai_stream): copy stream, tile events, pinned buffers
    hipStream_t copy_stream = nullptr;
    hipEvent_t st_done[2] = {nullptr, nullptr}, st_copied[2] = {nullptr, nullptr};
    void* st_host = nullptr;
    size_t st_host_bytes = 0;
    DevBuf st_dev;
    int64_t st_events = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
    bool timed = false;
    int rows_kernel = 0;  // RowsKernel of the current run
    int32_t last_walk = -1;      // PFAAI_WALK_* of the last run's k_rows_pl launches (pfaai_run_walk)
    bool last_narrow = false;    // the last run's narrow rows ran beside it (launch_narrow)
    // per-run event triples for pfaai_timing (pool reused after each reset)
    std::vector<hipEvent_t> pool;
    size_t pool_used = 0;
    bool windows = false;  // this run: absolute column windows, a run table per window
    DevBuf blkw;           // the window tables (window-major), built by k_blk<true>
    bool win_valid = false, win_key = false;
    int64_t win_cols = 0;
    // the next (start, after build, after rows) event triple of the pool
    hipEvent_t* take_events() {
        while (pool.size() < pool_used + 3) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return nullptr;
            pool.push_back(e);
        }
        hipEvent_t* ev = &pool[pool_used];
        pool_used += 3;
        ev0 = ev[0];
        ev1 = ev[1];
        ev2 = ev[2];
        return ev;
    }
};

namespace pfaai_impl {

using namespace pfaai;

// Row kernels.  PL (k_rows_pl, 1024 threads, <= 64 VGPRs so two workgroups
// share a CU: 12.2 ms at 10k vs 15.6 at one per CU) is the default for
// genome-major input; PL512 is its 512-thread form (13.9 ms); FUSED (k_rows<true>) takes
// G lists longer than k_rows_pl does; WORKLIST (k_rows<false> over sorted
// work lists) serves F-only input.  PFAAI_ROWS_KERNEL=pl|pl512|fused|worklist
// overrides the choice (A/B runs, tools/gpu/ab_rows.py; tests).
constexpr int64_t kMaxF = ((int64_t)1 << 32) - 64;
constexpr int32_t kGposMaxIds = 20480;  // G_pos built for all-vs-all problems up to two row chunks wide

enum RowsKernel { RK_PL = 0, RK_PL512 = 1, RK_FUSED = 2, RK_WORKLIST = 3 };

// scalars buffer layout (u64 each)
// SC_HF / SC_HG: the both-given load's membership sums over F (k_hash_f) and
// over G (k_gend), pfaai_sort.hpp DstGpos
// (second lanes SC_HF2 / SC_HG2 = SC_HF / SC_HG + 2, keyed by an independent seed)
enum { SC_GRAND = 0, SC_FIRST_KEY = 1, SC_EVENTS = 2, SC_ERR = 3, SC_NC = 4, SC_HF = 5, SC_HG = 6, SC_HF2 = 7, SC_HG2 = 8,
       SC_N = 9 };

inline int fail(pfaai_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

inline int hip_fail(pfaai_ctx* c, hipError_t e, const char* what) {
    if (e == hipErrorOutOfMemory)
        return fail(c, PFAAI_RC_OOM, std::string(what) + ": " + hipGetErrorString(e));
    return fail(c, PFAAI_RC_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIPCHK(ctx, call)                                  \
    do {                                                   \
        hipError_t e_ = (call);                            \
        if (e_ != hipSuccess) return hip_fail(ctx, e_, #call); \
    } while (0)

inline int ensure(pfaai_ctx* c, DevBuf& b, size_t bytes) {
    if (b.bytes >= bytes && b.p) return PFAAI_RC_OK;
    if (b.p) {
        (void)hipFree(b.p);
        b.p = nullptr;
        b.bytes = 0;
    }
    if (bytes == 0) bytes = 8;
    hipError_t e = hipMalloc(&b.p, bytes);
    if (e != hipSuccess) return hip_fail(c, e, "hipMalloc");
    b.bytes = bytes;
    return PFAAI_RC_OK;
}

inline void release(DevBuf& b) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
}

// pfaai_hip.hip: pageable host <-> device through the context's pinned slots
int staged_copy(pfaai_ctx* c, void* dst, const void* src, size_t bytes, bool to_device, hipStream_t s);

template <typename T>
inline int upload(pfaai_ctx* c, DevBuf& b, const T* src, size_t n) {
    int rc = ensure(c, b, n * sizeof(T));
    if (rc) return rc;
    // 4 MB .. 512 MB through the pinned slots (the CLI's C2 G_tet, 230 MB:
    // 15.6 -> 8.0 ms); above that the runtime's own pageable path is faster
    // (the bench's 1.15-GB arrays: ~25 ms each against 38 staged, round 5)
    const size_t nb = n * sizeof(T);
    if (nb >= ((size_t)4 << 20) && nb <= ((size_t)512 << 20)) return staged_copy(c, b.p, src, nb, true, c->stream);
    if (n) HIPCHK(c, hipMemcpy(b.p, src, n * sizeof(T), hipMemcpyHostToDevice));
    return PFAAI_RC_OK;
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Counter words per thread: the smallest KW with KW * nt >= the widest row
// (in u16 pairs); wider rows are cut into column chunks of 2 * KW * nt.
template <int NT>
inline int pick_kw(int32_t max_cols, int kw_max) {
    const int64_t words = ceil_div((int64_t)std::max<int32_t>(max_cols, 1) + 1, 2);
    for (int kw = 1; kw < kw_max; ++kw)
        if (words <= (int64_t)kw * NT) return kw;
    return kw_max;
}

// k_rows_pl's chunk width for this problem (launch_rows' KW choice)
inline int64_t pl_chunk_cols(pfaai_ctx* c) {
    if (c->rows_kernel == RK_PL512) return 2 * 512 * (int64_t)pick_kw<512>(c->cols_run, 10);
    const char* km = DIAG_ENV("PFAAI_PL_KWMAX");
    return 2 * 1024 * (int64_t)pick_kw<1024>(c->cols_run, km ? std::max(1, std::min(5, atoi(km))) : 5);
}

// k_rows_pl WK 3 -- all-vs-all rows in one chunk with G_pos loaded -- reads
// only the END of each G entry's run, so the step builds the u32 end table
// (k_blk_end) instead of k_blk's 16-B entries.  One predicate for the run
// table build (run_mode) and the kernel choice (launch_pl).
inline bool pl_uses_ends(pfaai_ctx* c, int mode) {
    return mode == 0 && (c->rows_kernel == RK_PL || c->rows_kernel == RK_PL512) && c->dev.G_pe && c->t_exact && !c->windows &&
           (c->order_n ? c->order_in_pos : c->run_rb >= c->pos_lo && c->run_re <= c->pos_hi) &&
           ceil_div((int64_t)c->cols_run + 1, pl_chunk_cols(c)) == 1 && !DIAG_ENV("PFAAI_PL_NOGPOS") &&
           !DIAG_ENV("PFAAI_PL_WK0");
}

// Column-window runs (c->windows) of all-vs-all and query-vs-target rows take
// k_rows_pl WK 4 where a window's sub-run holds only the row's partners: one
// launch over a grid of (row, window) with the member codes and no window
// test -- all-vs-all windows past the row's first column, every
// query-vs-target window (the tables stop at n_tgt); the all-vs-all rows'
// diagonal windows take one WK 1 launch.  PFAAI_PL_NOWK4=1 (diagnostics)
// keeps round 5's launch per window (A/B).
inline bool pl_win_spans(pfaai_ctx* c, int mode) {
    return c->windows && (mode == 0 || mode == 2) && c->rows_kernel == RK_PL && !DIAG_ENV("PFAAI_PL_NOWK4");
}

// Row kernels for output rows [rb, re) (pfaai_launch.hpp; instantiated per
// mode in pfaai_rows_m{0,1,2}.hip).
template <int MODE>
void launch_rows(pfaai_ctx* c, int64_t rb, int64_t re, uint32_t flags, double* aji, double* S, int32_t* N,
                 hipStream_t s);
template <int MODE>
void preload_rows();  // load the mode's row-kernel code object (pfaai_create)

}  // namespace pfaai_impl
