// pfaai_launch.hpp -- launchers of the row kernels (k_rows_pl, k_rows):
// kernel variant, counter words per thread, column chunks and column
// windows.  Included by the per-mode translation units pfaai_rows_m{0..3}.hip
// only.
#pragma once
#include "pfaai_ctx.hpp"
#include "pfaai_rows_pl.hpp"

namespace pfaai_impl {

// k_rows_pl's variant bits for the WK 3 walks (pfaai_rows_pl.hpp V): the
// release form kPlV; PFAAI_PL_V=0 selects round 4's form (diagnostics, A/B).
// The other forms (column windows, -q, -r, full rows) take kPlVG's S5 bits;
// MODE 2 (-r) only without PFAAI_FLAG_REF_COMPAT, as V kPlVG | 64 (compat
// compiled out: with both S5 forms in one kernel it spilled 114 VGPRs, none
// without); PFAAI_PL_VG=0 overrides (A/B).
constexpr int kPlV = 27;
constexpr int kPlVG = 9;

template <int MODE, int KW, int NT, int WPE, int NK>
void launch_pl(pfaai_ctx* c, int64_t rb, int64_t re, uint32_t flags, double* aji, double* S, int32_t* N,
               hipStream_t s) {
    const int32_t chunk = 2 * KW * NT;
    const int32_t nchunks = (int32_t)ceil_div((int64_t)c->cols_run + 1, chunk);
    const size_t lds = pl_lds_bytes<KW, NT, NK>(c->prob.n_prot);
    auto* sc = static_cast<unsigned long long*>(c->scalars.p);
    // |F| past 2^30 entries: member loads by 64-bit address (PFAAI_PL_BIGF=1 forces it, A/B)
    const bool bigf = (uint64_t)(c->prob.n_f + 16) * 4u > 0xFFFFFFFFull || DIAG_ENV("PFAAI_PL_BIGF");
    // member window test (k_rows_pl WK): one chunk per row reaches the last
    // id, so all-vs-all rows test only b > a and -q / full rows test nothing
    constexpr int kWk1 = MODE == 0 ? 1 : MODE == 2 ? 0 : 2;
    const int wk = nchunks == 1 && !DIAG_ENV("PFAAI_PL_WK0") ? kWk1 : 0;
    // all-vs-all rows in one chunk with G_pos loaded: each run walk starts just
    // past the row genome (k_rows_pl WK 3, pl_issue_m2<A8>)
    const bool gp = MODE == 0 && wk == 1 && pl_uses_ends(c, MODE);
#define PLK(BF, WKV, VV)                                                                                             \
    hipLaunchKernelGGL((k_rows_pl<MODE, KW, NT, WPE, false, NK, BF, WKV, VV>), dim3(r1 - r0, gy), dim3(NT), lds, s, \
                       dv, r0, chunk, ac, flags, sc + SC_FIRST_KEY, aji, S, N, sc + SC_EVENTS)
    auto rows = [&](const Dev& dv, int64_t r0, int64_t r1, int32_t gy, int32_t ac) {
        c->last_walk = gp ? PFAAI_WALK_GPOS : PFAAI_WALK_SPLITTERS;
        // MODE 2 (-r): kPlVG's bits only with the reference-compat quirk off,
        // compiled out (V bit 64); with it, V 0
        constexpr int VG = MODE == 2 ? (kPlVG | 64) : kPlVG;
        const bool vg = VG != 0 && !(MODE == 2 && (flags & PFAAI_FLAG_REF_COMPAT)) &&
                        !(DIAG_ENV("PFAAI_PL_VG") && atoi(DIAG_ENV("PFAAI_PL_VG")) == 0);
        if (wk == 0 || ac >= 0) {
            c->last_walk = PFAAI_WALK_SPLITTERS;
            if (vg) {
                if (bigf) PLK(true, 0, VG); else PLK(false, 0, VG);
            } else {
                if (bigf) PLK(true, 0, 0); else PLK(false, 0, 0);
            }
        } else if constexpr (kWk1 != 0) {
            if constexpr (MODE == 0) {
                if (gp) {  // (G_pos is built up to 20 480 genomes only: never BIGF)
                    if (bigf) { PLK(true, 3, 0); return; }
#ifdef PFAAI_DIAGNOSTICS
                    if (const char* v = DIAG_ENV("PFAAI_PL_V"); v && atoi(v) == 0) {  // round 4's form (A/B)
                        PLK(false, 3, 0);
                        return;
                    }
#endif
                    PLK(false, 3, kPlV);
                    return;
                }
            }
            if (vg) {
                if (bigf) PLK(true, kWk1, VG); else PLK(false, kWk1, VG);
            } else {
                if (bigf) PLK(true, kWk1, 0); else PLK(false, kWk1, 0);
            }
        }
    };
    if (nchunks == 1 || !c->windows) {
        rows(c->dev, rb, re, nchunks, kWinRow);
        return;
    }
    if (pl_win_spans(c, MODE)) {
        // WK 4 (pl_win_spans): the windows whose sub-runs hold only partners
        // as one launch over (row, window); all-vs-all rows' diagonal windows
        // (the window of the row's first column, unless it starts there) as
        // one WK 1 launch over the rows
        const int64_t ncols = MODE == 2 ? c->prob.n_tgt : c->prob.n_ids;
        const int32_t nwin = (int32_t)ceil_div(ncols, chunk);
        // the first window some row of [rb, re) reaches from its start: a+1 <= w * chunk
        const int32_t w_lo = MODE == 0 ? (int32_t)std::min<int64_t>(ceil_div(rb + 1, chunk), nwin) : 0;
        c->last_walk = PFAAI_WALK_SPANS;
        // the kernel offsets the window-major tables by its window index
        Dev dv = c->dev;
        dv.blk = static_cast<uint4*>(c->blkw.p);
        // (V 4: S5 without the denominator clamp where T is every list's
        // length.  V 32, 24-member tasks, only in the diagnostics build behind
        // PFAAI_PL_T24=1: fewer member rounds but slower, C4 rows 6.62 -> 6.87
        // ms, C5 rows 531 -> 557 ms (profiles/r06/ab_t24.txt); 8-member tasks,
        // one per lane, were slower still: C4 rows 6.92 -> 11.05 ms, C5 545 ->
        // 643 ms, profiles/r06/qt_c4_t8_ab.txt)
        constexpr int VS = MODE == 2 ? (kPlVG | 64 | 2) : (kPlVG | 2);
        const bool cm = MODE == 2 && (flags & PFAAI_FLAG_REF_COMPAT);  // V 0: the QT quirk's per-column division
        const bool tx = c->t_exact;
        if (w_lo < nwin) {
            const int64_t r0 = rb, r1 = re;
            const int32_t ac = kWinGrid0 - w_lo;
            const int32_t gy = nwin - w_lo;
#ifdef PFAAI_DIAGNOSTICS
            // stage clocks of the query-vs-target window spans (PFAAI_PL_CLK,
            // tools/gpu/stage_clocks.py --qt): the release form with the clock registers
            if constexpr (MODE == 2 && KW == 5 && NT == 1024) {
                if (!cm && tx && DIAG_ENV("PFAAI_PL_CLK") && c->dbg.bytes >= kClkBlocks * 16 * 8 * 8) {
                    auto* clk = static_cast<unsigned long long*>(c->dbg.p);
                    const bool t24 = DIAG_ENV("PFAAI_PL_T24") != nullptr;
                    if (bigf) {
                        if (t24)
                            hipLaunchKernelGGL((k_rows_pl<MODE, KW, NT, WPE, true, NK, true, 4, VS | 32 | 4>),
                                               dim3(r1 - r0, gy), dim3(NT), lds, s, dv, r0, chunk, ac, flags,
                                               sc + SC_FIRST_KEY, aji, S, N, sc + SC_EVENTS, clk);
                        else
                            hipLaunchKernelGGL((k_rows_pl<MODE, KW, NT, WPE, true, NK, true, 4, VS | 4>),
                                               dim3(r1 - r0, gy), dim3(NT), lds, s, dv, r0, chunk, ac, flags,
                                               sc + SC_FIRST_KEY, aji, S, N, sc + SC_EVENTS, clk);
                    } else {
                        if (t24)
                            hipLaunchKernelGGL((k_rows_pl<MODE, KW, NT, WPE, true, NK, false, 4, VS | 32 | 4>),
                                               dim3(r1 - r0, gy), dim3(NT), lds, s, dv, r0, chunk, ac, flags,
                                               sc + SC_FIRST_KEY, aji, S, N, sc + SC_EVENTS, clk);
                        else
                            hipLaunchKernelGGL((k_rows_pl<MODE, KW, NT, WPE, true, NK, false, 4, VS | 4>),
                                               dim3(r1 - r0, gy), dim3(NT), lds, s, dv, r0, chunk, ac, flags,
                                               sc + SC_FIRST_KEY, aji, S, N, sc + SC_EVENTS, clk);
                    }
                    return;
                }
            }
            if (DIAG_ENV("PFAAI_PL_T24")) {
                if (bigf) {
                    if (cm) PLK(true, 4, 0); else if (tx) PLK(true, 4, VS | 32 | 4); else PLK(true, 4, VS | 32);
                } else {
                    if (cm) PLK(false, 4, 0); else if (tx) PLK(false, 4, VS | 32 | 4); else PLK(false, 4, VS | 32);
                }
            } else
#endif
            {
                if (bigf) {
                    if (cm) PLK(true, 4, 0); else if (tx) PLK(true, 4, VS | 4); else PLK(true, 4, VS);
                } else {
                    if (cm) PLK(false, 4, 0); else if (tx) PLK(false, 4, VS | 4); else PLK(false, 4, VS);
                }
            }
        }
        if constexpr (MODE == 0) {
            const int64_t r0 = rb, r1 = re;
            const int32_t ac = kWinDiag;
            const int32_t gy = 1;
            if (tx) {  // (V 4 as above)
                if (bigf) PLK(true, 1, kPlVG | 4); else PLK(false, 1, kPlVG | 4);
            } else {
                if (bigf) PLK(true, 1, kPlVG); else PLK(false, 1, kPlVG);
            }
        }
        return;
    }
    // rows wider than one chunk (c->windows, set by run_mode, which built the
    // window tables): per absolute column window, the rows with columns in it
    // over that window's table
    const int64_t ncols = MODE == 2 ? c->prob.n_tgt : c->prob.n_ids;
    const int32_t nwin = (int32_t)ceil_div(ncols, chunk);
    for (int32_t w = 0; w < nwin; ++w) {
        int64_t r1 = re;
        if (MODE == 0) r1 = std::min<int64_t>(re, (int64_t)(w + 1) * chunk - 1);  // row a has columns a+1 ..
        if (r1 <= rb) continue;
        Dev dw = c->dev;
        dw.blk = static_cast<uint4*>(c->blkw.p) + (int64_t)w * c->prob.n_prot * kNTetramers;
        rows(dw, rb, r1, 1, w);
    }
#undef PLK
}

// One k_rows_pl launch shape (KW, NT, WPE) with the N storage (nl: u8 in
// LDS, P <= 255; else u16 in registers).
template <int MODE, int KW, int NT, int WPE>
void launch_pl_n(pfaai_ctx* c, bool nl, int64_t rb, int64_t re, uint32_t flags, double* aji, double* S,
                   int32_t* N, hipStream_t s) {
    if (nl) launch_pl<MODE, KW, NT, WPE, 1>(c, rb, re, flags, aji, S, N, s);
    else launch_pl<MODE, KW, NT, WPE, 0>(c, rb, re, flags, aji, S, N, s);
}

template <int MODE, int KW>
void launch_k_rows(pfaai_ctx* c, int64_t rb, int64_t re, uint32_t flags, double* aji, double* S, int32_t* N,
                   hipStream_t s) {
    const int32_t chunk = 2 * KW * kRowThreads;
    const int32_t nchunks = (int32_t)ceil_div(std::max<int32_t>(c->cols_run, 1), chunk);
    const size_t lds = (size_t)KW * kRowThreads * sizeof(uint32_t);
    auto* sc = static_cast<unsigned long long*>(c->scalars.p);
    auto* rowptr = static_cast<const unsigned long long*>(c->rowptr.p);
    auto* recs = static_cast<const uint2*>(c->recs.p);
    if (MODE == kModeFull || c->rows_kernel == RK_FUSED)
        hipLaunchKernelGGL((k_rows<MODE, KW, true>), dim3(re - rb, nchunks), dim3(kRowThreads), lds, s, c->dev, rb,
                           rowptr, recs, chunk, flags, sc + SC_FIRST_KEY, aji, S, N, sc + SC_EVENTS);
    else if constexpr (MODE != kModeFull)  // work lists: the reference modes only
        hipLaunchKernelGGL((k_rows<MODE, KW, false>), dim3(re - rb, nchunks), dim3(kRowThreads), lds, s, c->dev, rb,
                           rowptr, recs, chunk, flags, sc + SC_FIRST_KEY, aji, S, N, sc + SC_EVENTS);
}

// The narrow all-vs-all rows (<= kNarrowCols columns) as 512-thread WK 3
// workgroups, four per CU: a narrow row's time is its 100-protein chain, not
// its width, so twice the rows in flight per CU finish the narrow end sooner
// (the narrowest 8-way shard of 10k 1.11 -> 0.96 ms).  A launch reaching into
// the narrow end runs those rows on the second stream, concurrently with its
// wide rows on the caller's (10k all-vs-all 7.72 -> 7.58 ms;
// profiles/r03v/); a launch of narrow rows only runs them on the caller's
// stream.  Returns false where it does not apply (not the WK 3 path, or no
// narrow row in [rb, re)).  PFAAI_PL_NO512=1 (diagnostics) turns it off.
// (a row of c columns needs (c + 1) / 2 counter words -- its chunk starts at
// an even column -- so two words per thread of 512 cover 2 047 columns)
constexpr int kNarrowCols = 2 * 2 * 512 - 1;

// (a template, instantiated by launch_rows<0> only: as a plain inline
// function it instantiated the all-vs-all kernels in every mode's unit)
template <int MODE>
bool launch_narrow(pfaai_ctx* c, int64_t rb, int64_t re, uint32_t flags, double* aji, double* S, int32_t* N,
                          hipStream_t s) {
    if (DIAG_ENV("PFAAI_PL_NO512") || !pl_uses_ends(c, 0) || !c->side_stream || !c->narrow_ev[0] || !c->narrow_ev[1])
        return false;
    // all-vs-all: row r is genome g = row_genome_h[r] (r itself unless
    // pfaai_set_row_order gave an ascending list), n - 1 - g columns
    const int64_t n = c->prob.n_ids;
    const auto& rg = c->row_genome_h;
    const int64_t cut = std::lower_bound(rg.begin() + rb, rg.begin() + re, (int32_t)(n - 1 - kNarrowCols)) - rg.begin();
    if (cut >= re) return false;
    const int64_t cols_cut = n - 1 - rg[cut];
    const int32_t cols_all = c->cols_run;
    if (ceil_div(cols_cut + 1, 2 * 2 * 512) != 1) return false;  // one chunk, or not the WK 3 form
    auto narrow = [&](hipStream_t st) {
        c->last_narrow = true;
        c->cols_run = (int32_t)cols_cut;  // the narrow launch's widest row
        if (pick_kw<512>(c->cols_run, 2) == 1)
            launch_pl_n<0, 1, 512, 8>(c, true, cut, re, flags, aji, S, N, st);
        else
            launch_pl_n<0, 2, 512, 8>(c, true, cut, re, flags, aji, S, N, st);
        c->cols_run = cols_all;
    };
    if (cut == rb) {
        narrow(s);
        return true;
    }
    // fork: the narrow rows on the side stream after everything before this
    // launch on s; join: s waits for them before what follows (the run's end event)
    if (hipEventRecord(c->narrow_ev[0], s) != hipSuccess || hipStreamWaitEvent(c->side_stream, c->narrow_ev[0], 0) != hipSuccess)
        return false;
    narrow(c->side_stream);
    switch (pick_kw<1024>(cols_all, 5)) {
        case 1: launch_pl_n<0, 1, 1024, 8>(c, true, rb, cut, flags, aji, S, N, s); break;
        case 2: launch_pl_n<0, 2, 1024, 8>(c, true, rb, cut, flags, aji, S, N, s); break;
        case 3: launch_pl_n<0, 3, 1024, 8>(c, true, rb, cut, flags, aji, S, N, s); break;
        case 4: launch_pl_n<0, 4, 1024, 8>(c, true, rb, cut, flags, aji, S, N, s); break;
        default: launch_pl_n<0, 5, 1024, 8>(c, true, rb, cut, flags, aji, S, N, s); break;
    }
    (void)hipEventRecord(c->narrow_ev[1], c->side_stream);
    (void)hipStreamWaitEvent(s, c->narrow_ev[1], 0);
    return true;
}

template <int MODE>
void launch_rows(pfaai_ctx* c, int64_t rb, int64_t re, uint32_t flags, double* aji, double* S, int32_t* N,
                 hipStream_t s) {
#define KR_CASE(K) \
    case K: launch_k_rows<MODE, K>(c, rb, re, flags, aji, S, N, s); break;
    // N in LDS (P <= 255; PFAAI_PL_NREG=1 keeps it in registers, A/B)
    const bool nl = c->prob.n_prot <= 255 && !DIAG_ENV("PFAAI_PL_NREG");
#ifdef PFAAI_DIAGNOSTICS
    // (RK_PL512 is reachable only through PFAAI_ROWS_KERNEL: the release
    // library compiles none of its instantiations)
    if constexpr (MODE != kModeFull) {  // full rows: k_rows_pl / fused only
        if (c->rows_kernel == RK_PL512) {
            // 512-thread workgroups, four per CU (<= 64 VGPRs), for A/B of
            // narrow launches (more rows in flight per CU); KW >= 5 keeps N
            // in registers at two workgroups per CU
            switch (pick_kw<512>(c->cols_run, 10)) {
                case 1: launch_pl_n<MODE, 1, 512, 8>(c, nl, rb, re, flags, aji, S, N, s); break;
                case 2: launch_pl_n<MODE, 2, 512, 8>(c, nl, rb, re, flags, aji, S, N, s); break;
                case 3: launch_pl_n<MODE, 3, 512, 8>(c, nl, rb, re, flags, aji, S, N, s); break;
                case 4: launch_pl_n<MODE, 4, 512, 8>(c, nl, rb, re, flags, aji, S, N, s); break;
                case 5: launch_pl_n<MODE, 5, 512, 4>(c, false, rb, re, flags, aji, S, N, s); break;
                case 6: launch_pl_n<MODE, 6, 512, 4>(c, false, rb, re, flags, aji, S, N, s); break;
                case 7: launch_pl_n<MODE, 7, 512, 4>(c, false, rb, re, flags, aji, S, N, s); break;
                case 8: launch_pl_n<MODE, 8, 512, 4>(c, false, rb, re, flags, aji, S, N, s); break;
                case 9: launch_pl_n<MODE, 9, 512, 4>(c, false, rb, re, flags, aji, S, N, s); break;
                default: launch_pl_n<MODE, 10, 512, 4>(c, false, rb, re, flags, aji, S, N, s); break;
            }
            return;
        }
    }
#endif
    if (c->rows_kernel == RK_PL || (MODE == kModeFull && c->rows_kernel != RK_FUSED)) {
        const char* km = DIAG_ENV("PFAAI_PL_KWMAX");  // diagnostics: cap the counter words per thread
        const int kw = pick_kw<1024>(c->cols_run, km ? std::max(1, std::min(5, atoi(km))) : 5);
#ifdef PFAAI_DIAGNOSTICS
        // stage clocks at the benchmark shape (PFAAI_PL_CLK, tools/gpu/stage_clocks.py)
        if (MODE == 0 && kw == 5 && !c->windows && c->prob.n_prot <= 255 && DIAG_ENV("PFAAI_PL_CLK") &&
            c->dbg.bytes >= kClkBlocks * 16 * 8 * 8) {
            const int32_t chunk = 2 * 5 * 1024;
            const int32_t nchunks = (int32_t)ceil_div((int64_t)c->cols_run + 1, chunk);
            auto* sc = static_cast<unsigned long long*>(c->scalars.p);
            auto* clk = static_cast<unsigned long long*>(c->dbg.p);
            // the shipped wide form (WK 3 when the walk bounds are loaded, V = kPlV; 64 VGPRs, no spills
            // with the clock registers), all rows as 1024-thread workgroups
            if (pl_uses_ends(c, 0)) {
                hipLaunchKernelGGL((k_rows_pl<0, 5, 1024, 8, true, 1, false, 3, kPlV>), dim3(re - rb, 1), dim3(1024),
                                   (pl_lds_bytes<5, 1024, 1>(c->prob.n_prot)), s, c->dev, rb, chunk, -1, flags,
                                   sc + SC_FIRST_KEY, aji, S, N, sc + SC_EVENTS, clk);
                return;
            }
            hipLaunchKernelGGL((k_rows_pl<0, 5, 1024, 8, true, 1, false, 1, 0>), dim3(re - rb, nchunks), dim3(1024),
                               (pl_lds_bytes<5, 1024, 1>(c->prob.n_prot)), s, c->dev, rb, chunk, -1, flags,
                               sc + SC_FIRST_KEY, aji, S, N, sc + SC_EVENTS, clk);
            return;
        }
#endif
        if constexpr (MODE == 0) {
            if (nl && launch_narrow<MODE>(c, rb, re, flags, aji, S, N, s)) return;
        }
        switch (kw) {
            case 1: launch_pl_n<MODE, 1, 1024, 8>(c, nl, rb, re, flags, aji, S, N, s); break;
            case 2: launch_pl_n<MODE, 2, 1024, 8>(c, nl, rb, re, flags, aji, S, N, s); break;
            case 3: launch_pl_n<MODE, 3, 1024, 8>(c, nl, rb, re, flags, aji, S, N, s); break;
            case 4: launch_pl_n<MODE, 4, 1024, 8>(c, nl, rb, re, flags, aji, S, N, s); break;
            default: launch_pl_n<MODE, 5, 1024, 8>(c, nl, rb, re, flags, aji, S, N, s); break;
        }
    } else {
        switch (pick_kw<kRowThreads>(c->cols_run, 10)) {
            KR_CASE(1) KR_CASE(2) KR_CASE(3) KR_CASE(4) KR_CASE(5) KR_CASE(6) KR_CASE(8) KR_CASE(10)
            case 7: launch_k_rows<MODE, 8>(c, rb, re, flags, aji, S, N, s); break;
            case 9: launch_k_rows<MODE, 10>(c, rb, re, flags, aji, S, N, s); break;
            default: break;
        }
    }
#undef KR_CASE
}

// Load this translation unit's code object now (pfaai_create): the HIP
// runtime otherwise loads it at the first launch of one of its kernels, i.e.
// inside a caller's first timed run (k_rows_pl 9.0 ms cold vs 1.4 ms at C2).
template <int MODE>
void preload_rows() {
    hipFuncAttributes a;
    (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&k_rows_pl<MODE, 5, 1024, 8, false, 1, false, 0, 0>));
}

}  // namespace pfaai_impl
