/*
 * pfaai_oracle.c -- CPU restatement of ParFastAAI's all-pairs AJI path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (parfastaai_amd/, the
 * C-ABI library, the CLI) links or calls this file; only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load it, and only as
 * the checker.  It is compiled by oracle/Makefile into oracle/_build/.
 *
 * Parity pinning: the reference restatement (oracle_ref_run) reproduces every
 * JAC/AJI golden vector the reference's own test-suite holds, bit-exactly
 * (tests/test_oracle.py: xanthodb, xdb_subset1/2, -q subset, -r QT incl. the
 * T-index quirk), and the E it builds equals the sorted-E fixtures.
 *
 * Two formulations are provided:
 *   oracle_ref_run   -- the reference's algorithm step for step: generate E
 *                       (ds_helper.hpp:206-357), sort it by (gA,gB,p)
 *                       (psort.hpp:27-53; here an LSD radix sort), find the
 *                       per-pair extents (algorithm_impl.hpp:123-219), walk the
 *                       protein sub-blocks (algorithm_impl.hpp:222-277) and
 *                       divide (algorithm_impl.hpp:309-322).
 *   oracle_dense_rows -- SURVEY.md Appendix A: dense per-protein intersection
 *                       counts for a window of output rows, then the same fp64
 *                       protein-ordered reduction.  Used to spot-check rows of
 *                       full-size GPU runs.
 *
 * Mode semantics (ds_impl.hpp):
 *   mode 0 all-vs-all      ParFAAIData      (ds_impl.hpp:38-151)
 *   mode 1 query subset    ParFAAIQSubData  (ds_impl.hpp:158-337)
 *   mode 2 query-vs-target ParFAAIQryTgtData(ds_impl.hpp:343-490)
 * compat = 1 reproduces the reference's quirks;
 * compat = 0 gives the corrected semantics (zero-overlap pairs -> 0, QT
 * denominators from the E ids).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORACLE_NTETRAMERS 160000

typedef struct {
    int32_t mode;      /* 0 all-vs-all, 1 query subset, 2 query-vs-target */
    int32_t n_ids;     /* genome ids used in F (mode 2: n_tgt + n_qry) */
    int32_t n_prot;    /* P: rows of T */
    int32_t t_cols;    /* columns of T (row-major P x t_cols) */
    int32_t n_qry;     /* |Q| (mode 1: query-file size, mode 2: query DB size) */
    int32_t n_tgt;     /* mode 1: n_ids - n_qry ; mode 2: target DB size */
    int32_t compat;    /* 1: reproduce reference quirks */
    int32_t pad_;
    const uint8_t* is_q;     /* [n_ids] (modes 1,2) */
    const int32_t* q_index;  /* [n_ids] query-file index (mode 1), -1 otherwise */
    const int32_t* t_rank;   /* [n_ids] rank among non-query genomes (mode 1) */
    const int32_t* q_lookup; /* [n_qry] DB id of i-th query (mode 1) */
    const int32_t* t_lookup; /* [n_tgt] DB id of i-th non-query (mode 1) */
} oracle_mode;

/* ---- mode index maps ---------------------------------------------------- */

static int is_qry(const oracle_mode* m, int32_t g) {
    /* isQryGenome: ds_impl.hpp:89, 267-269, 418-420 */
    return m->mode == 0 ? 1 : m->is_q[g];
}

static int is_valid(const oracle_mode* m, int32_t a, int32_t b) {
    if (m->mode == 0) return a < b; /* ds_impl.hpp:90-92 */
    if (m->mode == 1)               /* ds_impl.hpp:270-273 */
        return (m->is_q[a] && m->is_q[b] && a < b) ||
               (m->is_q[a] && !m->is_q[b] && a != b);
    return m->is_q[a] && !m->is_q[b]; /* ds_impl.hpp:421-423 */
}

int64_t oracle_n_pairs(const oracle_mode* m) {
    int64_t q = m->n_qry, t = m->n_tgt, n = m->n_ids;
    if (m->mode == 0) return n * (n - 1) / 2;      /* ds_impl.hpp:78-80 */
    if (m->mode == 1) return q * t + q * (q - 1) / 2; /* ds_impl.hpp:244-249 */
    return q * t;                                   /* ds_impl.hpp:406 */
}

static int64_t pair_index(const oracle_mode* m, int32_t a, int32_t b) {
    if (m->mode == 0) { /* ds_impl.hpp:83-86 */
        int64_t n = m->n_ids;
        return n * a + b - (int64_t)(a + 2) * (a + 1) / 2;
    }
    if (m->mode == 1) { /* ds_impl.hpp:251-263 */
        int qind = m->is_q[a] && !m->is_q[b];
        if (qind) return (int64_t)m->q_index[a] * m->n_tgt + m->t_rank[b];
        int64_t gia = m->q_index[a], gib = m->q_index[b];
        if (!m->compat && gia > gib) { int64_t x = gia; gia = gib; gib = x; }
        return (int64_t)m->n_qry * m->n_tgt +
               ((int64_t)m->n_qry * gia + gib - (gia + 2) * (gia + 1) / 2);
    }
    /* ds_impl.hpp:411-417: mapQueryId(a) * nT + mapTargetId(b) */
    return (int64_t)(a - m->n_tgt) * m->n_tgt + b;
}

/* initJAC: the genome ids stored in each JAC tuple (ds_impl.hpp:99-114,
 * 278-305, 428-439).  In mode 2 with compat these are the reference's
 * (buggy) ids i/nT, nQ + i%nT, which also drive its T lookups. */
void oracle_init_jac(const oracle_mode* m, int32_t* ga, int32_t* gb) {
    int64_t np = oracle_n_pairs(m);
    if (m->mode == 0) {
        int32_t a = 0, b = 1;
        for (int64_t i = 0; i < np; i++) {
            ga[i] = a; gb[i] = b;
            if (b == m->n_ids - 1) { a += 1; b = a + 1; } else { b += 1; }
        }
    } else if (m->mode == 1) {
        int64_t qt = (int64_t)m->n_qry * m->n_tgt;
        for (int64_t i = 0; i < qt; i++) {
            ga[i] = m->q_lookup[i / m->n_tgt];
            gb[i] = m->t_lookup[i % m->n_tgt];
        }
        int32_t a = 0, b = 1;
        for (int64_t i = qt; i < np; i++) {
            ga[i] = m->q_lookup[a]; gb[i] = m->q_lookup[b];
            if (b == m->n_qry - 1) { a += 1; b = a + 1; } else { b += 1; }
        }
    } else {
        for (int64_t i = 0; i < np; i++) {
            if (m->compat) {
                ga[i] = (int32_t)(i / m->n_tgt);
                gb[i] = (int32_t)(m->n_qry + i % m->n_tgt);
            } else {
                ga[i] = (int32_t)(m->n_tgt + i / m->n_tgt);
                gb[i] = (int32_t)(i % m->n_tgt);
            }
        }
    }
}

/* ---- E construction (ds_helper.hpp:206-357) ----------------------------- */

typedef struct { int32_t p, a, b; } etriple; /* ETriple: interface.hpp:92-121 */

/* countTetramerTuples (ds_helper.hpp:206-265) summed over all tetramers. */
int64_t oracle_count_e(const oracle_mode* m, const int64_t* Lp,
                       const int32_t* Fp, const int32_t* Fg) {
    int64_t total = 0;
    for (int t = 0; t < ORACLE_NTETRAMERS; t++) {
        int64_t s = Lp[t], e = Lp[t + 1];
        int64_t i = s;
        while (i < e) {
            int64_t j = i;
            int64_t nq = 0, nt = 0;
            while (j < e && Fp[j] == Fp[i]) {
                if (is_qry(m, Fg[j])) nq++; else nt++;
                j++;
            }
            /* countGenomePairs: ds_impl.hpp:93-96, 274-276, 424-426 */
            if (m->mode == 0) total += nq * (nq - 1) / 2;
            else if (m->mode == 1) total += nq * nt + nq * (nq - 1) / 2;
            else total += nq * nt;
            i = j;
        }
    }
    return total;
}

/* constructTetramerTuples (ds_helper.hpp:270-357): every valid (gi, gj) of
 * every (tetramer, protein) block, in F order. */
static int64_t generate_e(const oracle_mode* m, const int64_t* Lp,
                          const int32_t* Fp, const int32_t* Fg, etriple* E) {
    int64_t n = 0;
    for (int t = 0; t < ORACLE_NTETRAMERS; t++) {
        int64_t s = Lp[t], e = Lp[t + 1];
        int64_t l = s;
        while (l < e) {
            int64_t r = l;
            while (r < e && Fp[r] == Fp[l]) r++;
            for (int64_t i = l; i < r; i++) {
                int32_t ga = Fg[i];
                if (!is_qry(m, ga)) continue;
                for (int64_t j = l; j < r; j++) {
                    int32_t gb = Fg[j];
                    if (!is_valid(m, ga, gb)) continue;
                    E[n].p = Fp[l]; E[n].a = ga; E[n].b = gb;
                    n++;
                }
            }
            l = r;
        }
    }
    return n;
}

/* Sort E by (gA, gB, p) -- ETriple::operator< (interface.hpp:103-111).  The
 * reference uses a merge sort (psort.hpp:27-53); any correct sort gives the
 * same array because the key is total.  LSD radix on a 64-bit composite. */
static void sort_e(etriple* E, int64_t n, int32_t n_ids, int32_t n_prot) {
    if (n <= 1) return;
    uint64_t* key = (uint64_t*)malloc(sizeof(uint64_t) * n * 2);
    etriple* tmp = (etriple*)malloc(sizeof(etriple) * n);
    uint64_t* key2 = key + n;
    uint64_t maxk = 0;
    for (int64_t i = 0; i < n; i++) {
        key[i] = ((uint64_t)E[i].a * (uint64_t)n_ids + (uint64_t)E[i].b) *
                     (uint64_t)n_prot + (uint64_t)E[i].p;
        if (key[i] > maxk) maxk = key[i];
    }
    int64_t* cnt = (int64_t*)malloc(sizeof(int64_t) * 65536);
    for (int shift = 0; shift < 64 && (maxk >> shift) != 0; shift += 16) {
        memset(cnt, 0, sizeof(int64_t) * 65536);
        for (int64_t i = 0; i < n; i++) cnt[(key[i] >> shift) & 0xFFFF]++;
        int64_t run = 0;
        for (int d = 0; d < 65536; d++) { int64_t c = cnt[d]; cnt[d] = run; run += c; }
        for (int64_t i = 0; i < n; i++) {
            int64_t pos = cnt[(key[i] >> shift) & 0xFFFF]++;
            key2[pos] = key[i];
            tmp[pos] = E[i];
        }
        memcpy(key, key2, sizeof(uint64_t) * n);
        memcpy(E, tmp, sizeof(etriple) * n);
    }
    free(cnt); free(tmp); free(key);
}

/* Build the sorted E array (for the sorted-E fixtures).  Returns |E| or -1. */
int64_t oracle_build_sorted_e(const oracle_mode* m, const int64_t* Lp,
                              const int32_t* Fp, const int32_t* Fg,
                              int32_t* out_pab, int64_t cap) {
    int64_t ne = oracle_count_e(m, Lp, Fp, Fg);
    if (ne > cap) return -1;
    etriple* E = (etriple*)malloc(sizeof(etriple) * (ne > 0 ? ne : 1));
    int64_t got = generate_e(m, Lp, Fp, Fg, E);
    if (got != ne) { free(E); return -2; }
    sort_e(E, ne, m->n_ids, m->n_prot);
    memcpy(out_pab, E, sizeof(etriple) * ne);
    free(E);
    return ne;
}

/* ---- JAC / AJI (algorithm_impl.hpp:123-329) ------------------------------ */

/*
 * Full reference restatement.  Outputs in JAC-index order: S, N, AJI and the
 * tuple genome ids.  Returns |E| (>= 0) or a negative error.
 */
int64_t oracle_ref_run(const oracle_mode* m, const int64_t* Lp,
                       const int32_t* Fp, const int32_t* Fg, const int32_t* T,
                       double* S, int32_t* N, double* AJI, int32_t* ga,
                       int32_t* gb) {
    int64_t np = oracle_n_pairs(m);
    int64_t ne = oracle_count_e(m, Lp, Fp, Fg);
    etriple* E = (etriple*)malloc(sizeof(etriple) * (ne > 0 ? ne : 1));
    if (!E) return -1;
    if (generate_e(m, Lp, Fp, Fg, E) != ne) { free(E); return -2; }
    sort_e(E, ne, m->n_ids, m->n_prot);

    /* extents (algorithm_impl.hpp:123-219), value-initialised to 0 (90-91) */
    int64_t* st = (int64_t*)calloc(np > 0 ? np : 1, sizeof(int64_t));
    int64_t* en = (int64_t*)calloc(np > 0 ? np : 1, sizeof(int64_t));
    for (int64_t i = 0; i < ne;) {
        int64_t j = i;
        while (j < ne && E[j].a == E[i].a && E[j].b == E[i].b) j++;
        int64_t idx = pair_index(m, E[i].a, E[i].b);
        if (idx >= 0 && idx < np) { st[idx] = i; en[idx] = j - 1; }
        i = j;
    }
    oracle_init_jac(m, ga, gb);
    int32_t p0 = ne > 0 ? E[0].p : 0;
    for (int64_t k = 0; k < np; k++) {
        double s = 0.0;
        int32_t nn = 0;
        int32_t A = ga[k], B = gb[k];
        int64_t bl = st[k], bh = en[k];
        int has_events = !(bl == 0 && bh == 0) ||
                         (ne > 0 && pair_index(m, E[0].a, E[0].b) == k);
        if (has_events) {
            /* computeEBlockJAC (algorithm_impl.hpp:222-277) */
            int64_t ks = bl, ke = bl;
            while (ke <= bh) {
                int32_t p = E[ks].p;
                while (ke <= bh && E[ke].p == p) ke++;
                int64_t c = ke - ks;
                double j = (double)c / (double)((int64_t)T[(int64_t)p * m->t_cols + A] +
                                                T[(int64_t)p * m->t_cols + B] - c);
                s += j;
                nn += 1;
                ks = ke;
            }
        } else if (m->compat && ne > 0) {
            /* extents 0/0 -> one sub-block E[0..0] */
            double j = 1.0 / (double)((int64_t)T[(int64_t)p0 * m->t_cols + A] +
                                      T[(int64_t)p0 * m->t_cols + B] - 1);
            s += j;
            nn += 1;
        }
        S[k] = 0.0 + s;
        N[k] = nn;
        AJI[k] = nn ? s / nn : (m->compat ? s / nn : 0.0);
    }
    free(st); free(en); free(E);
    return ne;
}

/*
 * SURVEY.md Appendix A, restricted to a window of output rows.  A "row" is a
 * genome that can be the first element of a valid pair (mode 0: every
 * genome; modes 1/2: query genomes) and is identified by its genome id.
 * For each row id a in [row_lo, row_hi) and each genome id b, writes
 *   S[(a-row_lo)*n_ids + b], N[...]  (0 where (a,b) is not a valid pair).
 * Correct semantics only (compat ignored): T columns by E ids.
 * Returns the number of E events counted in the window.
 */
int64_t oracle_dense_rows(const oracle_mode* m, const int64_t* Lp,
                          const int32_t* Fp, const int32_t* Fg, const int32_t* T,
                          int32_t row_lo, int32_t row_hi, double* S, int32_t* N) {
    int64_t nr = row_hi - row_lo, ni = m->n_ids, P = m->n_prot;
    uint16_t* cnt = (uint16_t*)calloc((size_t)(nr * P * ni), sizeof(uint16_t));
    if (!cnt) return -1;
    int64_t events = 0;
    for (int t = 0; t < ORACLE_NTETRAMERS; t++) {
        int64_t s = Lp[t], e = Lp[t + 1];
        int64_t l = s;
        while (l < e) {
            int64_t r = l;
            while (r < e && Fp[r] == Fp[l]) r++;
            int32_t p = Fp[l];
            for (int64_t i = l; i < r; i++) {
                int32_t a = Fg[i];
                if (a < row_lo || a >= row_hi || !is_qry(m, a)) continue;
                for (int64_t j = l; j < r; j++) {
                    int32_t b = Fg[j];
                    if (!is_valid(m, a, b)) continue;
                    cnt[((a - row_lo) * P + p) * ni + b]++;
                    events++;
                }
            }
            l = r;
        }
    }
    for (int64_t r = 0; r < nr; r++) {
        int32_t a = (int32_t)(row_lo + r);
        for (int64_t b = 0; b < ni; b++) {
            double sum = 0.0;
            int32_t nn = 0;
            for (int64_t p = 0; p < P; p++) { /* ascending protein order */
                int64_t c = cnt[(r * P + p) * ni + b];
                if (c > 0) {
                    sum += (double)c / (double)((int64_t)T[p * m->t_cols + a] +
                                                T[p * m->t_cols + b] - c);
                    nn += 1;
                }
            }
            S[r * ni + b] = sum;
            N[r * ni + b] = nn;
        }
    }
    free(cnt);
    return events;
}

/*
 * SURVEY.md Appendix A for whole output rows, written in JAC-index order --
 * the form the full-output digests (tests/golden/make_full_digests.py) hash.
 * Same counts and the same fp64 reduction as oracle_dense_rows: c(p, a, b) =
 * the number of tetramer blocks whose protein-p run (ds_helper.hpp:312-331)
 * holds both a and b, S = sum over ascending p of c / (T[p][a] + T[p][b] - c)
 * (algorithm_impl.hpp:222-277: E sorted by (gA, gB, p), so the sub-blocks of
 * a pair come in protein order), N = proteins with c > 0, AJI = S / N
 * (algorithm_impl.hpp:318); a pair with no event gets 0 (corrected
 * semantics; compat is not supported here).  Derived from F alone: one walk
 * of F collects, for every row genome in the window, the runs (t, p) it is a
 * member of (in t order per protein), then the rows are counted
 * independently (OpenMP over rows, per-thread u16 counters).
 *
 * Rows [row_lo, row_hi) in the mode's row space: mode 0 row r = genome r,
 * columns b > r, JAC index n*r + b - (r+2)(r+1)/2 (ds_impl.hpp:83-86); mode 2
 * row q = query genome n_tgt + q, columns the targets b < n_tgt, JAC index
 * q*n_tgt + b (ds_impl.hpp:411-417).  Mode 1 is not supported (-3).  Outputs
 * are indexed by JAC index - (the first JAC index of row_lo).  Returns |E| of
 * the rows, or a negative error.
 */
int64_t oracle_full_rows(const oracle_mode* m, const int64_t* Lp, const int32_t* Fp, const int32_t* Fg,
                         const int32_t* T, int64_t row_lo, int64_t row_hi, double* S, int32_t* N, double* AJI) {
    if (m->mode == 1) return -3;
    const int64_t ni = m->n_ids, P = m->n_prot, tc = m->t_cols;
    const int64_t nrows = m->mode == 0 ? ni : m->n_qry;
    if (row_lo < 0 || row_hi > nrows || row_lo > row_hi) return -4;
    const int64_t nr = row_hi - row_lo;
    if (nr == 0) return 0;
    const int64_t g_lo = m->mode == 0 ? row_lo : m->n_tgt + row_lo; /* row genomes [g_lo, g_lo + nr) */
    /* the runs of every row genome, grouped by (row, protein), t-ascending */
    int64_t* off = (int64_t*)calloc((size_t)(nr * P + 1), sizeof(int64_t));
    if (!off) return -1;
    for (int t = 0; t < ORACLE_NTETRAMERS; t++)
        for (int64_t i = Lp[t]; i < Lp[t + 1]; i++) {
            const int64_t r = (int64_t)Fg[i] - g_lo;
            if (r >= 0 && r < nr) off[r * P + Fp[i] + 1]++;
        }
    for (int64_t k = 0; k < nr * P; k++) off[k + 1] += off[k];
    const int64_t nl = off[nr * P];
    uint32_t* run = (uint32_t*)malloc(sizeof(uint32_t) * 2 * (size_t)(nl > 0 ? nl : 1));
    int64_t* cur = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nr * P));
    if (!run || !cur) { free(off); free(run); free(cur); return -1; }
    memcpy(cur, off, sizeof(int64_t) * (size_t)(nr * P));
    for (int t = 0; t < ORACLE_NTETRAMERS; t++) {
        int64_t l = Lp[t];
        while (l < Lp[t + 1]) {
            int64_t r = l;
            while (r < Lp[t + 1] && Fp[r] == Fp[l]) r++;
            for (int64_t i = l; i < r; i++) {
                const int64_t w = (int64_t)Fg[i] - g_lo;
                if (w < 0 || w >= nr) continue;
                const int64_t k = cur[w * P + Fp[l]]++;
                run[2 * k] = (uint32_t)l;
                run[2 * k + 1] = (uint32_t)r;
            }
            l = r;
        }
    }
    free(cur);
    const int64_t first = m->mode == 0 ? ni * row_lo - (row_lo + 1) * row_lo / 2 : row_lo * m->n_tgt;
    int64_t events = 0;
    int bad = 0;
#pragma omp parallel reduction(+ : events)
    {
        uint16_t* cnt = (uint16_t*)calloc((size_t)ni, sizeof(uint16_t));
        int32_t* touched = (int32_t*)malloc(sizeof(int32_t) * (size_t)ni);
        double* srow = (double*)malloc(sizeof(double) * (size_t)ni);
        int32_t* nrow = (int32_t*)malloc(sizeof(int32_t) * (size_t)ni);
        if (!cnt || !touched || !srow || !nrow) {
#pragma omp atomic write
            bad = 1;
        } else {
#pragma omp for schedule(dynamic, 4)
            for (int64_t w = 0; w < nr; w++) {
                const int32_t a = (int32_t)(g_lo + w);
                const int64_t c_lo = m->mode == 0 ? a + 1 : 0, c_hi = m->mode == 0 ? ni : m->n_tgt;
                for (int64_t b = c_lo; b < c_hi; b++) { srow[b] = 0.0; nrow[b] = 0; }
                for (int64_t p = 0; p < P; p++) { /* ascending protein order */
                    int64_t nt = 0;
                    for (int64_t k = off[w * P + p]; k < off[w * P + p + 1]; k++)
                        for (uint32_t j = run[2 * k]; j < run[2 * k + 1]; j++) {
                            const int32_t b = Fg[j];
                            if (!is_valid(m, a, b)) continue;
                            if (cnt[b]++ == 0) touched[nt++] = b;
                        }
                    for (int64_t x = 0; x < nt; x++) {
                        const int32_t b = touched[x];
                        const int64_t c = cnt[b];
                        srow[b] += (double)c / (double)((int64_t)T[p * tc + a] + T[p * tc + b] - c);
                        nrow[b] += 1;
                        events += c;
                        cnt[b] = 0;
                    }
                }
                const int64_t base = (m->mode == 0 ? ni * a + c_lo - (int64_t)(a + 2) * (a + 1) / 2
                                                   : (g_lo + w - m->n_tgt) * m->n_tgt) - first;
                for (int64_t b = c_lo; b < c_hi; b++) {
                    const int64_t k = base + (b - c_lo);
                    S[k] = srow[b];
                    N[k] = nrow[b];
                    AJI[k] = nrow[b] ? srow[b] / nrow[b] : 0.0;
                }
            }
        }
        free(cnt); free(touched); free(srow); free(nrow);
    }
    free(run); free(off);
    return bad ? -1 : events;
}
