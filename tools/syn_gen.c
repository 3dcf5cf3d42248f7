/*
 * syn_gen.c -- deterministic synthetic SCP/tetramer databases (SYN spec of
 * SURVEY.md §8d), produced directly as the arrays the reference's
 * DataStructInterface exposes (interface.hpp:246-250): Lc/Lp, F ordered by
 * (tetramer, protein, genome), T (P x G).  Bench and test infrastructure;
 * parfastaai_amd/syn.py wraps it and can also write the SQLite form.
 *
 * Spec: P SCPs; clades of K genomes (genome g in clade g / K, or, for a
 * query DB, q mod C); per protein a length L_p ~ U[120, 580); per (clade,
 * protein) an ancestral set of L_p tetramers uniform in [0, 160000); protein
 * 0 carries 2 core tetramers in every genome (so every pair overlaps);
 * genome g has protein p w.p. 0.98 (p = 0 always); its set is
 * {ancestral, each kept w.p. 0.9} U core U 5 uniform tetramers, deduplicated
 * and sorted.  Ancestral sets / lengths / core depend on `anc_seed` only, so
 * a query DB generated with another `genome_seed` shares the clades of its
 * target DB.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define NTET 160000

typedef struct {
    uint64_t anc_seed;     /* clades, protein lengths, core tetramers */
    uint64_t genome_seed;  /* per-genome sampling */
    int32_t n_genomes;
    int32_t n_prot;
    int32_t clade_size;    /* K */
    int32_t n_clades;      /* C (0: ceil(n_genomes / K)) */
    int32_t clade_mod;     /* 0: clade = g / K ; 1: clade = g mod C */
    int32_t n_random;      /* uniform extras per (g, p), default 5 */
    int32_t keep_permille; /* 900 */
    int32_t has_permille;  /* 980 */
} syn_params;

static uint64_t splitmix(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static uint64_t seed_of(uint64_t base, uint64_t a, uint64_t b, uint64_t c) {
    uint64_t s = base ^ (a * 0xD1B54A32D192ED03ull) ^ (b * 0xABC98388FB8FAC03ull) ^ (c * 0x8CB92BA72F3D8DD7ull);
    splitmix(&s);
    return s;
}

static uint32_t uni(uint64_t* s, uint32_t n) { return (uint32_t)(((splitmix(s) >> 32) * (uint64_t)n) >> 32); }

static int cmp_i32(const void* a, const void* b) {
    int32_t x = *(const int32_t*)a, y = *(const int32_t*)b;
    return (x > y) - (x < y);
}

static int32_t n_clades_of(const syn_params* p) {
    if (p->n_clades > 0) return p->n_clades;
    return (p->n_genomes + p->clade_size - 1) / p->clade_size;
}

static int32_t prot_len(const syn_params* p, int32_t prot) {
    uint64_t s = seed_of(p->anc_seed, 1, (uint64_t)prot, 0);
    return 120 + (int32_t)uni(&s, 460);
}

/* sorted, deduplicated ancestral set of (clade, prot); returns its size */
static int32_t ancestral(const syn_params* p, int32_t clade, int32_t prot, int32_t* out) {
    int32_t L = prot_len(p, prot);
    uint64_t s = seed_of(p->anc_seed, 2, (uint64_t)clade, (uint64_t)prot);
    for (int32_t i = 0; i < L; i++) out[i] = (int32_t)uni(&s, NTET);
    qsort(out, L, sizeof(int32_t), cmp_i32);
    int32_t n = 0;
    for (int32_t i = 0; i < L; i++)
        if (n == 0 || out[i] != out[n - 1]) out[n++] = out[i];
    return n;
}

/* tetramer set of (genome g, protein prot) given the clade's ancestral set;
 * returns size (0 if the genome lacks the protein). */
static int32_t genome_set(const syn_params* p, int32_t g, int32_t prot, const int32_t* anc, int32_t na,
                          int32_t* out) {
    uint64_t s = seed_of(p->genome_seed, 3, (uint64_t)g, (uint64_t)prot);
    if (prot != 0 && (int32_t)uni(&s, 1000) >= p->has_permille) return 0;
    int32_t extra[16];
    int32_t ne = 0;
    if (prot == 0) {
        uint64_t cs = seed_of(p->anc_seed, 4, 0, 0);
        extra[ne++] = (int32_t)uni(&cs, NTET);
        extra[ne++] = (int32_t)uni(&cs, NTET);
    }
    for (int32_t i = 0; i < p->n_random && ne < 16; i++) extra[ne++] = (int32_t)uni(&s, NTET);
    qsort(extra, ne, sizeof(int32_t), cmp_i32);
    /* merge filtered ancestral with extras, dedup */
    int32_t n = 0, i = 0, j = 0;
    while (i < na || j < ne) {
        int32_t v;
        if (j >= ne || (i < na && anc[i] <= extra[j])) {
            v = anc[i++];
            if ((int32_t)uni(&s, 1000) >= p->keep_permille) continue;
        } else {
            v = extra[j++];
        }
        if (n == 0 || out[n - 1] != v) out[n++] = v;
        else if (out[n - 1] > v) { /* cannot happen: inputs sorted */ }
    }
    return n;
}

static int32_t clade_of(const syn_params* p, int32_t g) {
    return p->clade_mod ? g % n_clades_of(p) : g / p->clade_size;
}

/*
 * Pass 1: T[prot * n_genomes + g] = |set(g, prot)|; returns |F| = sum T.
 */
int64_t syn_counts(const syn_params* p, int32_t* T) {
    const int32_t G = p->n_genomes, P = p->n_prot, C = n_clades_of(p);
    int64_t total = 0;
#pragma omp parallel reduction(+ : total)
    {
        int32_t* anc = (int32_t*)malloc(sizeof(int32_t) * 600);
        int32_t* set = (int32_t*)malloc(sizeof(int32_t) * 640);
#pragma omp for schedule(dynamic, 1)
        for (int32_t prot = 0; prot < P; prot++) {
            int32_t cur_clade = -1, na = 0;
            for (int32_t g = 0; g < G; g++) {
                int32_t cl = clade_of(p, g) % C;
                if (cl != cur_clade) { na = ancestral(p, cl, prot, anc); cur_clade = cl; }
                int32_t n = genome_set(p, g, prot, anc, na, set);
                T[(int64_t)prot * G + g] = n;
                total += n;
            }
        }
        free(anc);
        free(set);
    }
    return total;
}

/*
 * Pass 2: given T (from pass 1), fill
 *   G_off[n_genomes * n_prot + 1], G_tet[|F|]: the genome-major sets (the
 *       `<p>_genomes` blobs), (genome, protein)-major CSR;
 *   Lp[NTET + 1], F_prot / F_genome[|F|]: F ordered by (tetramer, protein,
 *       genome) (the `<p>_tetras` rows, as the reference's loader orders them).
 */
int syn_fill(const syn_params* p, const int32_t* T, int64_t* Lp, int32_t* Fp, int32_t* Fg, int64_t* G_off,
             int32_t* G_tet) {
    const int32_t G = p->n_genomes, P = p->n_prot, C = n_clades_of(p);
    G_off[0] = 0;
    for (int32_t g = 0; g < G; g++)
        for (int32_t prot = 0; prot < P; prot++) {
            const int64_t k = (int64_t)g * P + prot;
            G_off[k + 1] = G_off[k] + T[(int64_t)prot * G + g];
        }
    int bad = 0;
#pragma omp parallel reduction(| : bad)
    {
        int32_t* anc = (int32_t*)malloc(sizeof(int32_t) * 600);
#pragma omp for schedule(dynamic, 1)
        for (int32_t prot = 0; prot < P; prot++) {
            int32_t cur_clade = -1, na = 0;
            for (int32_t g = 0; g < G; g++) {
                int32_t cl = clade_of(p, g) % C;
                if (cl != cur_clade) { na = ancestral(p, cl, prot, anc); cur_clade = cl; }
                int32_t n = genome_set(p, g, prot, anc, na, G_tet + G_off[(int64_t)g * P + prot]);
                if (n != T[(int64_t)prot * G + g]) bad = 1;
            }
        }
        free(anc);
    }
    if (bad) return 1;
    const int64_t nf = G_off[(int64_t)G * P];
    memset(Lp, 0, sizeof(int64_t) * (NTET + 1));
    for (int64_t i = 0; i < nf; i++) Lp[G_tet[i] + 1]++;
    for (int32_t t = 0; t < NTET; t++) Lp[t + 1] += Lp[t];
    /* stable scatter by tetramer of the (protein, genome)-ordered stream */
    int64_t* cur = (int64_t*)malloc(sizeof(int64_t) * NTET);
    memcpy(cur, Lp, sizeof(int64_t) * NTET);
    for (int32_t prot = 0; prot < P; prot++)
        for (int32_t g = 0; g < G; g++) {
            const int64_t o = G_off[(int64_t)g * P + prot], n = G_off[(int64_t)g * P + prot + 1] - o;
            for (int64_t k = 0; k < n; k++) {
                int64_t pos = cur[G_tet[o + k]]++;
                Fp[pos] = prot;
                Fg[pos] = g;
            }
        }
    free(cur);
    return 0;
}

/* The sorted tetramer set of one (genome, protein) -- the `<p>_genomes`
 * blob -- for writing SQLite DBs.  Returns its size. */
int32_t syn_genome_set(const syn_params* p, int32_t g, int32_t prot, int32_t* out) {
    int32_t anc[600];
    int32_t C = n_clades_of(p);
    int32_t na = ancestral(p, clade_of(p, g) % C, prot, anc);
    return genome_set(p, g, prot, anc, na, out);
}

/*
 * QT join of two F arrays (both ordered by (tetramer, protein, genome)), as
 * the reference's query-vs-target loader builds it (scp_db.hpp:450-528): for
 * every (tetramer, protein) block present in BOTH, the target genomes then
 * the query genomes offset by n_tgt.  Lp_out[NTET + 1]; Fp_out / Fg_out may
 * be NULL (count only).  Returns |F_out|.
 */
int64_t syn_qt_merge(const int64_t* Lpt, const int32_t* Fpt, const int32_t* Fgt, const int64_t* Lpq,
                     const int32_t* Fpq, const int32_t* Fgq, int32_t n_tgt, int64_t* Lp_out, int32_t* Fp_out,
                     int32_t* Fg_out) {
    int64_t o = 0;
    Lp_out[0] = 0;
    for (int32_t t = 0; t < NTET; t++) {
        int64_t i = Lpt[t], ie = Lpt[t + 1], j = Lpq[t], je = Lpq[t + 1];
        while (i < ie && j < je) {
            const int32_t pt = Fpt[i], pq = Fpq[j];
            int64_t i2 = i, j2 = j;
            while (i2 < ie && Fpt[i2] == pt) i2++;
            while (j2 < je && Fpq[j2] == pq) j2++;
            if (pt == pq) {
                if (Fp_out) {
                    for (int64_t k = i; k < i2; k++, o++) { Fp_out[o] = pt; Fg_out[o] = Fgt[k]; }
                    for (int64_t k = j; k < j2; k++, o++) { Fp_out[o] = pq; Fg_out[o] = Fgq[k] + n_tgt; }
                } else {
                    o += (i2 - i) + (j2 - j);
                }
                i = i2;
                j = j2;
            } else if (pt < pq) {
                i = i2;
            } else {
                j = j2;
            }
        }
        Lp_out[t + 1] = o;
    }
    return o;
}
