/*
 * pfaai_hip.h -- C ABI of libpfaai_hip.so, the MI355X-native all-pairs
 * Average Jaccard Index (AJI) engine (HIP, gfx950).
 *
 * This is the drop-in boundary for ParFastAAI's hot path.  The reference has
 * no FFI: its boundary is a header-only C++ template contract
 *   producer  DataStructInterface   include/pfaai/interface.hpp:200-328
 *   consumer  ParFAAIImpl           include/pfaai/algorithm_impl.hpp:38-357
 * and every entry point below replaces one piece of that contract (cited per
 * function).  Plain C types only: pointers, sizes, int codes.  The C++
 * adapter with the ParFAAIImpl surface (run/computeJAC/computeAJI/getJAC/
 * getAJI) is include/pfaai_hip.hpp; the Python mirror is parfastaai_amd/.
 *
 * Conventions
 *   - return 0 on success; 1..3 are the reference's PFAAI_ERROR_CODE values
 *     (interface.hpp:39-44), 4..7 are new (HIP runtime, device OOM, RCCL,
 *     invalid argument).  pfaai_last_error() gives a message.  The names
 *     carry a PFAAI_RC_ prefix so that this header can be included next to
 *     the reference's interface.hpp, whose enum PFAAI_ERROR_CODE already
 *     defines PFAAI_OK / PFAAI_ERR_SQLITE_DB / _SQLITE_MEM_ALLOC / _CONSTRUCT
 *     with the same values.
 *   - no C++ exception crosses the ABI (allocation failures -> PFAAI_RC_OOM).
 *   - host inputs are borrowed for the duration of the call; device buffers
 *     are owned by the context; outputs are caller-owned.
 *   - one host thread drives one context; a context owns one device (a
 *     pfaai_group owns several, with an RCCL communicator over them).
 */
#ifndef PFAAI_HIP_H
#define PFAAI_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PFAAI_ABI_VERSION 6 /* 4: F or G built on the device at load, pfaai_run_info,
                                 PFAAI_RC_* names, dense row matrices (pfaai_stream_matrix);
                                 5: pfaai_load_rows, pfaai_run_walk, the multi-device
                                 group with its RCCL communicator (pfaai_group_*);
                                 6: pfaai_group_create_flags (PFAAI_GROUP_PEER_GATHER) */
#define PFAAI_NTETRAMERS 160000 /* 20^4, interface.hpp:233 */

/* Error codes: 0..3 have PFAAI_ERROR_CODE's values (interface.hpp:39-44). */
enum {
    PFAAI_RC_OK = 0,
    PFAAI_RC_SQLITE_DB = 1,
    PFAAI_RC_SQLITE_MEM_ALLOC = 2,
    PFAAI_RC_CONSTRUCT = 3,
    PFAAI_RC_HIP = 4,
    PFAAI_RC_OOM = 5,
    PFAAI_RC_RCCL = 6,
    PFAAI_RC_INVALID = 7
};

/* Modes: which genome pairs are valid and how they index the JAC array.
 *   ALL  = ParFAAIData        (ds_impl.hpp:38-151)   pairs a<b
 *   QSUB = ParFAAIQSubData    (ds_impl.hpp:158-337)  -q query subset
 *   QT   = ParFAAIQryTgtData  (ds_impl.hpp:343-490)  -r query DB vs target DB */
enum { PFAAI_MODE_ALL = 0, PFAAI_MODE_QSUB = 1, PFAAI_MODE_QT = 2 };

/* Run flags */
#define PFAAI_FLAG_REF_COMPAT 1u /* reproduce reference quirks */
#define PFAAI_FLAG_EMIT_JAC 2u   /* also write the JAC S (f64) and N (i32) */
#define PFAAI_FLAG_KEEP_RUNS 4u  /* reuse the run table an earlier pfaai_run on this
                                    load built (same stream or ordered after it):
                                    row tiles / pipelined shards pay k_blk once */
#define PFAAI_FLAG_FULL_ROWS 8u  /* pfaai_run writes the rows of printOutput's dense
                                    matrix (main.cpp:143-154) instead of JAC pairs:
                                    out[row * n_cols + col], n_cols = n_ids (ALL,
                                    QSUB: every genome) or n_tgt (QT), the mirror
                                    half included, the diagonal left unwritten */

/* Row kernels (pfaai_run_info): k_rows_pl (genome-major walk), its 512-
 * thread form, the fused k_rows (G lists > 1024 entries), the work-list
 * k_rows (no genome-major view could be formed), and k_rows_v2 (wave-local
 * line tasks, every load one protein ahead). */
enum { PFAAI_ROWS_PL = 0, PFAAI_ROWS_PL512 = 1, PFAAI_ROWS_FUSED = 2, PFAAI_ROWS_WORKLIST = 3, PFAAI_ROWS_V2 = 4 };

typedef struct pfaai_ctx pfaai_ctx;

/*
 * The data-structure view the reference's DataStructInterface exposes
 * (refLp/refF/refT, interface.hpp:246-250) plus the mode's index maps
 * (isQryGenome/isValidPair/genomePairToIndex, interface.hpp:276-293).
 * F is ordered by (tetramer, protein, genome): block t = [Lp[t], Lp[t+1]).
 */
typedef struct {
    int32_t mode;          /* PFAAI_MODE_* */
    int32_t n_ids;         /* genome ids used in F (QT: n_tgt + n_qry; query ids offset by n_tgt) */
    int32_t n_prot;        /* P */
    int32_t t_cols;        /* columns of T (T is P x t_cols, row-major) */
    int32_t n_qry;         /* QSUB: |query list|; QT: genomes of the query DB */
    int32_t n_tgt;         /* QSUB: n_ids - n_qry; QT: genomes of the target DB; ALL: unused */
    int64_t n_f;           /* |F| (<= 2^32 - 64); ignored when F is built from G */
    const int64_t* Lp;     /* [PFAAI_NTETRAMERS + 1] exclusive prefix of Lc, Lp[160000] = n_f */
    const int32_t* F_prot; /* [n_f] F[i].first  (protein index) */
    const int32_t* F_genome; /* [n_f] F[i].second (genome id)
                              * Lp, F_prot and F_genome may all be NULL when
                              * G_off / G_tet are given: F is then built on the
                              * device from G (stable radix sort by tetramer *
                              * n_prot + protein, ds_helper.hpp:126-162). */
    const int32_t* T;      /* [n_prot * t_cols] T(p, g) tetramer counts */
    const uint8_t* is_q;   /* [n_ids] QSUB/QT: 1 for query genomes (NULL for ALL) */
    const int32_t* q_index; /* [n_ids] QSUB: position of the genome in the query file, -1 otherwise */
    const int32_t* t_rank; /* [n_ids] QSUB: rank among the non-query genomes, -1 otherwise */
    /* Optional genome-major view (NULL if absent): the `<p>_genomes` blobs of
     * the SCP database (scp_db.hpp:219-262 reads only their lengths), as a
     * (genome, protein)-major CSR: tetramers of genome g, protein p are
     * G_tet[G_off[g*n_prot+p] .. G_off[g*n_prot+p+1]), ascending.  With it
     * the row kernel walks genome g's tetramer list directly and looks each
     * (protein, tetramer) run of F up in a dense run table built once per
     * run (no sort, no per-step work lists).  When G is NULL, pfaai_load
     * builds it on the device from F (stable radix sort of the F entries by
     * genome * n_prot + protein), so F-only callers -- the reference's own
     * DataStructInterface classes -- run the same kernels.  When both F and
     * G are given, G must hold every membership of F, and may hold more only
     * where F has no run (t, p) at all -- the -r case: both DBs' lists vs
     * the inner-joined F (checked on the device).  Lists are strictly
     * ascending sets of tetramer ids. */
    const int64_t* G_off;  /* [n_ids * n_prot + 1] */
    const int32_t* G_tet;  /* [G_off[n_ids * n_prot]] */
} pfaai_problem;

/* ---- lifecycle ---------------------------------------------------------- */
int pfaai_version(void);
int pfaai_create(pfaai_ctx** ctx, int device_id);
int pfaai_destroy(pfaai_ctx* ctx);
const char* pfaai_last_error(const pfaai_ctx* ctx);

/* Copy a problem to the device and keep it resident (replaces the reference
 * handing ParFAAIImpl const refs to Lc/Lp/F/T, algorithm_impl.hpp:50-55,
 * 75-79).  Replaces any previously loaded problem. */
int pfaai_load(pfaai_ctx* ctx, const pfaai_problem* prob);

/* pfaai_load for a context that will run only output rows [row_begin,
 * row_end) -- one rank of a row-block partition (the reference's
 * distributeGenomePairs, algorithm_impl.hpp:100-120).  The whole problem is
 * loaded; the per-entry walk data of all-vs-all rows (G_pos, G_end) is built
 * for those rows' genomes only, so a rank's load sorts and writes ~1/N of it.
 * Rows outside the block: when the caller hands over both F and G, the load
 * checks G against F for the block's genomes only, so pfaai_run /
 * pfaai_compute / pfaai_compute_rows / pfaai_stream refuse rows outside it
 * (PFAAI_RC_INVALID); with G built on the device from F (or F from G) they
 * run through the run table (correct, slower).  Other modes: as pfaai_load. */
int pfaai_load_rows(pfaai_ctx* ctx, const pfaai_problem* prob, int64_t row_begin, int64_t row_end);

/* F construction on the device (replaces DataStructHelper::constructLc /
 * constructF / constructT, ds_helper.hpp:46-162, and the SQL UNION ALL +
 * ORDER BY of SQLiteSCPDataBase::proteinSetGPPairs, scp_db.hpp:161-216).
 * Input: n (protein, genome, tetramer) triples -- the `<p>_genomes` blobs
 * expanded -- where each protein's triples come in non-decreasing genome
 * order (any (genome, protein)- or (protein, genome)-major walk of the blobs).
 * A stable LSD radix sort (8-bit digits) by tetramer * n_prot + protein
 * yields F ordered by (tetramer, protein, genome).  Outputs (host, caller-
 * allocated): Lc[160000], Lp[160001], F_prot / F_genome[n], and optionally
 * T[n_prot * n_genome] (counts per (protein, genome); NULL to skip).  Does
 * not change the loaded problem. */
int pfaai_build_f(pfaai_ctx* ctx, const int32_t* prot, const int32_t* genome, const int32_t* tetra,
                  int64_t n, int32_t n_prot, int32_t n_genome, int32_t* Lc_out, int64_t* Lp_out,
                  int32_t* F_prot_out, int32_t* F_genome_out, int32_t* T_out);

/* Number of output rows (ALL: n_ids; QSUB/QT: n_qry) and of JAC pairs
 * (nGenomePairs: ds_impl.hpp:78-80, 244-249, 406). */
int pfaai_shape(const pfaai_ctx* ctx, int64_t* n_rows, int64_t* n_pairs);

/* JAC-index span [first, first+count) written by rows [row_begin, row_end).
 * Rows map to contiguous spans in ALL and QT; in QSUB each row has two
 * segments (cross block, triangle block) and the span is their hull. */
int pfaai_row_span(const pfaai_ctx* ctx, int64_t row_begin, int64_t row_end,
                   int64_t* first, int64_t* count);

/*
 * Device-resident hot path for output rows [row_begin, row_end):
 *   E construction (ds_helper.hpp:206-421) -> per-(row,protein) work lists,
 *   pair-expansion scatter of intersection counts (no E, no sort),
 *   Jaccard normalisation + protein-ordered fp64 S/N reduction
 *   (algorithm_impl.hpp:222-306), AJI = S/N (algorithm_impl.hpp:309-322).
 * d_aji / d_S / d_N are DEVICE pointers to arrays indexed by the full JAC
 * index (length n_pairs); only the rows' entries are written.  d_aji may be
 * NULL (then only S/N), d_S/d_N are required with PFAAI_FLAG_EMIT_JAC.
 * stream: a hipStream_t (NULL = the context's own stream).  Asynchronous.
 */
int pfaai_run(pfaai_ctx* ctx, int64_t row_begin, int64_t row_end, uint32_t flags,
              double* d_aji, double* d_S, int32_t* d_N, void* stream);

/* Synchronous convenience: all rows, results copied into HOST arrays of
 * length n_pairs (any may be NULL).  The ParFAAIImpl::run() equivalent
 * (algorithm_impl.hpp:325-329). */
int pfaai_compute(pfaai_ctx* ctx, uint32_t flags, double* h_aji, double* h_S,
                  int32_t* h_N);

/*
 * Output-tile streaming (the output too large
 * to hold whole).  Rows [row_begin, row_end) are cut into row tiles of at
 * most tile_pairs JAC entries (at least one row each); every tile is
 * computed on the device, copied to pinned host memory while the next tile
 * computes, and handed to sink() in row order on the calling thread:
 *   sink(user, tile_row_begin, tile_row_end, first, count, aji, S, N)
 * with aji[i] (and, under PFAAI_FLAG_EMIT_JAC, S[i], N[i]) the pair at JAC
 * index first + i (ds_impl.hpp:83-86, 411-413).  The host arrays are valid
 * only during the sink call.  A non-zero sink return stops the stream and
 * is returned.  ALL and QT modes (contiguous row spans).  Synchronous; the
 * device holds two tiles, never the whole output.
 */
typedef int (*pfaai_sink_fn)(void* user, int64_t row_begin, int64_t row_end, int64_t first,
                             int64_t count, const double* aji, const double* S, const int32_t* N);
int pfaai_stream(pfaai_ctx* ctx, int64_t row_begin, int64_t row_end, int64_t tile_pairs,
                 uint32_t flags, pfaai_sink_fn sink, void* user);
/*
 * Dense output rows (the streamed CSV of config C5): rows [row_begin,
 * row_end) of printOutput's nQ x nT AJI matrix (main.cpp:133-175) -- ALL:
 * N x N with the mirror half and a zero diagonal; QSUB: query rows in
 * query-file order x all genomes, query-query cells mirrored; QT: queries x
 * targets -- in tiles of at most tile_rows rows.  Every row is computed whole
 * (AJI(A, B) and AJI(B, A) are bit-identical: the same counts, denominators
 * and protein order), so no tile depends on another; tile k computes while
 * tile k-1 is copied to pinned host memory, and
 *   sink(user, tile_row_begin, tile_row_end, n_cols, block)
 * gets block[(r - tile_row_begin) * n_cols + col] in row order on the calling
 * thread (valid during the call).  A non-zero sink return stops the stream
 * and is returned.  |E| of the tiles (pfaai_stream_events) counts every
 * (p, A, B) of the full rows, i.e. both orientations of a pair.
 */
typedef int (*pfaai_matrix_sink_fn)(void* user, int64_t row_begin, int64_t row_end, int64_t n_cols,
                                    const double* block);
int pfaai_stream_matrix(pfaai_ctx* ctx, int64_t row_begin, int64_t row_end, int64_t tile_rows, uint32_t flags,
                        pfaai_matrix_sink_fn sink, void* user);
/* |E| summed over the tiles of the last pfaai_stream / pfaai_stream_matrix. */
int pfaai_stream_events(const pfaai_ctx* ctx, int64_t* n_events);

/* ParFAAIImpl::run() (algorithm_impl.hpp:325-329) for a block of rows:
 * rows [row_begin, row_end) into HOST arrays of length n_pairs indexed by
 * the JAC index (only the rows' entries are written; any may be NULL).
 * Synchronous.  ALL and QT: disjoint row blocks have disjoint spans, so one
 * host thread per context (one context per device) fills a shared host
 * array for a multi-GPU run without a gather (CLI --devices; the C++
 * adapter's multi-device constructor).  QSUB (round 6): a block's cross
 * cells are its contiguous span; its query-query cells (placed by query file
 * index, owned by the pair's smaller genome id -- not contiguous) are
 * merged into the triangle cell by cell, so the blocks of a split fill
 * disjoint cells of one output. */
int pfaai_compute_rows(pfaai_ctx* ctx, int64_t row_begin, int64_t row_end, uint32_t flags,
                       double* h_aji, double* h_S, int32_t* h_N);

/* ---- multi-device group (pfaai_create over a device list, the
 * RCCL communicator inside) -------------------------------------------------
 * The device-side counterpart of distributeGenomePairs (algorithm_impl.hpp:
 * 100-120) in one process: one context per device, one RCCL communicator
 * over them (ncclCommInitAll), one stream per device; one host thread drives
 * the group.  pfaai_group_load loads the caller's host arrays on every
 * device concurrently (one host copy feeds all of them) and builds each
 * device's walk data for its own row block only (pfaai_load_rows); blocks
 * by the row-cost model of pfaai::split_rows (pfaai_hip.hpp) for ALL, equal
 * rows for QT; a QSUB problem runs on the first device alone (its rows'
 * JAC spans are not contiguous).  pfaai_group_run computes every block on
 * its device and gathers them into the caller's arrays on the FIRST device
 * (device_ids[0]; length n_pairs, JAC index order) by grouped ncclSend /
 * ncclRecv over xGMI; synchronous.  d_S / d_N are required with
 * PFAAI_FLAG_EMIT_JAC; PFAAI_FLAG_FULL_ROWS is not supported here.
 * Errors: PFAAI_RC_INVALID for a bad or repeated device id, PFAAI_RC_RCCL
 * for a communicator failure; pfaai_group_last_error gives the message.
 * Row blocks: pfaai::split_rows with the first device's CU count, i.e. the
 * cuts of bench.py's ranks (shard.split_rows(..., cus=)).
 * pfaai_group_create_flags with PFAAI_GROUP_PEER_GATHER: no communicator;
 * pfaai_group_run gathers each block by hipMemcpyPeerAsync on the first
 * device's stream, after an event of the block's run, and a device id may
 * repeat (several members on one GPU: the n > 1 path -- rank loads, block
 * buffers, the gather's offsets -- on a one-GPU machine). */
#define PFAAI_GROUP_PEER_GATHER 1u
typedef struct pfaai_group pfaai_group;
int pfaai_group_create(pfaai_group** group, const int* device_ids, int n_devices);
int pfaai_group_create_flags(pfaai_group** group, const int* device_ids, int n_devices, uint32_t flags);
int pfaai_group_destroy(pfaai_group* group);
const char* pfaai_group_last_error(const pfaai_group* group);
int pfaai_group_size(const pfaai_group* group, int* n_devices);
/* the context of device_ids[i] (stats, timing, row spans); owned by the group */
pfaai_ctx* pfaai_group_ctx(pfaai_group* group, int i);
int pfaai_group_load(pfaai_group* group, const pfaai_problem* prob);
/* the row blocks of the loaded problem: cuts[0] = 0 .. cuts[n_devices] = rows */
int pfaai_group_blocks(const pfaai_group* group, int64_t* cuts);
int pfaai_group_run(pfaai_group* group, uint32_t flags, double* d_aji, double* d_S, int32_t* d_N);

/* Times (ms) of the last pfaai_load: host-side checks and H2D copies (wall),
 * and the device span of the F / G build (or G-covers-F check), HIP events
 * on the context stream from its first kernel to its last. */
int pfaai_load_timing(const pfaai_ctx* ctx, double* ms_checks, double* ms_upload, double* ms_device);

/* Which orientation the last pfaai_load built on the device (the
 * replacement of the reference's F construction, ds_helper.hpp:126-162 /
 * scp_db.hpp:161-216, and of its G read, scp_db.hpp:219-262):
 *   AS_GIVEN    nothing built (both given, G a superset of F: QT lists of
 *               both DBs, checked by search)
 *   G_CHECKED   both given: one sort of F by (genome, protein) proved G to
 *               be F's transpose and produced G_pos
 *   G_FROM_F    F only: G by the same sort (list bounds from T, verified)
 *   F_FROM_G    G only: F by a two-pass sort of the protein-major G entries
 *               by tetramer
 *   LEGACY      the general 8-bit LSD radix sort (inputs whose record fields
 *               do not fit the transposition sort's 64-bit records) */
enum { PFAAI_LOAD_AS_GIVEN = 0, PFAAI_LOAD_G_CHECKED = 1, PFAAI_LOAD_G_FROM_F = 2, PFAAI_LOAD_F_FROM_G = 3,
       PFAAI_LOAD_LEGACY = 4 };
int pfaai_load_info(const pfaai_ctx* ctx, int32_t* path);

/* Which row kernel the last pfaai_run launched (PFAAI_ROWS_*) and whether it
 * ran by absolute column windows (rows wider than one kernel chunk). */
int pfaai_run_info(const pfaai_ctx* ctx, int32_t* rows_kernel, int32_t* column_windows);

/* How the last pfaai_run's k_rows_pl launches walked the F runs of each row
 * genome's G entries (the reference's E construction for that row,
 * ds_helper.hpp:270-357, without E):
 *   SPLITTERS  run-table lookups, members pruned to the column chunk by the
 *              table's line splitters (query rows, column windows, F only)
 *   GPOS       all-vs-all: from the row genome's own F position + 1 (G_pos)
 *              to its run end (G_end), both built at load -- the
 *              benchmarked form; no run table in the step
 *   SPANS      column windows whose sub-runs hold only the row's partners
 *              (all-vs-all windows past the row's first column, every
 *              query-vs-target window): the window table's sub-run walked
 *              whole, one launch over (row, window); the all-vs-all rows'
 *              diagonal windows by the table + splitters
 * and whether the narrow rows (<= 2 047 columns) ran as a 512-thread launch
 * on the context's side stream beside the wide rows.  -1: no k_rows_pl ran. */
enum { PFAAI_WALK_NONE = -1, PFAAI_WALK_SPLITTERS = 0, PFAAI_WALK_GPOS = 3, PFAAI_WALK_SPANS = 4 };
int pfaai_run_walk(const pfaai_ctx* ctx, int32_t* walk, int32_t* narrow_launch);

/* All-vs-all, genome-major loads: make rows [0, n) of later pfaai_runs the
 * genomes of `genomes` (strictly ascending ids; the others follow, but rows
 * >= n are refused while the list is set), so one launch covers any subset
 * of output rows -- e.g. a rank's block-cyclic share of the matrix (row
 * groups dealt round robin, so every rank holds the whole matrix's mix of
 * wide and narrow rows; distributeGenomePairs, algorithm_impl.hpp:100-120,
 * deals contiguous pair ranges instead).  Outputs stay at the reference's
 * JAC index, so a run writes its rows' entries into arrays of n_pairs.
 * Only pfaai_run uses the list (the span APIs -- pfaai_row_span,
 * pfaai_compute*, pfaai_stream* -- refuse it).  genomes == NULL or n == 0:
 * back to rows = genomes in id order.  Synchronises the device. */
int pfaai_set_row_order(pfaai_ctx* ctx, const int32_t* genomes, int64_t n);

/* |E| of the last run, counted by the scatter kernel (equals the reference's
 * countTetramerTuples total over the run's rows, ds_helper.hpp:206-265), and
 * device times (ms) of its two phases: work-list build, row kernel.
 * Valid after the run's stream has been synchronised. */
int pfaai_last_stats(pfaai_ctx* ctx, int64_t* n_events, float* ms_build,
                     float* ms_rows);

/* Accumulated device times of every pfaai_run since the last reset: number
 * of runs and the summed ms of the work-list build and of the row kernel
 * (HIP events on the run's stream).  Synchronises on those events; reset != 0
 * starts a new accumulation window afterwards. */
int pfaai_timing(pfaai_ctx* ctx, int reset, int32_t* n_runs, double* ms_build,
                 double* ms_rows);

/* Debug materialiser for integer parity: intersection counts c(p, a, b) of
 * output row `row` for every protein, written to a HOST array
 * counts[p * n_ids + b] (int32, n_prot x n_ids).  Equals the run-lengths of
 * the reference's sorted E (ds_helper.hpp:414-418) restricted to genomeA. */
int pfaai_debug_row_counts(pfaai_ctx* ctx, int64_t row, int32_t* h_counts);

/* Self-test of the row kernels' exact small-integer division: compares
 * c / d computed by the fast paths with IEEE '/' for every 1 <= c <= c_max,
 * c <= d <= d_max on the device -- exact_div_small, and the paired form of
 * k_rows_pl's S5 (one reciprocal for two columns) with six partner
 * denominators per (c, d), both of its columns checked; *mismatches receives
 * the count (0 = every quotient bit-identical). */
int pfaai_debug_div_check(pfaai_ctx* ctx, int32_t c_max, int32_t d_max, int64_t* mismatches);

/* Diagnostics: per-stage shader-clock sums of k_rows_pl (PFAAI_PL_CLK=1,
 * all-vs-all, KW = 5): n == 0 arms (allocates + clears) the buffer; n > 0
 * copies up to n u64 = [256 workgroups][16 waves][8 stages] to the host. */
int pfaai_debug_clocks(pfaai_ctx* ctx, uint64_t* out, int64_t n);

/* Device memory helpers (so callers without a GPU framework can run the
 * device-resident path): allocate/free on the context's device, copy. */
int pfaai_device_alloc(pfaai_ctx* ctx, void** ptr, int64_t bytes);
int pfaai_device_free(pfaai_ctx* ctx, void* ptr);
int pfaai_memcpy_d2h(pfaai_ctx* ctx, void* dst, const void* src, int64_t bytes);
int pfaai_synchronize(pfaai_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* PFAAI_HIP_H */
