// scp_db.hpp -- SQLite SCP/tetramer loader for the host CLI.
//
// Same SQL, same id rules and the same resulting arrays as the reference's
// DB layer:
//   SQLiteHelper        include/pfaai/db_helper.hpp:33-219
//   SQLiteSCPDataBase   include/pfaai/scp_db.hpp:59-263
//   QTSQLiteSCPDataBase include/pfaai/scp_db.hpp:267-590
// Two ingest paths, both parallel over proteins (one read-only connection
// per OpenMP thread):
//   load_*_g  (the default, north_star's device F build): every protein's
//             `<p>_genomes` table -- the blobs the reference reads only the
//             lengths of for T (scp_db.hpp:219-262) -- becomes the genome-
//             major lists G (CSR over (genome, protein)); F is then built on
//             the device by pfaai_load (a stable radix sort), never on the
//             host.  No UNION ALL, no ORDER BY.
//   load_*    (--dump-arrays, and the fallback when a `<p>_genomes` blob is
//             not a set): every protein's `<p>_tetras` table, F assembled by a
//             stable counting sort on the tetramer id -- the reference's
//             (tetramer, protein, blob order) layout of scp_db.hpp:161-216.
#pragma once
#include <omp.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <random>
#include <cstring>
#include <string>
#include <vector>

#include "sqlite_min.h"

namespace pfaai_host {

constexpr int kNTetramers = 160000;

struct DPair {
    int32_t first, second;
};

struct DMatrix {
    std::size_t nrows = 0, ncols = 0;
    std::vector<int32_t> data;
    DMatrix() = default;
    DMatrix(std::size_t r, std::size_t c) : nrows(r), ncols(c), data(r * c, 0) {}
    int32_t& operator()(std::size_t i, std::size_t j) { return data[i * ncols + j]; }
    int32_t operator()(std::size_t i, std::size_t j) const { return data[i * ncols + j]; }
    std::size_t rows() const { return nrows; }
    std::size_t cols() const { return ncols; }
};

struct DBMetaData {
    std::vector<std::string> proteinSet, genomeSet, qyGenomeSet;
};

struct LoadedArrays {
    std::vector<int32_t> Lc;  // F path only
    std::vector<DPair> F;     // F path only
    DMatrix T;
    std::vector<int64_t> G_off;  // G path only: [n_ids * P + 1], list (g, p) at g * P + p
    std::vector<int32_t> G_tet;  // G path only: ascending tetramers of each list
};

class Conn {
  public:
    explicit Conn(const std::string& path) {
        rc = sqlite3_open_v2(path.c_str(), &db, SQLITE_OPEN_READONLY, nullptr);
    }
    ~Conn() {
        if (db) sqlite3_close(db);
    }
    Conn(const Conn&) = delete;
    Conn& operator=(const Conn&) = delete;
    bool ok() const { return rc == SQLITE_OK && db; }
    std::string error() const { return db ? sqlite3_errmsg(db) : sqlite3_errstr(rc); }
    int exec(const std::string& sql) { return sqlite3_exec(db, sql.c_str(), nullptr, nullptr, nullptr); }

    // run a query, call fn(stmt) per row; returns SQLITE_OK or the error code
    template <typename Fn>
    int each(const std::string& sql, Fn&& fn) {
        sqlite3_stmt* st = nullptr;
        int e = sqlite3_prepare_v2(db, sql.c_str(), -1, &st, nullptr);
        if (e != SQLITE_OK) {
            last_sql = sql;
            return e;
        }
        while ((e = sqlite3_step(st)) == SQLITE_ROW) fn(st);
        sqlite3_finalize(st);
        return e == SQLITE_DONE ? SQLITE_OK : e;
    }

    sqlite3* db = nullptr;
    int rc = 0;
    std::string last_sql;
};

inline std::vector<std::string> column_strings(Conn& c, const std::string& sql, int* err) {
    std::vector<std::string> out;
    *err = c.each(sql, [&](sqlite3_stmt* st) {
        const unsigned char* s = sqlite3_column_text(st, 0);
        out.emplace_back(s ? reinterpret_cast<const char*>(s) : "");
    });
    return out;
}

// per-protein (tetramer, genome list) rows, in table order
struct ProteinRows {
    std::vector<int32_t> tet, cnt, genomes;
    int err = SQLITE_OK;
};

// Assemble Lc and F (tetramer, protein, blob order) from per-protein rows.
inline void assemble_f(const std::vector<ProteinRows>& rows, LoadedArrays& out) {
    out.Lc.assign(kNTetramers, 0);
    for (const auto& r : rows)
        for (std::size_t k = 0; k < r.tet.size(); ++k) out.Lc[r.tet[k]] += r.cnt[k];
    std::vector<int64_t> cur(kNTetramers + 1, 0);
    for (int t = 0; t < kNTetramers; ++t) cur[t + 1] = cur[t] + out.Lc[t];
    out.F.resize(cur[kNTetramers]);
    // protein-major pass: within a tetramer, proteins arrive in index order
    for (std::size_t p = 0; p < rows.size(); ++p) {
        const auto& r = rows[p];
        std::size_t off = 0;
        for (std::size_t k = 0; k < r.tet.size(); ++k) {
            int64_t& pos = cur[r.tet[k]];
            for (int32_t j = 0; j < r.cnt[k]; ++j) out.F[pos++] = DPair{(int32_t)p, r.genomes[off + j]};
            off += r.cnt[k];
        }
    }
}

// SQLiteSCPDataBase: one DB, genome ids = genome_metadata order.
inline int load_single(const std::string& path, DBMetaData& meta, LoadedArrays& out, std::string& err) {
    Conn c(path);
    if (!c.ok()) {
        err = "Error in opening " + path + ": " + c.error();
        return 1;  // PFAAI_RC_SQLITE_DB
    }
    int e = 0;
    meta.proteinSet = column_strings(c, "SELECT DISTINCT scp_acc FROM scp_data", &e);  // db_helper.hpp:195-215
    if (e == SQLITE_OK) meta.genomeSet = column_strings(c, "SELECT genome_name FROM genome_metadata", &e);
    if (e != SQLITE_OK) {
        err = "Error in reading metadata of " + path + ": " + c.error();
        return 1;
    }
    const int P = (int)meta.proteinSet.size();
    const int G = (int)meta.genomeSet.size();
    std::vector<ProteinRows> rows(P);
    out.T = DMatrix(P, G);
    int bad = 0;
#pragma omp parallel
    {
        Conn tc(path);  // one read-only connection per thread
#pragma omp for schedule(dynamic, 1)
        for (int p = 0; p < P; ++p) {
            if (!tc.ok()) {
                rows[p].err = 1;
                continue;
            }
            auto& r = rows[p];
            const std::string& acc = meta.proteinSet[p];
            r.err = tc.each("SELECT tetramer, genomes FROM `" + acc + "_tetras`", [&](sqlite3_stmt* st) {
                const int32_t t = sqlite3_column_int(st, 0);
                const int nb = sqlite3_column_bytes(st, 1) / 4;
                const auto* g = static_cast<const int32_t*>(sqlite3_column_blob(st, 1));
                r.tet.push_back(t);
                r.cnt.push_back(nb);
                r.genomes.insert(r.genomes.end(), g, g + nb);
            });
            if (r.err == SQLITE_OK)  // proteinTetramerCounts (scp_db.hpp:219-262)
                r.err = tc.each("SELECT genome_id, length(tetramers) FROM `" + acc + "_genomes`",
                                [&](sqlite3_stmt* st) {
                                    const int gid = sqlite3_column_int(st, 0);
                                    if (gid >= 0 && gid < G) out.T(p, gid) = sqlite3_column_int(st, 1) / 4;
                                });
            for (int32_t t : r.tet)
                if (t < 0 || t >= kNTetramers) r.err = 1;
            for (int32_t g : r.genomes)
                if (g < 0 || g >= G) r.err = 1;
        }
    }
    for (int p = 0; p < P; ++p)
        if (rows[p].err) {
            err = "Error in reading tables of protein " + meta.proteinSet[p] + " from " + path;
            bad = 1;
            break;
        }
    if (bad) return 3;  // PFAAI_RC_CONSTRUCT
    assemble_f(rows, out);
    return 0;
}

// QTSQLiteSCPDataBase: target DB `main` + ATTACHed query DB `QueryDB`;
// shared proteins only, tetramers present in both (inner join), query
// genome ids offset by the number of target genomes.
inline int load_qt(const std::string& tgt, const std::string& qry, DBMetaData& meta, LoadedArrays& out,
                   std::string& err) {
    Conn c(tgt);
    if (!c.ok()) {
        err = "Error in opening " + tgt + ": " + c.error();
        return 1;
    }
    if (c.exec("ATTACH DATABASE '" + qry + "' as QueryDB ;") != SQLITE_OK) {
        err = "Error in attaching query database : " + qry + ": " + c.error();
        return 1;
    }
    int e = 0;
    meta.proteinSet = column_strings(c,
                                     "SELECT DISTINCT target_table.scp_acc \n"
                                     "  FROM `main`.scp_data as target_table, `QueryDB`.scp_data as query_table \n"
                                     "  WHERE target_table.scp_acc = query_table.scp_acc;",
                                     &e);  // db_helper.hpp:109-166
    if (e == SQLITE_OK) meta.genomeSet = column_strings(c, "SELECT genome_name FROM `main`.genome_metadata", &e);
    if (e == SQLITE_OK) meta.qyGenomeSet = column_strings(c, "SELECT genome_name FROM `QueryDB`.genome_metadata", &e);
    if (e != SQLITE_OK) {
        err = "Error in reading metadata: " + c.error();
        return 1;
    }
    const int P = (int)meta.proteinSet.size();
    const int nT = (int)meta.genomeSet.size(), nQ = (int)meta.qyGenomeSet.size();
    std::vector<ProteinRows> rows(P);
    out.T = DMatrix(P, nT + nQ);
#pragma omp parallel
    {
        Conn tc(tgt);
        bool ok = tc.ok() && tc.exec("ATTACH DATABASE '" + qry + "' as QueryDB ;") == SQLITE_OK;
#pragma omp for schedule(dynamic, 1)
        for (int p = 0; p < P; ++p) {
            auto& r = rows[p];
            if (!ok) {
                r.err = 1;
                continue;
            }
            const std::string& acc = meta.proteinSet[p];
            r.err = tc.each("SELECT target_table.tetramer, target_table.genomes, query_table.genomes "
                            "FROM main.`" + acc + "_tetras` as target_table, QueryDB.`" + acc +
                                "_tetras` as query_table WHERE target_table.tetramer = query_table.tetramer",
                            [&](sqlite3_stmt* st) {
                                const int32_t t = sqlite3_column_int(st, 0);
                                const int nt = sqlite3_column_bytes(st, 1) / 4, nq = sqlite3_column_bytes(st, 2) / 4;
                                const auto* gt = static_cast<const int32_t*>(sqlite3_column_blob(st, 1));
                                const auto* gq = static_cast<const int32_t*>(sqlite3_column_blob(st, 2));
                                r.tet.push_back(t);
                                r.cnt.push_back(nt + nq);
                                r.genomes.insert(r.genomes.end(), gt, gt + nt);
                                for (int j = 0; j < nq; ++j) r.genomes.push_back(nT + gq[j]);
                            });
            if (r.err == SQLITE_OK)
                r.err = tc.each("SELECT genome_id, length(tetramers) FROM main.`" + acc + "_genomes`",
                                [&](sqlite3_stmt* st) {
                                    const int gid = sqlite3_column_int(st, 0);
                                    if (gid >= 0 && gid < nT) out.T(p, gid) += sqlite3_column_int(st, 1) / 4;
                                });
            if (r.err == SQLITE_OK)
                r.err = tc.each("SELECT genome_id, length(tetramers) FROM QueryDB.`" + acc + "_genomes`",
                                [&](sqlite3_stmt* st) {
                                    const int gid = sqlite3_column_int(st, 0);
                                    if (gid >= 0 && gid < nQ) out.T(p, nT + gid) += sqlite3_column_int(st, 1) / 4;
                                });
            for (int32_t g : r.genomes)
                if (g < 0 || g >= nT + nQ) r.err = 1;
        }
    }
    for (int p = 0; p < P; ++p)
        if (rows[p].err) {
            err = "Error in reading tables of protein " + meta.proteinSet[p];
            return 3;
        }
    assemble_f(rows, out);
    return 0;
}


// ---------------------------------------------------------------------------
// G path: `<p>_genomes` (genome_id INTEGER PK, tetramers BLOB int32[]).
// ---------------------------------------------------------------------------
struct ProteinLists {  // one protein's lists, in table order
    std::vector<int32_t> gid, len, tet;
    int err = SQLITE_OK;
};

// Read `<schema>.<acc>_genomes` into r, genome ids offset by id_base and
// checked against [0, n_ids_db); T(p, id_base + gid) = list length.
inline int read_genome_lists(Conn& tc, const std::string& schema, const std::string& acc, int32_t id_base,
                             int32_t n_ids_db, ProteinLists& r) {
    return tc.each("SELECT genome_id, tetramers FROM " + schema + "`" + acc + "_genomes`", [&](sqlite3_stmt* st) {
        const int gid = sqlite3_column_int(st, 0);
        const int nb = sqlite3_column_bytes(st, 1) / 4;
        const auto* t = static_cast<const int32_t*>(sqlite3_column_blob(st, 1));
        if (gid < 0 || gid >= n_ids_db) {
            r.err = 1;
            return;
        }
        r.gid.push_back(id_base + gid);
        r.len.push_back(nb);
        r.tet.resize(r.tet.size() + nb);
        if (nb) std::memcpy(r.tet.data() + r.tet.size() - nb, t, (std::size_t)nb * 4);  // (unaligned blob)
    });
}


// Exact consistency of the two orientations.  The reference builds F from
// `<p>_tetras` (scp_db.hpp:161-216) and reads only the lengths of the
// `<p>_genomes` blobs (scp_db.hpp:219-262); the G path builds everything
// from `<p>_genomes`.  The two give the same output exactly when, per
// protein, the multisets of memberships (genome, tetramer) of the two tables
// are equal.  Both sides are folded into order-independent keyed sums of a
// 64-bit mix of the injective code g << 32 | (p * 160000 + t), in two lanes
// with independent per-run random seeds and different mixers (a difference
// has to cancel in both lanes at once; ~2^-128 per protein is a heuristic
// figure, not a proof), plus the membership counts.  A protein
// whose two tables disagree sends the whole DB through the `<p>_tetras`
// path, so the output is the reference's either way.
// Thread time (ns, summed over the reading threads) of the last G-path
// load: reading the `<p>_genomes` lists, and the membership check (the G
// side's sums and the `<p>_tetras` blobs read and summed) -- the CLI prints
// both beside the load's wall time (the check's host cost).
struct GLoadClock {
    std::atomic<int64_t> read_ns{0}, check_ns{0};
    std::atomic<int> threads{0};
};
inline GLoadClock& g_load_clock() {
    static GLoadClock c;
    return c;
}
inline int64_t ns_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t).count();
}

struct MemberSum {
    uint64_t n = 0, a = 0, b = 0;
    bool operator==(const MemberSum& o) const { return n == o.n && a == o.a && b == o.b; }
    bool operator!=(const MemberSum& o) const { return !(*this == o); }
};

struct MemberSeeds {
    uint64_t a, b;
    static MemberSeeds fresh() {
        std::random_device rd;
        const uint64_t t = (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
        return {((uint64_t)rd() << 32 ^ rd()) ^ t, ((uint64_t)rd() << 32 ^ rd()) ^ (t * 0x9E3779B97F4A7C15ull)};
    }
};

// One multiply per lane and two different xorshift-multiply-xorshift
// bijections for the two lanes (the device check's mixers, pfaai_sort.hpp):
// splitmix64's two multiplies per lane made the check ~40 % of the G path's
// per-thread time at C2 (34 of 90 ms; round 5)
inline uint64_t member_mix_a(uint64_t x) {
    x ^= x >> 32;
    x *= 0xD6E8FEB86659FD93ull;
    return x ^ (x >> 32);
}
inline uint64_t member_mix_b(uint64_t x) {
    x ^= x >> 29;
    x *= 0xBF58476D1CE4E5B9ull;
    return x ^ (x >> 31);
}

inline void member_add(MemberSum& m, const MemberSeeds& sd, uint32_t g, uint32_t p, uint32_t t) {
    const uint64_t key = (uint64_t)g << 32 | (uint64_t)(p * (uint32_t)kNTetramers + t);
    m.n += 1;
    m.a += member_mix_a(sd.a ^ key);
    m.b += member_mix_b(sd.b ^ key);
}

// The largest protein count whose codes p * 160000 + t fit 32 bits.
constexpr int kMemberMaxProt = (int)(0xFFFFFFFFull / kNTetramers);

// Memberships of `<schema>.<acc>_tetras` (protein index p, genome ids
// checked against [0, n_ids_db)); *ok = false for an id or tetramer out of
// range (the `<p>_tetras` path then reports it as the reference would).
inline MemberSum tetras_members(Conn& tc, const std::string& schema, const std::string& acc, uint32_t p,
                                int32_t n_ids_db, const MemberSeeds& sd, int* rc, bool* ok) {
    MemberSum m;
    *ok = true;
    *rc = tc.each("SELECT tetramer, genomes FROM " + schema + "`" + acc + "_tetras`", [&](sqlite3_stmt* st) {
        const int32_t t = sqlite3_column_int(st, 0);
        const int nb = sqlite3_column_bytes(st, 1) / 4;
        const auto* g = static_cast<const int32_t*>(sqlite3_column_blob(st, 1));
        if (t < 0 || t >= kNTetramers) {
            *ok = false;
            return;
        }
        for (int j = 0; j < nb; ++j) {
            int32_t x;
            std::memcpy(&x, g + j, 4);  // (blob pointers need not be 4-aligned)
            if (x < 0 || x >= n_ids_db) {
                *ok = false;
                return;
            }
            member_add(m, sd, (uint32_t)x, p, (uint32_t)t);
        }
    });
    return m;
}

// The G side of the consistency sums: the lists of genomes [id_base, id_base
// + n) (DB-local ids gid - id_base) of protein p, entries [from, to) of r.
inline MemberSum genome_members(const ProteinLists& r, std::size_t k_from, std::size_t k_to, std::size_t off,
                                int32_t id_base, uint32_t p, const MemberSeeds& sd) {
    MemberSum m;
    for (std::size_t k = k_from; k < k_to; ++k) {
        const uint32_t g = (uint32_t)(r.gid[k] - id_base);
        for (int32_t j = 0; j < r.len[k]; ++j) {
            const int32_t t = r.tet[off + j];
            member_add(m, sd, g, p, (uint32_t)(t < 0 || t >= kNTetramers ? 0xFFFFFFFFu : t));
        }
        off += r.len[k];
    }
    return m;
}

// Sort each list (a blob is normally ascending already) and check that it
// is a set of valid tetramer ids.  false: a duplicate or an id out of range
// (the caller falls back to the `<p>_tetras` path, which reads F as stored).
inline bool normalise_lists(ProteinLists& r) {
    std::size_t off = 0;
    for (std::size_t k = 0; k < r.gid.size(); ++k) {
        int32_t* b = r.tet.data() + off;
        int32_t* e = b + r.len[k];
        if (!std::is_sorted(b, e)) std::sort(b, e);
        for (int32_t* x = b; x < e; ++x)
            if (*x < 0 || *x >= kNTetramers || (x > b && *x == x[-1])) return false;
        off += r.len[k];
    }
    return true;
}

// CSR over (genome, protein) from per-protein lists; T from the lengths.
inline void assemble_g(std::vector<ProteinLists>& lists, int32_t n_ids, LoadedArrays& out) {
    const int64_t P = (int64_t)lists.size();
    out.G_off.assign((int64_t)n_ids * P + 1, 0);
    for (int64_t p = 0; p < P; ++p)
        for (std::size_t k = 0; k < lists[p].gid.size(); ++k) {
            out.G_off[(int64_t)lists[p].gid[k] * P + p + 1] = lists[p].len[k];
            out.T((std::size_t)p, (std::size_t)lists[p].gid[k]) = lists[p].len[k];
        }
    for (int64_t k = 0; k < (int64_t)n_ids * P; ++k) out.G_off[k + 1] += out.G_off[k];
    out.G_tet.resize(out.G_off.back());
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t p = 0; p < P; ++p) {
        std::size_t off = 0;
        for (std::size_t k = 0; k < lists[p].gid.size(); ++k) {
            std::copy(lists[p].tet.begin() + off, lists[p].tet.begin() + off + lists[p].len[k],
                      out.G_tet.begin() + out.G_off[(int64_t)lists[p].gid[k] * P + p]);
            off += lists[p].len[k];
        }
        std::vector<int32_t>().swap(lists[p].gid);
        std::vector<int32_t>().swap(lists[p].tet);
    }
}

// SQLiteSCPDataBase metadata + `<p>_genomes` lists.  Returns 0, an error
// code (1 SQLite, 3 construct), or -1: a blob is not a set (use load_single).
inline int load_single_g(const std::string& path, DBMetaData& meta, LoadedArrays& out, std::string& err) {
    Conn c(path);
    if (!c.ok()) {
        err = "Error in opening " + path + ": " + c.error();
        return 1;  // PFAAI_RC_SQLITE_DB
    }
    int e = 0;
    meta.proteinSet = column_strings(c, "SELECT DISTINCT scp_acc FROM scp_data", &e);  // db_helper.hpp:195-215
    if (e == SQLITE_OK) meta.genomeSet = column_strings(c, "SELECT genome_name FROM genome_metadata", &e);
    if (e != SQLITE_OK) {
        err = "Error in reading metadata of " + path + ": " + c.error();
        return 1;
    }
    const int P = (int)meta.proteinSet.size();
    const int G = (int)meta.genomeSet.size();
    if (P > kMemberMaxProt) return -1;
    std::vector<ProteinLists> lists(P);
    std::vector<char> sets(P, 1);
    const MemberSeeds sd = MemberSeeds::fresh();
    GLoadClock& clk = g_load_clock();
    clk.read_ns = 0;
    clk.check_ns = 0;
    clk.threads = 0;
#pragma omp parallel
    {
        clk.threads.fetch_add(1);
        Conn tc(path);
        int64_t t_read = 0, t_check = 0;
#pragma omp for schedule(dynamic, 1)
        for (int p = 0; p < P; ++p) {
            auto& r = lists[p];
            if (!tc.ok()) {
                r.err = 1;
                continue;
            }
            auto t0 = std::chrono::steady_clock::now();
            int rc = read_genome_lists(tc, "", meta.proteinSet[p], 0, G, r);
            t_read += ns_since(t0);
            if (rc != SQLITE_OK) r.err = rc;
            if (r.err) continue;
            // both orientations hold exactly the same memberships
            t0 = std::chrono::steady_clock::now();
            const MemberSum mg = genome_members(r, 0, r.gid.size(), 0, 0, (uint32_t)p, sd);
            bool ok = true;
            const MemberSum mt = tetras_members(tc, "", meta.proteinSet[p], (uint32_t)p, G, sd, &rc, &ok);
            t_check += ns_since(t0);
            if (rc != SQLITE_OK) r.err = rc;
            else sets[p] = ok && mg == mt && normalise_lists(r);
        }
        clk.read_ns += t_read;
        clk.check_ns += t_check;
    }
    for (int p = 0; p < P; ++p)
        if (lists[p].err) {
            err = "Error in reading tables of protein " + meta.proteinSet[p] + " from " + path;
            return 3;  // PFAAI_RC_CONSTRUCT
        }
    for (int p = 0; p < P; ++p)
        if (!sets[p]) return -1;
    out.T = DMatrix(P, G);
    assemble_g(lists, G, out);
    return 0;
}

// QTSQLiteSCPDataBase metadata + both DBs' `<p>_genomes` lists over the
// shared proteins (db_helper.hpp:109-166); query ids offset by nT.  F built
// from these holds every tetramer of either DB; the reference's inner join
// (scp_db.hpp:459-466) keeps only those in both -- the rest form runs with
// no query-target pair, so counts, S, N and |E| are the same.
inline int load_qt_g(const std::string& tgt, const std::string& qry, DBMetaData& meta, LoadedArrays& out,
                     std::string& err) {
    Conn c(tgt);
    if (!c.ok()) {
        err = "Error in opening " + tgt + ": " + c.error();
        return 1;
    }
    if (c.exec("ATTACH DATABASE '" + qry + "' as QueryDB ;") != SQLITE_OK) {
        err = "Error in attaching query database : " + qry + ": " + c.error();
        return 1;
    }
    int e = 0;
    meta.proteinSet = column_strings(c,
                                     "SELECT DISTINCT target_table.scp_acc \n"
                                     "  FROM `main`.scp_data as target_table, `QueryDB`.scp_data as query_table \n"
                                     "  WHERE target_table.scp_acc = query_table.scp_acc;",
                                     &e);
    if (e == SQLITE_OK) meta.genomeSet = column_strings(c, "SELECT genome_name FROM `main`.genome_metadata", &e);
    if (e == SQLITE_OK) meta.qyGenomeSet = column_strings(c, "SELECT genome_name FROM `QueryDB`.genome_metadata", &e);
    if (e != SQLITE_OK) {
        err = "Error in reading metadata: " + c.error();
        return 1;
    }
    const int P = (int)meta.proteinSet.size();
    const int nT = (int)meta.genomeSet.size(), nQ = (int)meta.qyGenomeSet.size();
    if (P > kMemberMaxProt) return -1;
    std::vector<ProteinLists> lists(P);
    std::vector<char> sets(P, 1);
    const MemberSeeds sd = MemberSeeds::fresh();
#pragma omp parallel
    {
        Conn tc(tgt);
        const bool ok = tc.ok() && tc.exec("ATTACH DATABASE '" + qry + "' as QueryDB ;") == SQLITE_OK;
#pragma omp for schedule(dynamic, 1)
        for (int p = 0; p < P; ++p) {
            auto& r = lists[p];
            if (!ok) {
                r.err = 1;
                continue;
            }
            int rc = read_genome_lists(tc, "main.", meta.proteinSet[p], 0, nT, r);
            const std::size_t k_main = r.gid.size(), n_main = r.tet.size();
            if (rc == SQLITE_OK) rc = read_genome_lists(tc, "QueryDB.", meta.proteinSet[p], nT, nQ, r);
            if (rc != SQLITE_OK) r.err = rc;
            if (r.err) continue;
            // per DB: both orientations hold exactly the same memberships
            const MemberSum mg_t = genome_members(r, 0, k_main, 0, 0, (uint32_t)p, sd);
            const MemberSum mg_q = genome_members(r, k_main, r.gid.size(), n_main, nT, (uint32_t)p, sd);
            bool ok_t = true, ok_q = true;
            const MemberSum mt_t = tetras_members(tc, "main.", meta.proteinSet[p], (uint32_t)p, nT, sd, &rc, &ok_t);
            MemberSum mt_q;
            if (rc == SQLITE_OK) mt_q = tetras_members(tc, "QueryDB.", meta.proteinSet[p], (uint32_t)p, nQ, sd, &rc, &ok_q);
            if (rc != SQLITE_OK) r.err = rc;
            else sets[p] = ok_t && ok_q && mg_t == mt_t && mg_q == mt_q && normalise_lists(r);
        }
    }
    for (int p = 0; p < P; ++p)
        if (lists[p].err) {
            err = "Error in reading tables of protein " + meta.proteinSet[p];
            return 3;
        }
    for (int p = 0; p < P; ++p)
        if (!sets[p]) return -1;
    out.T = DMatrix(P, nT + nQ);
    assemble_g(lists, nT + nQ, out);
    return 0;
}

}  // namespace pfaai_host
