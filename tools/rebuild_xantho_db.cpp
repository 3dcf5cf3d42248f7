// rebuild_xantho_db -- rebuild the reference's 20-genome test DB
// (data/modified_xantho_fastaai2.db, a missing blob upstream; BASELINE
// config C1) from its committed arrays, so that the SQLite loader and the
// CLI can be run on C1.
//
//   rebuild_xantho_db F.bin Lc.bin T.bin names.txt out.db
//
// Inputs: the reference's own fixtures xanthodb_f_array.bin (cereal
// vector<DPair<int,int>>: (protein, genome) by (tetramer, protein, genome)),
// xanthodb_lc_array.bin (vector<int>[160000]), xanthodb_t_matrix.bin
// (DMatrix<int> P x G) and tests/golden/xantho_names.txt ("P <acc>" lines in
// protein-index order, "G <name>" lines in genome-id order; from
// tests/pfaai_tests.hpp:23-39, 159-179).  Output: a FastAAI-layout DB with
// the schema of the reference's own xdb_subset*.db (scp_db.hpp:37-55):
//   genome_metadata(genome_name, genome_id PK, ...)    genome id = index
//   scp_data(genome_id, SCP_acc, SCP_score, tetra_count)  rows protein-major,
//        so SELECT DISTINCT SCP_acc (db_helper.hpp:195-215) yields protein order
//   `<acc>_tetras`(tetramer PK, genomes BLOB int32[])   one row per run of F
//   `<acc>_genomes`(genome_id PK, tetramers BLOB int32[]) sorted tetramer sets;
//        their lengths are T (scp_db.hpp:219-262, checked against the T fixture)
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "../parfastaai_amd/host/sqlite_min.h"

namespace {

std::vector<char> slurp(const char* path) {
    std::ifstream in(path, std::ios::binary);
    if (!in) {
        std::fprintf(stderr, "cannot read %s\n", path);
        std::exit(2);
    }
    return std::vector<char>((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
}

template <class T>
std::vector<T> cereal_vector(const char* path) {  // u64 n, then n packed records
    const auto b = slurp(path);
    uint64_t n = 0;
    std::memcpy(&n, b.data(), 8);
    if (b.size() != 8 + n * sizeof(T)) {
        std::fprintf(stderr, "%s: bad size\n", path);
        std::exit(2);
    }
    std::vector<T> v(n);
    std::memcpy(v.data(), b.data() + 8, n * sizeof(T));
    return v;
}

void check(int rc, sqlite3* db, const char* what) {
    if (rc != SQLITE_OK && rc != SQLITE_DONE && rc != SQLITE_ROW) {
        std::fprintf(stderr, "%s: %s\n", what, sqlite3_errmsg(db));
        std::exit(3);
    }
}

void exec(sqlite3* db, const std::string& sql) { check(sqlite3_exec(db, sql.c_str(), nullptr, nullptr, nullptr), db, sql.c_str()); }

sqlite3_stmt* prepare(sqlite3* db, const std::string& sql) {
    sqlite3_stmt* st = nullptr;
    check(sqlite3_prepare_v2(db, sql.c_str(), -1, &st, nullptr), db, sql.c_str());
    return st;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc != 6) {
        std::fprintf(stderr, "usage: %s F.bin Lc.bin T.bin names.txt out.db\n", argv[0]);
        return 1;
    }
    struct Pair { int32_t p, g; };
    const auto F = cereal_vector<Pair>(argv[1]);
    const auto Lc = cereal_vector<int32_t>(argv[2]);
    const auto Tb = slurp(argv[3]);
    uint64_t th[3];
    std::memcpy(th, Tb.data(), 24);
    const int64_t P = (int64_t)th[0], G = (int64_t)th[1];
    std::vector<int32_t> T(P * G);
    std::memcpy(T.data(), Tb.data() + 24, T.size() * 4);
    std::vector<std::string> prot, gen;
    {
        std::ifstream in(argv[4]);
        std::string line;
        while (std::getline(in, line))
            if (line.size() > 2) (line[0] == 'P' ? prot : gen).push_back(line.substr(2));
    }
    if ((int64_t)prot.size() != P || (int64_t)gen.size() != G || Lc.size() != 160000) {
        std::fprintf(stderr, "names / arrays disagree: P %lld vs %zu, G %lld vs %zu\n", (long long)P, prot.size(),
                     (long long)G, gen.size());
        return 2;
    }
    std::vector<int64_t> Lp(160001, 0);
    for (int t = 0; t < 160000; ++t) Lp[t + 1] = Lp[t] + Lc[t];
    if (Lp[160000] != (int64_t)F.size()) {
        std::fprintf(stderr, "Lc does not sum to |F|\n");
        return 2;
    }
    // genome-major sets: tetramers of (p, g), ascending (F is tetramer-major)
    std::vector<std::vector<int32_t>> sets(P * G);
    for (int t = 0; t < 160000; ++t)
        for (int64_t i = Lp[t]; i < Lp[t + 1]; ++i) sets[F[i].p * G + F[i].g].push_back(t);
    for (int64_t p = 0; p < P; ++p)
        for (int64_t g = 0; g < G; ++g)
            if ((int64_t)sets[p * G + g].size() != T[p * G + g]) {
                std::fprintf(stderr, "T(%lld, %lld) != |F entries| -- arrays inconsistent\n", (long long)p, (long long)g);
                return 2;
            }

    std::remove(argv[5]);
    sqlite3* db = nullptr;
    check(sqlite3_open_v2(argv[5], &db, SQLITE_OPEN_READWRITE | SQLITE_OPEN_CREATE, nullptr), db, "open");
    exec(db, "BEGIN");
    exec(db, "CREATE TABLE 'genome_metadata' (genome_name TEXT, genome_id INTEGER PRIMARY KEY, genome_length INTEGER, "
             "genome_class INTEGER, SCP_count INTEGER)");
    exec(db, "CREATE TABLE 'scp_data' (genome_id INTEGER, SCP_acc TEXT, SCP_score REAL, tetra_count INTEGER)");
    sqlite3_stmt* st = prepare(db, "INSERT INTO genome_metadata VALUES (?, ?, 0, 0, ?)");
    for (int64_t g = 0; g < G; ++g) {
        int scps = 0;
        for (int64_t p = 0; p < P; ++p) scps += T[p * G + g] > 0;
        sqlite3_bind_text(st, 1, gen[g].c_str(), -1, PFAAI_SQLITE_TRANSIENT);
        sqlite3_bind_int(st, 2, (int)g);
        sqlite3_bind_int(st, 3, scps);
        check(sqlite3_step(st), db, "genome_metadata");
        sqlite3_reset(st);
    }
    sqlite3_finalize(st);
    st = prepare(db, "INSERT INTO scp_data VALUES (?, ?, 0.0, ?)");
    for (int64_t p = 0; p < P; ++p)  // protein-major: first appearances in protein order
        for (int64_t g = 0; g < G; ++g) {
            if (!T[p * G + g]) continue;
            sqlite3_bind_int(st, 1, (int)g);
            sqlite3_bind_text(st, 2, prot[p].c_str(), -1, PFAAI_SQLITE_TRANSIENT);
            sqlite3_bind_int(st, 3, T[p * G + g]);
            check(sqlite3_step(st), db, "scp_data");
            sqlite3_reset(st);
        }
    sqlite3_finalize(st);
    for (int64_t p = 0; p < P; ++p) {
        const std::string& a = prot[p];
        exec(db, "CREATE TABLE '" + a + "_tetras' (tetramer INTEGER PRIMARY KEY, genomes BLOB)");
        exec(db, "CREATE TABLE '" + a + "_genomes' (genome_id INTEGER PRIMARY KEY, tetramers BLOB)");
        st = prepare(db, "INSERT INTO `" + a + "_tetras` VALUES (?, ?)");
        std::vector<int32_t> run;
        for (int t = 0; t < 160000; ++t) {
            run.clear();
            for (int64_t i = Lp[t]; i < Lp[t + 1]; ++i)
                if (F[i].p == p) run.push_back(F[i].g);
            if (run.empty()) continue;
            sqlite3_bind_int(st, 1, t);
            sqlite3_bind_blob(st, 2, run.data(), (int)(run.size() * 4), PFAAI_SQLITE_TRANSIENT);
            check(sqlite3_step(st), db, "tetras");
            sqlite3_reset(st);
        }
        sqlite3_finalize(st);
        st = prepare(db, "INSERT INTO `" + a + "_genomes` VALUES (?, ?)");
        for (int64_t g = 0; g < G; ++g) {
            const auto& s = sets[p * G + g];
            if (s.empty()) continue;
            sqlite3_bind_int(st, 1, (int)g);
            sqlite3_bind_blob(st, 2, s.data(), (int)(s.size() * 4), PFAAI_SQLITE_TRANSIENT);
            check(sqlite3_step(st), db, "genomes");
            sqlite3_reset(st);
        }
        sqlite3_finalize(st);
    }
    exec(db, "COMMIT");
    sqlite3_close(db);
    std::printf("wrote %s: %lld proteins, %lld genomes, |F| = %zu\n", argv[5], (long long)P, (long long)G, F.size());
    return 0;
}
