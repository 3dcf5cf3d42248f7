// par_fastaai_amd -- drop-in for the reference CLI `par_fastaai.x`
// (src/main.cpp:56-356) on the MI355X engine.
//
//   par_fastaai_amd [-r query_db] [-s sep] [-q query_list] in_db out_csv
//                   [--corrected] [--device N] [--bin PREFIX]
//
// Ingest reads the `<p>_genomes` blobs (genome-major lists G) and pfaai_load
// builds F on the device (stable radix sort), so the run takes the
// benchmarked k_blk + k_rows_pl path; `--loader tetras` reads F from the
// `<p>_tetras` tables instead (the reference's own F; G is then built on the
// device).  The default output is the reference's, byte for byte, quirks
// included (a pair sharing no tetramer gets the J of
// E[0]'s protein, algorithm_impl.hpp:90-91; -r divides by T[p][i/nT] +
// T[p][nQ + i%nT], ds_impl.hpp:434-436) -- the same default as the C++
// adapter's drop-in constructor.  --corrected opts into the corrected values
// for those cells (AJI 0; the query's and the target's own counts); every
// other cell is identical either way.  (--ref-compat, the default, is still
// accepted.)
//
// Same options, same mode dispatch (main.cpp:337-356), same validation
// errors and exit codes (3 for a bad -q list or overlapping -r genomes,
// main.cpp:204-300; 105 / 106 / 109 for option validation / missing
// required / unexpected arguments, as CLI11 returns them), same CSV.
// The AJI hot path runs on the GPU through pfaai::ParFAAIHipImpl
// (include/pfaai_hip.hpp -> libpfaai_hip.so); SQLite ingest and CSV
// formatting are parallel host code.
#include <sys/stat.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <string>
#include <thread>
#include <unordered_set>
#include <vector>

#include "datastruct.hpp"
#include <sstream>

#include "output.hpp"
#include "pfaai_hip.hpp"
#include "scp_db.hpp"

using namespace pfaai_host;

namespace {

struct AppParams {  // main.cpp:56-131
    std::string pathToDatabase, pathToQryDatabase, pathToQrySubsetFile, pathToOutputFile;
    std::string outFieldSeparator = ",";
    std::string binPrefix;
    std::vector<std::string> qryGenomeSet;
    bool refCompat = true;  // reference-exact by default (--corrected clears it)
    int device = 0;
    std::string dumpPrefix;    // --dump-arrays: write the loader's Lc/F/T (cereal) and exit (no GPU)
    std::string formatSelftest;  // --format-selftest FILE: print fmt-formatted doubles (hex input)
    std::string streamAji;       // --stream-aji FILE: pfaai_stream the AJI vector to FILE (no CSV)
    bool streamCsv = false;      // --stream-csv: the CSV from streamed dense row tiles (no whole matrix)
    long long tileRows = 0;      // --tile-rows N (0: ~256 MB tiles)
    long long tilePairs = 1ll << 27;
    std::vector<int> devices;    // --devices 0,1,...: one context per device, rows split (ALL / QT)
    bool loaderTetras = false;   // --loader tetras: F from `<p>_tetras` (else G from `<p>_genomes`)
    std::string dumpGenomes;     // --dump-genomes PREFIX: write the G-path arrays (G_off, G_tet, T) and exit

    void print() const {
        std::vector<std::string> args = {" Input Database  : " + pathToDatabase + " ",
                                         " Query Database  : " + pathToQryDatabase + " ",
                                         " Query Subset    : " + pathToQrySubsetFile + " ",
                                         " Output File     : " + pathToOutputFile + " ",
                                         " Field Separator : " + outFieldSeparator + " "};
        std::size_t w = 0;
        for (auto& a : args) w = std::max(w, a.size());
        std::string bar;
        for (std::size_t i = 0; i < w; ++i) bar += "─";
        std::cout << " ┌" << bar << "┐\n";
        for (auto& a : args) std::cout << " │" << a << std::string(w - a.size(), ' ') << "│\n";
        std::cout << " └" << bar << "┘\n";
    }

    void load_query_genomes() {  // main.cpp:114-124
        std::ifstream in(pathToQrySubsetFile);
        std::string s;
        while (in >> s) qryGenomeSet.push_back(s);
    }
};

bool is_file(const std::string& p) {
    struct stat st;
    return stat(p.c_str(), &st) == 0 && S_ISREG(st.st_mode);
}

const char* kUsage =
    "MI355X-native ParFastAAI (all-pairs AJI)\n"
    "Usage: par_fastaai_amd [OPTIONS] path_to_input_db path_to_output_file\n\n"
    "Positionals:\n"
    "  path_to_input_db TEXT:FILE REQUIRED   Path to the Input Database\n"
    "  path_to_output_file TEXT REQUIRED     Path to output csv file.\n\n"
    "Options:\n"
    "  -h,--help                Print this help message and exit\n"
    "  -r,--query_db TEXT:FILE  Path to the Query Database [Optional (default: Same as the Input DB)]\n"
    "  -s,--separator TEXT [,]  Field Separator in the output file [Optional (default: ,)].\n"
    "  -q,--query_subset TEXT:FILE  Path to Query List (Should be subset of genomoes in the input DB.)\n"
    "  --corrected              Correct the reference's quirks instead of reproducing them (the default\n"
    "                           output is par_fastaai.x's, byte for byte): pairs sharing no tetramer get\n"
    "                           AJI 0, and -r divides by the query's and the target's own tetramer counts.\n"
    "                           All other cells are identical either way.\n"
    "  --ref-compat             Reproduce the reference's values (the default)\n"
    "  --loader TEXT [genomes]  genomes: read <p>_genomes, F built on the GPU; tetras: read <p>_tetras\n"
    "  --device INT [0]         HIP device\n"
    "  --devices LIST           Comma-separated HIP devices: rows split over them (all-vs-all, -r)\n"
    "  --bin TEXT               Also write cereal binaries PREFIX_{jac,aji,aji_matrix}.bin\n"
    "  --stream-aji TEXT        Stream the AJI vector (JAC-index order, cereal vector<double>) to FILE\n"
    "                           tile by tile instead of writing the CSV matrix (-q not supported)\n"
    "  --tile-pairs INT [134217728]  Pairs per streamed output tile\n"
    "  --stream-csv             Write the CSV from streamed tiles of whole output rows (bounded memory;\n"
    "                           same bytes as the default writer)\n"
    "  --tile-rows INT          Rows per --stream-csv tile [about 256 MB of doubles]\n";

// CLI11-compatible parse: returns -1 to continue, else the exit code.
int parse(int argc, char** argv, AppParams& a) {
    std::vector<std::string> pos, extras;
    for (int i = 1; i < argc; ++i) {
        std::string s = argv[i];
        auto value = [&](std::string& dst) -> bool {
            auto eq = s.find('=');
            if (s.rfind("--", 0) == 0 && eq != std::string::npos) {
                dst = s.substr(eq + 1);
                return true;
            }
            if (i + 1 >= argc) return false;
            dst = argv[++i];
            return true;
        };
        auto is = [&](const char* sh, const char* lg) {
            return s == sh || s == lg || (s.rfind(std::string(lg) + "=", 0) == 0);
        };
        if (s == "-h" || s == "--help") {
            std::cout << kUsage;
            return 0;
        } else if (is("-r", "--query_db")) {
            if (!value(a.pathToQryDatabase)) { std::cerr << "--query_db: 1 required TEXT:FILE missing\n"; return 114; }
        } else if (is("-s", "--separator")) {
            if (!value(a.outFieldSeparator)) { std::cerr << "--separator: 1 required TEXT missing\n"; return 114; }
        } else if (is("-q", "--query_subset")) {
            if (!value(a.pathToQrySubsetFile)) { std::cerr << "--query_subset: 1 required TEXT:FILE missing\n"; return 114; }
        } else if (s == "--ref-compat") {
            a.refCompat = true;
        } else if (s == "--corrected") {
            a.refCompat = false;
        } else if (is("--device", "--device")) {
            std::string v;
            if (!value(v)) return 114;
            a.device = std::atoi(v.c_str());
        } else if (is("--stream-aji", "--stream-aji")) {
            if (!value(a.streamAji)) return 114;
        } else if (is("--devices", "--devices")) {
            std::string v;
            if (!value(v)) return 114;
            std::stringstream ss(v);
            std::string tok;
            while (std::getline(ss, tok, ','))
                if (!tok.empty()) a.devices.push_back(std::atoi(tok.c_str()));
            if (a.devices.empty()) return 105;
        } else if (is("--tile-pairs", "--tile-pairs")) {
            std::string v;
            if (!value(v)) return 114;
            a.tilePairs = std::atoll(v.c_str());
            if (a.tilePairs < 1) return 105;
        } else if (is("--loader", "--loader")) {
            std::string v;
            if (!value(v)) return 114;
            if (v != "genomes" && v != "tetras") {
                std::cerr << "--loader: " << v << " not in {genomes, tetras}\nRun with --help for more information.\n";
                return 105;
            }
            a.loaderTetras = v == "tetras";
        } else if (is("--dump-genomes", "--dump-genomes")) {
            if (!value(a.dumpGenomes)) return 114;
        } else if (s == "--stream-csv") {
            a.streamCsv = true;
        } else if (is("--tile-rows", "--tile-rows")) {
            std::string v;
            if (!value(v)) return 114;
            a.tileRows = std::atoll(v.c_str());
            if (a.tileRows < 1) return 105;
        } else if (is("--bin", "--bin")) {
            if (!value(a.binPrefix)) return 114;
        } else if (is("--dump-arrays", "--dump-arrays")) {
            if (!value(a.dumpPrefix)) return 114;
        } else if (is("--format-selftest", "--format-selftest")) {
            if (!value(a.formatSelftest)) return 114;
            return -2;
        } else if (s.size() > 1 && s[0] == '-') {
            extras.push_back(s);
        } else {
            pos.push_back(s);
        }
    }
    if (pos.size() > 2) extras.insert(extras.end(), pos.begin() + 2, pos.end());
    if (!extras.empty()) {
        std::cerr << "The following arguments were not expected:";
        for (auto& e : extras) std::cerr << " " << e;
        std::cerr << "\nRun with --help for more information.\n";
        return 109;  // CLI11 ExtrasError
    }
    if (pos.size() >= 1) a.pathToDatabase = pos[0];
    if (pos.size() >= 2) a.pathToOutputFile = pos[1];
    auto must_exist = [](const std::string& opt, const std::string& p) {
        if (!p.empty() && !is_file(p)) {
            std::cerr << opt << ": File does not exist: " << p << "\nRun with --help for more information.\n";
            return false;
        }
        return true;
    };
    if (pos.empty()) {
        std::cerr << "path_to_input_db is required\nRun with --help for more information.\n";
        return 106;  // CLI11 RequiredError
    }
    if (!must_exist("path_to_input_db", a.pathToDatabase)) return 105;  // CLI11 ValidationError
    if (pos.size() < 2) {
        std::cerr << "path_to_output_file is required\nRun with --help for more information.\n";
        return 106;
    }
    if (!must_exist("--query_db", a.pathToQryDatabase)) return 105;
    if (!must_exist("--query_subset", a.pathToQrySubsetFile)) return 105;
    return -1;
}

double ms_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

// --dump-arrays: the loader's arrays in the reference's fixture format
// (vector<int> Lc, vector<DPair<int,int>> F, DMatrix<int> T), no GPU.
int dump_arrays(const std::string& prefix, const LoadedArrays& arr) {
    auto put = [](FILE* f, const void* p, std::size_t n) { return n == 0 || std::fwrite(p, 1, n, f) == n; };  // (empty vectors: data() may be null)
    bool ok = true;
    if (FILE* f = std::fopen((prefix + "_lc_array.bin").c_str(), "wb")) {
        uint64_t n = arr.Lc.size();
        ok &= put(f, &n, 8) && put(f, arr.Lc.data(), 4 * n);
        std::fclose(f);
    } else ok = false;
    if (FILE* f = std::fopen((prefix + "_f_array.bin").c_str(), "wb")) {
        uint64_t n = arr.F.size();
        ok &= put(f, &n, 8) && put(f, arr.F.data(), 8 * n);
        std::fclose(f);
    } else ok = false;
    if (FILE* f = std::fopen((prefix + "_t_matrix.bin").c_str(), "wb")) {
        uint64_t h[3] = {arr.T.rows(), arr.T.cols(), arr.T.rows() * arr.T.cols()};
        ok &= put(f, h, 24) && put(f, arr.T.data.data(), 4 * arr.T.data.size());
        std::fclose(f);
    } else ok = false;
    return ok ? 0 : 1;
}

// --dump-genomes: the G-path arrays (cereal vector<int64> G_off, vector<int>
// G_tet, DMatrix<int> T), no GPU.
int dump_genomes(const std::string& prefix, const LoadedArrays& arr) {
    auto put = [](FILE* f, const void* p, std::size_t n) { return n == 0 || std::fwrite(p, 1, n, f) == n; };  // (empty vectors: data() may be null)
    bool ok = true;
    if (FILE* f = std::fopen((prefix + "_g_off.bin").c_str(), "wb")) {
        uint64_t n = arr.G_off.size();
        ok &= put(f, &n, 8) && put(f, arr.G_off.data(), 8 * n);
        std::fclose(f);
    } else ok = false;
    if (FILE* f = std::fopen((prefix + "_g_tet.bin").c_str(), "wb")) {
        uint64_t n = arr.G_tet.size();
        ok &= put(f, &n, 8) && put(f, arr.G_tet.data(), 4 * n);
        std::fclose(f);
    } else ok = false;
    if (FILE* f = std::fopen((prefix + "_t_matrix.bin").c_str(), "wb")) {
        uint64_t h[3] = {arr.T.rows(), arr.T.cols(), arr.T.rows() * arr.T.cols()};
        ok &= put(f, h, 24) && put(f, arr.T.data.data(), 4 * arr.T.data.size());
        std::fclose(f);
    } else ok = false;
    return ok ? 0 : 1;
}

const char* kRowsKernelName[] = {"k_rows_pl", "k_rows_pl512", "k_rows(fused)", "k_rows(worklist)", "k_rows_v2"};

// The loader: G from `<p>_genomes` unless --loader tetras / --dump-arrays, or
// a blob that is not a set (then the `<p>_tetras` F, as the reference reads).
template <class LoadG, class LoadF>
int ingest(const AppParams& app, LoadG load_g, LoadF load_f, DBMetaData& meta, LoadedArrays& arr, std::string& err) {
    auto t0 = std::chrono::steady_clock::now();
    int rc = -1;
    const char* what = "<p>_genomes -> G";
    if (!app.loaderTetras && app.dumpPrefix.empty()) rc = load_g(meta, arr, err);
    if (rc == -1) {
        meta = DBMetaData();
        arr = LoadedArrays();
        rc = load_f(meta, arr, err);
        what = "<p>_tetras -> F";
    }
    if (rc) {
        std::cerr << err << std::endl;
        return rc;
    }
    std::printf("Load (SQLite)       : %10.2f ms  (%s, %zu entries)\n", ms_since(t0), what,
                arr.F.empty() ? arr.G_tet.size() : arr.F.size());
    const auto& gc = pfaai_host::g_load_clock();
    if (!arr.G_tet.empty() && gc.read_ns > 0 && gc.threads > 0)  // thread time over the reading threads
        std::printf("  G-path threads    : %d; per thread <p>_genomes read %.1f ms, orientation check "
                    "(<p>_tetras read + sums) %.1f ms\n",
                    gc.threads.load(), gc.read_ns / 1e6 / gc.threads, gc.check_ns / 1e6 / gc.threads);
    return 0;
}

// The HIP runtime's first initialisation (~80 ms on the box) and the engine's
// contexts are made on a helper thread while the main thread reads SQLite;
// run_and_print joins it first.
static std::thread g_warm;
static void warm_gpu_join() {
    if (g_warm.joinable()) g_warm.join();
}
struct WarmGuard {
    ~WarmGuard() { warm_gpu_join(); }
};

// end of the last printed phase (the CLI's teardown line measures from here)
static std::chrono::steady_clock::time_point g_t_phases_end;
static bool g_have_phases_end = false;

template <typename DS>
int run_and_print(const DS& ds, int mode, const AppParams& app, bool isSubset) {
    const auto tw = std::chrono::steady_clock::now();
    warm_gpu_join();
    std::printf("HIP init (helper)   : %10.2f ms  waited for after the load\n", ms_since(tw));
    auto t0 = std::chrono::steady_clock::now();
    try {
        const std::vector<int> devs = app.devices.empty() ? std::vector<int>{app.device} : app.devices;
        // the run()-and-print path prepares its host outputs during construction
        // (initJAC, output pages); the streamed paths never hold them
        // the reference's QT rows overlap when nQ > nT (its column placement,
        // ds_impl.hpp:434-436 + main.cpp:149, writes later rows over earlier
        // ones): pfaai_stream_matrix cannot reproduce that tile by tile, so
        // such a run takes the dense writer below (same bytes)
        const bool stream_ok = !(mode == PFAAI_MODE_QT && app.refCompat && ds.qrySetSize() > ds.tgtSetSize());
        const bool streamed = !app.streamAji.empty() || (app.streamCsv && stream_ok && !app.pathToOutputFile.empty());
        pfaai::ParFAAIHipImpl<int32_t, double, DS> impl(ds, mode, devs, app.refCompat, !streamed);
        pfaai::release_parked_contexts();  // prewarmed contexts no engine adopted
        if (!app.streamAji.empty()) {  // output-tile streaming: no CSV, no whole matrix anywhere
            if (mode == PFAAI_MODE_QSUB) {
                std::cerr << "--stream-aji does not support -q" << std::endl;
                return PFAAI_RC_INVALID;
            }
            int rc = impl.streamAJI(app.streamAji, app.tilePairs);
            std::printf("AJI stream (MI355X) : %10.2f ms  (|E| = %lld) -> %s\n", ms_since(t0),
                        (long long)impl.nEvents(), app.streamAji.c_str());
            return rc;
        }
        if (app.streamCsv && !stream_ok)
            std::printf("--stream-csv: -r with more query than target genomes reproduces the reference's overlapping "
                        "rows only through the dense writer; writing the CSV that way\n");
        if (app.streamCsv && stream_ok && !app.pathToOutputFile.empty()) {  // CSV from streamed dense row tiles
            auto t1 = std::chrono::steady_clock::now();
            std::printf("Writing output with %lld query genomes and %lld target genomes. \n",
                        (long long)ds.qrySetSize(), (long long)ds.tgtSetSize());
            CsvWriter w(app.pathToOutputFile, ds.refTargetSet(), app.outFieldSeparator);
            if (!w.ok()) {
                std::cerr << "Error in writing " << app.pathToOutputFile << std::endl;
                return 1;
            }
            struct Ctx { CsvWriter* w; const std::vector<std::string>* names; };
            Ctx cx{&w, &ds.refQuerySet()};
            const int64_t ncols = (int64_t)ds.tgtSetSize();
            const int64_t tr = app.tileRows > 0 ? app.tileRows : std::max<int64_t>(1, ((int64_t)1 << 25) / std::max<int64_t>(ncols, 1));
            impl.streamMatrix(tr, [](void* u, int64_t r0, int64_t r1, int64_t, const double* block) -> int {
                auto* x = static_cast<Ctx*>(u);
                return x->w->rows(*x->names, block, r0, r1) ? 0 : PFAAI_RC_INVALID;
            }, &cx);
            if (!w.close()) {
                std::cerr << "Error in writing " << app.pathToOutputFile << std::endl;
                return 1;
            }
            std::printf("AJI + CSV (streamed): %10.2f ms  (%lld-row tiles; |E| both orientations = %lld)\n",
                        ms_since(t1), (long long)tr, (long long)impl.nEvents());
            return 0;
        }
        auto t1 = std::chrono::steady_clock::now();
        impl.run();
        const double ms_run = ms_since(t1);
        const int rk = impl.rowsKernel();
        const int wf = impl.walkForm();
        std::printf("AJI (MI355X x%d)     : %10.2f ms  (|E| = %lld; %s; walk %s%s)\n", impl.nDevices(), ms_since(t0),
                    (long long)impl.nEvents(), rk >= 0 && rk < 5 ? kRowsKernelName[rk] : "?",
                    wf == PFAAI_WALK_GPOS ? "G_pos..G_end" : wf == PFAAI_WALK_SPANS ? "window spans" : wf == PFAAI_WALK_SPLITTERS ? "run table + splitters" : "-",
                    impl.narrowLaunch() ? ", 512-thread narrow rows" : "");
        double lc = 0, lu = 0, ld = 0;
        pfaai_load_timing(impl.context(), &lc, &lu, &ld);
        const double ms_ctor = std::chrono::duration<double, std::milli>(t1 - t0).count();
        std::printf("  breakdown         : context %.1f + load checks %.1f, H2D %.1f, device F/G %.1f ms; run %.1f ms = "
                    "run tables %.2f + %s %.2f + D2H / JAC fill %.1f ms\n"
                    "  host side of run  : engine compute + D2H done at %.1f, initJAC %s %.1f, JAC fill %.1f ms\n",
                    ms_ctor - lc - lu - ld, lc, lu, ld, ms_run, impl.msBuild(), rk >= 0 && rk < 5 ? kRowsKernelName[rk] : "?",
                    impl.msRows(), ms_run - impl.msBuild() - impl.msRows(), impl.msCompute(),
                    impl.preparedAhead() ? "+ output pages (during construction) took" : "(beside it) done at", impl.msIds(),
                    impl.msFill());
        if (app.pathToOutputFile.empty()) return 0;
        t1 = std::chrono::steady_clock::now();
        std::printf("Writing output with %lld query genomes and %lld target genomes. \n",
                    (long long)ds.qrySetSize(), (long long)ds.tgtSetSize());
        auto M = dense_matrix(ds, impl.getJAC(), impl.getAJI(), isSubset);
        if (write_csv(app.pathToOutputFile, ds.refQuerySet(), ds.refTargetSet(), M, app.outFieldSeparator)) {
            std::cerr << "Error in writing " << app.pathToOutputFile << std::endl;
            return 1;
        }
        if (!app.binPrefix.empty())
            write_bin(app.binPrefix, impl.getJAC(), impl.getAJI(), M, ds.qrySetSize(), ds.tgtSetSize());
        std::printf("Output              : %10.2f ms\n", ms_since(t1));
        g_t_phases_end = std::chrono::steady_clock::now();
        g_have_phases_end = true;
    } catch (const pfaai::HipError& e) {
        std::cerr << "MI355X engine error " << e.code << ": " << e.what() << std::endl;
        return e.code;
    }
    return 0;
}

int parallel_fastaai(const AppParams& app) {  // main.cpp:177-202
    DBMetaData meta;
    LoadedArrays arr;
    std::string err;
    const std::string& db = app.pathToDatabase;
    if (int rc = ingest(
            app, [&](DBMetaData& m, LoadedArrays& a, std::string& e) { return load_single_g(db, m, a, e); },
            [&](DBMetaData& m, LoadedArrays& a, std::string& e) { return load_single(db, m, a, e); }, meta, arr, err))
        return rc;
    if (!app.dumpPrefix.empty()) return dump_arrays(app.dumpPrefix, arr);
    if (!app.dumpGenomes.empty()) return dump_genomes(app.dumpGenomes, arr);
    AllData ds(std::move(meta), std::move(arr));
    return run_and_print(ds, PFAAI_MODE_ALL, app, true);
}

int validate_subset(const AppParams& app, const DBMetaData& meta) {  // main.cpp:204-232
    std::unordered_set<std::string> db(meta.genomeSet.begin(), meta.genomeSet.end());
    std::vector<std::string> missing;
    for (auto& g : app.qryGenomeSet)
        if (!db.count(g)) missing.push_back(g);
    if (!missing.empty()) {
        std::cout << "--------------------ERROR-----------------------------\n"
                  << " In the query subset file, the following genomes are \n"
                  << " missing from the database : \n";
        for (std::size_t i = 0; i < missing.size(); ++i) std::cout << (i ? "\n    " : "    ") << missing[i];
        std::cout << "\n\n Please remove them and before running Fast AAI. \n"
                  << "------------------------------------------------------\n";
        return 3;
    }
    return 0;
}

int parallel_subset_fastaai(const AppParams& app) {  // main.cpp:234-266
    DBMetaData meta;
    LoadedArrays arr;
    std::string err;
    const std::string& db = app.pathToDatabase;
    if (int rc = ingest(
            app, [&](DBMetaData& m, LoadedArrays& a, std::string& e) { return load_single_g(db, m, a, e); },
            [&](DBMetaData& m, LoadedArrays& a, std::string& e) { return load_single(db, m, a, e); }, meta, arr, err))
        return rc;
    if (validate_subset(app, meta)) return 3;
    if (!app.dumpPrefix.empty()) return dump_arrays(app.dumpPrefix, arr);
    if (!app.dumpGenomes.empty()) return dump_genomes(app.dumpGenomes, arr);
    QSubData ds(std::move(meta), std::move(arr), app.qryGenomeSet);
    return run_and_print(ds, PFAAI_MODE_QSUB, app, true);
}

int validate_qry2tgt(const DBMetaData& meta) {  // main.cpp:268-300
    std::unordered_set<std::string> db(meta.genomeSet.begin(), meta.genomeSet.end());
    std::vector<std::string> common;
    for (auto& g : meta.qyGenomeSet)
        if (db.count(g)) common.push_back(g);
    if (!common.empty()) {
        std::cout << "---------------------ERROR------------------------------\n"
                  << "  Query database should have no intersecting genes with \n"
                  << "  the main data base.\n\n"
                  << "  In the query data base, the following genomes are \n"
                  << "  overlapping with the target database:\n";
        for (std::size_t i = 0; i < common.size(); ++i) std::cout << (i ? "\n    " : "    ") << common[i];
        std::cout << "\n\n  Please remove them before running Fast AAI.\n"
                  << "--------------------------------------------------------\n";
        return 3;
    }
    return 0;
}

int parallel_qry2tgt_fastaai(const AppParams& app) {  // main.cpp:302-335
    DBMetaData meta;
    LoadedArrays arr;
    std::string err;
    const std::string &tdb = app.pathToDatabase, &qdb = app.pathToQryDatabase;
    if (int rc = ingest(
            app, [&](DBMetaData& m, LoadedArrays& a, std::string& e) { return load_qt_g(tdb, qdb, m, a, e); },
            [&](DBMetaData& m, LoadedArrays& a, std::string& e) { return load_qt(tdb, qdb, m, a, e); }, meta, arr,
            err))
        return rc;
    if (validate_qry2tgt(meta)) return 3;
    if (!app.dumpPrefix.empty()) return dump_arrays(app.dumpPrefix, arr);
    if (!app.dumpGenomes.empty()) return dump_genomes(app.dumpGenomes, arr);
    QTData ds(std::move(meta), std::move(arr));
    return run_and_print(ds, PFAAI_MODE_QT, app, false);
}

}  // namespace

int main(int argc, char** argv) {  // main.cpp:337-356
    AppParams app;
    int rc = parse(argc, argv, app);
    if (rc == -2) {  // --format-selftest: one hex double per line -> fmt `{}` text
        std::ifstream in(app.formatSelftest);
        std::string s;
        char buf[48];
        while (in >> s) {
            const double v = std::strtod(s.c_str(), nullptr);
            std::fwrite(buf, 1, fmt_double(v, buf), stdout);
            std::fputc('\n', stdout);
        }
        return 0;
    }
    if (rc >= 0) return rc;
    app.print();
    WarmGuard warm_guard;
    if (app.dumpPrefix.empty() && app.dumpGenomes.empty()) {
        const std::vector<int> devs = app.devices.empty() ? std::vector<int>{app.device} : app.devices;
        try {
            g_warm = std::thread([devs] {  // the engine adopts these contexts (pfaai::prewarm_context)
                for (int d : devs) pfaai::prewarm_context(d);
            });
        } catch (const std::system_error&) {  // no thread: the engine initialises HIP itself
        }
    }
    const auto t_main = std::chrono::steady_clock::now();
    if (app.pathToQryDatabase.empty() || app.pathToQryDatabase == app.pathToDatabase) {
        if (app.pathToQrySubsetFile.empty()) {
            rc = parallel_fastaai(app);
        } else {
            app.load_query_genomes();
            rc = parallel_subset_fastaai(app);
        }
    } else {
        rc = parallel_qry2tgt_fastaai(app);
    }
    if (g_have_phases_end)  // engine contexts destroyed, host arrays freed
        std::printf("Teardown            : %10.2f ms\n", ms_since(g_t_phases_end));
    std::printf("Total (CLI)         : %10.2f ms  (engine teardown included)\n", ms_since(t_main));
    // Every output file is closed and every engine context destroyed (both
    // inside the total above); what is left is the HIP runtime's exit-time
    // teardown of its own state.  Flush and leave without it, unless
    // PFAAI_CLI_FAST_EXIT=0.
    const char* fe = std::getenv("PFAAI_CLI_FAST_EXIT");
    if (!(fe && fe[0] == '0')) {
        warm_gpu_join();
        std::fflush(nullptr);
        std::_Exit(rc);
    }
    return rc;
}
