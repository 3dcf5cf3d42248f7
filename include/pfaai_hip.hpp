// pfaai_hip.hpp -- C++ adapter with the reference's ParFAAIImpl surface over
// the C ABI of libpfaai_hip.so.
//
// Drop-in for  ParFAAIImpl<IdType, ValueType, DSIT>
//              (reference include/pfaai/algorithm_impl.hpp:38-357):
//   explicit ParFAAIHipImpl(const DSIT&);  int run();  int computeJAC();
//   int computeAJI();  const std::vector<JACType>& getJAC() const;
//   const std::vector<ValueType>& getAJI() const;
// DSIT is any type with the reference's DataStructInterface accessors
// (interface.hpp:200-328): refLc(), refF() (elements with .first/.second),
// refT() (operator()(p, g), rows(), cols()), initJAC(), qrySetSize(),
// tgtSetSize(), isQryGenome(), mapQueryId(), plus the JACType typedef -- the
// reference's own ParFAAIData / ParFAAIQSubData / ParFAAIQryTgtData qualify
// unchanged, and so do the host classes of parfastaai_amd/host/datastruct.hpp.
// A DSIT that also holds the genome-major `<p>_genomes` lists (refGOff(),
// refGTet()) hands them over too; with an empty refF() only G is sent and F
// is built on the device.
//
// The mode is deduced from the DSIT (pfaai_mode_of<DSIT>, specialisable):
// a type with nUnionGenomes() is query-vs-target (ParFAAIQryTgtData,
// ds_impl.hpp:370); otherwise the index maps decide -- every genome a query
// under the identity map is all-vs-all (ParFAAIData, ds_impl.hpp:83-96),
// anything else the query subset (ParFAAIQSubData, ds_impl.hpp:251-276).
//
// The one-argument constructor is the drop-in: it reproduces the class it
// replaces bit for bit, quirks included (PFAAI_FLAG_REF_COMPAT: SURVEY 8a
// rows Z and Q).  The explicit forms choose the mode, the corrected
// semantics (ref_compat = false) and the device(s).
#pragma once
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <exception>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <system_error>
#include <thread>
#include <type_traits>
#include <utility>
#include <vector>

#include "pfaai_hip.h"

namespace pfaai {

struct HipError : std::runtime_error {
    int code;
    HipError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

namespace detail {
template <class T, class = void>
struct has_union_genomes : std::false_type {};
template <class T>
struct has_union_genomes<T, std::void_t<decltype(std::declval<const T&>().nUnionGenomes())>> : std::true_type {};
template <class T, class = void>
struct has_genome_major : std::false_type {};
template <class T>
struct has_genome_major<T, std::void_t<decltype(std::declval<const T&>().refGOff()),
                                       decltype(std::declval<const T&>().refGTet())>> : std::true_type {};

struct CtxDeleter {
    void operator()(pfaai_ctx* c) const { pfaai_destroy(c); }
};
using CtxPtr = std::unique_ptr<pfaai_ctx, CtxDeleter>;

// Contexts created ahead of the engine (prewarm_context) wait here for the
// first make_ctx of their device.
struct Parked {
    std::mutex mu;
    std::vector<std::pair<int, pfaai_ctx*>> ctx;
};
inline Parked& parked() {
    static Parked p;
    return p;
}

inline CtxPtr make_ctx(int device) {
    {
        Parked& pk = parked();
        std::lock_guard<std::mutex> lk(pk.mu);
        for (auto it = pk.ctx.begin(); it != pk.ctx.end(); ++it)
            if (it->first == device) {
                pfaai_ctx* c = it->second;
                pk.ctx.erase(it);
                return CtxPtr(c);
            }
    }
    pfaai_ctx* c = nullptr;
    const int rc = pfaai_create(&c, device);
    if (rc) throw HipError(rc, "pfaai_create failed for device " + std::to_string(device) + " (no visible MI355X?)");
    return CtxPtr(c);
}

// Ask for transparent huge pages on a large allocation nothing has touched
// yet: its first touch then faults 2-MB pages instead of 4-KB ones (the
// CLI's C2 output arrays, 64 MB, took ~15 ms of page faults at 4 KB,
// serialised in the kernel's page-table lock however many threads touch
// them).  A hint: no effect where THP is off.
inline void advise_huge(const void* p, std::size_t bytes) {
    const auto a = (reinterpret_cast<std::uintptr_t>(p) + (((std::uintptr_t)1 << 21) - 1)) & ~(((std::uintptr_t)1 << 21) - 1);
    const auto e = reinterpret_cast<std::uintptr_t>(p) + bytes;
    if (e > a + ((std::uintptr_t)1 << 21)) (void)madvise(reinterpret_cast<void*>(a), e - a, MADV_HUGEPAGE);
}

// [0, n) over up to 16 host threads (the adapter's array conversions)
template <class Fn>
void par_range(int64_t n, Fn fn, int max_threads = 16) {
    // >= 64k elements per thread (a 2M-pair JAC fill ran on one thread at the
    // old 4M grain: round-4's C2 "D2H / JAC fill" 25.5 ms)
    const int nt = (int)std::max<int64_t>(
        1, std::min<int64_t>({(int64_t)max_threads, (int64_t)std::thread::hardware_concurrency(), n >> 16}));
    std::vector<std::thread> th;
    int started = 0;
    try {
        for (; started < nt; ++started) th.emplace_back([&, t = started] { fn(n * t / nt, n * (t + 1) / nt); });
    } catch (const std::system_error&) {
        for (int t = started; t < nt; ++t) fn(n * t / nt, n * (t + 1) / nt);
    }
    for (auto& x : th) x.join();
}
}  // namespace detail

// Create device `device`'s context now (the HIP runtime's first
// initialisation, streams, pinned staging, code objects: ~100 ms on a fresh
// process) and keep it for the next engine constructed on that device.  The
// CLI calls it on a helper thread while it reads SQLite.  Thread-safe; false
// if the context could not be created (the engine then reports why).
inline bool prewarm_context(int device) {
    pfaai_ctx* c = nullptr;
    if (pfaai_create(&c, device) != PFAAI_RC_OK) return false;
    detail::Parked& pk = detail::parked();
    std::lock_guard<std::mutex> lk(pk.mu);
    pk.ctx.emplace_back(device, c);
    return true;
}

// Destroy the prewarmed contexts no engine adopted (e.g. the CLI's -q, which
// runs on the first of its devices only): their pinned staging memory,
// streams and buffers.  Returns how many were destroyed.
inline int release_parked_contexts() {
    detail::Parked& pk = detail::parked();
    std::vector<std::pair<int, pfaai_ctx*>> left;
    {
        std::lock_guard<std::mutex> lk(pk.mu);
        left.swap(pk.ctx);
    }
    for (auto& dc : left) pfaai_destroy(dc.second);
    return (int)left.size();
}

// Contiguous row blocks over `parts` devices: cut[0] = 0 .. cut[parts] = n,
// balanced by the row-cost model of parfastaai_amd/shard.py:split_rows (the
// same cuts, pinned by tests/test_adapter_split.py): all-vs-all row a costs
// fixed + width = 0.68 n + (n - 1 - a), times 0.93 for the narrow rows (width
// <= 2047, the 512-thread launch); QT / QSUB rows are equal.  The prefix sums
// are accumulated in row order in double, as numpy's cumsum does.  cus > 0
// (the device's compute units): the round-tail adjustment of shard.py's
// split_rows(cus=...) -- a cut that leaves a block up to a quarter of a round
// (2 * cus row workgroups) past a whole number of rounds, or up to that far
// past the first narrow row, moves back to the boundary.
inline std::vector<int64_t> split_rows(int64_t n, int parts, bool all_vs_all, int cus = 0) {
    std::vector<int64_t> cut{0};
    if (!all_vs_all) {
        for (int r = 1; r < parts; ++r) cut.push_back(n * r / parts);
        cut.push_back(n);
        return cut;
    }
    const double k = 0.68 * (double)n;  // shard.FIXED_COST_FRACTION
    std::vector<double> cum((size_t)n + 1, 0.0);
    for (int64_t a = 0; a < n; ++a) {
        const double width = (double)(n - 1 - a);
        double c = k + width;
        if (width <= 2047.0) c *= 0.93;  // shard.NARROW_COLS, NARROW_COST_FACTOR
        cum[(size_t)a + 1] = cum[(size_t)a] + c;
    }
    const double total = cum[(size_t)n];
    for (int r = 1; r < parts; ++r) {
        const double target = 0.0 + (total - 0.0) * r / parts;
        int64_t i = std::lower_bound(cum.begin(), cum.end(), target) - cum.begin();
        cut.push_back(std::min<int64_t>(std::max<int64_t>(i, cut.back()), n));
    }
    cut.push_back(n);
    if (cus <= 0 || parts <= 1) return cut;
    const int64_t S = 2 * (int64_t)cus;  // shard.ROUND_TAIL = 0.25, NARROW_COLS = 2047
    std::vector<int64_t> edge{0};
    for (int k = 0; k + 1 < parts; ++k) {
        const int64_t a = edge.back();
        int64_t b = cut[(size_t)k + 1];
        const int64_t m = b - a, tail = m % S;
        if (m > S && 0 < tail && (double)tail <= 0.25 * (double)S && n - 1 - (b - 1) > 2047) b -= tail;
        const int64_t narrow0 = n - 1 - 2047;
        if (0 < b - narrow0 && (double)(b - narrow0) <= 0.25 * (double)S) b = narrow0;
        edge.push_back(std::max(a, b));
    }
    edge.push_back(n);
    return edge;
}

// Mode of a DSIT (see the header comment); specialise for other types.
// Works through the abstract DataStructInterface too (the reference's
// PFDSInterface, main.cpp:48): a query-vs-target DSIT numbers its queries
// after its nT targets (ds_impl.hpp:381-383), so none of ids [0, nT) is a
// query; a query subset marks exactly its nQ queries among all genomes
// (ds_impl.hpp:230-232); all-vs-all marks every genome, identity map.
template <class DSIT>
struct pfaai_mode_of {
    static int deduce(const DSIT& ds) {
        if constexpr (detail::has_union_genomes<DSIT>::value) {
            return PFAAI_MODE_QT;
        } else {
            const int64_t nq = (int64_t)ds.qrySetSize(), n = (int64_t)ds.tgtSetSize();
            int64_t marked = 0;
            bool identity = true;
            for (int64_t g = 0; g < n; ++g) {
                if (!ds.isQryGenome((decltype(ds.qrySetSize()))g)) continue;
                ++marked;
                identity = identity && (int64_t)ds.mapQueryId((decltype(ds.qrySetSize()))g) == g;
            }
            if (marked != nq) return PFAAI_MODE_QT;
            return (nq == n && identity) ? PFAAI_MODE_ALL : PFAAI_MODE_QSUB;
        }
    }
};

// Side channel to the engine adapter (ParFAAIHipImpl::upload), which sees
// its DSIT through the reference's abstract interface: a producer that holds
// the genome-major `<p>_genomes` lists (pfaai::DeviceE, pfaai_dropin.hpp)
// hands them over by a cross-cast, and the device builds F from them.
class GenomeMajorSource {
  public:
    virtual ~GenomeMajorSource() = default;
    // the (genome, protein) lists, list (g, p) at g * P + p; nullptr: none
    virtual const std::vector<int64_t>* genomeMajorOff() const = 0;
    virtual const std::vector<int32_t>* genomeMajorTet() const = 0;
};

template <typename IdType, typename ValueType, typename DSIT>
class ParFAAIHipImpl {
  public:
    using JACType = typename DSIT::JACType;

    // the drop-in: ParFAAIImpl(const DSIT&) (algorithm_impl.hpp:75-79), mode
    // deduced, reference-exact (ref_compat), device 0
    // (ParFAAIImpl's callers continue with run() -- main.cpp:193-200, 256-264,
    // 324-332 -- so this constructor prepares computeJAC's host outputs ahead)
    explicit ParFAAIHipImpl(const DSIT& ds)
        : ParFAAIHipImpl(ds, pfaai_mode_of<DSIT>::deduce(ds), std::vector<int>{0}, true, true) {}
    // mode: PFAAI_MODE_ALL / QSUB / QT (the three reference DSIT classes)
    ParFAAIHipImpl(const DSIT& ds, int mode, int device = 0, bool ref_compat = false, bool prepare_ahead = false)
        : ParFAAIHipImpl(ds, mode, std::vector<int>{device}, ref_compat, prepare_ahead) {}
    // Multi-GPU (one process, one context per device, one host thread per
    // context): rows are split by the row-cost model of parfastaai_amd/shard.py
    // and every device writes its rows' JAC span of the shared host arrays
    // (pfaai_compute_rows); ALL, QSUB and QT.
    // prepare_ahead (opt-in, for callers that will call run() / computeJAC()
    // and not stream): computeJAC's host side -- initJAC and the first touch
    // of the output arrays, 44 B a pair -- on a helper thread while the
    // contexts are made and the problem uploads, for outputs of up to
    // kPrepPairs pairs: the CLI's C2 run phase was 21 ms of page faults and
    // initJAC beside 1.6 ms of device work (round 5).  streamAJI /
    // streamMatrix after it free what it prepared.
    ParFAAIHipImpl(const DSIT& ds, int mode, const std::vector<int>& devices, bool ref_compat = false,
                   bool prepare_ahead = false)
        : m_ds(ds), m_mode(mode), m_compat(ref_compat) {
        if (devices.empty()) throw HipError(PFAAI_RC_INVALID, "no device");
        const int64_t np = (int64_t)ds.nGenomePairs();
        if (prepare_ahead && np > 0 && np <= kPrepPairs) {
            try {
                m_prep.t = std::thread([this] {
                    try {
                        prepare_outputs();
                    } catch (...) {
                        m_prepErr = std::current_exception();
                    }
                });
            } catch (const std::system_error&) {  // no thread: computeJAC prepares them itself
            }
        }
        // contexts are owned by RAII handles: a throw below releases them
        m_ctx.push_back(detail::make_ctx(devices[0]));
        for (std::size_t i = 1; i < devices.size(); ++i) m_ctx.push_back(detail::make_ctx(devices[i]));
        upload();
    }
    ParFAAIHipImpl(const ParFAAIHipImpl&) = delete;
    ParFAAIHipImpl& operator=(const ParFAAIHipImpl&) = delete;

    // algorithm_impl.hpp:281-306
    int computeJAC() {
        // the reference's own initJAC (the genome ids of every pair) runs on
        // a host thread while the device computes S / N / AJI
        const auto t0 = std::chrono::steady_clock::now();
        auto ms_since = [](std::chrono::steady_clock::time_point t) {
            return (float)std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
        };
        int64_t rows = 0, pairs = 0;
        pfaai_shape(ctx(), &rows, &pairs);
        const std::size_t n = (std::size_t)pairs;
        join_prep();
        m_prepAhead = m_prepared && m_S && m_JAC.size() == n && m_AJIdev.size() == n;
        std::unique_ptr<double[]> S;
        std::unique_ptr<int32_t[]> N;
        if (m_prepAhead) {
            S = std::move(m_S);
            N = std::move(m_N);
        } else {
            alloc_outputs(n, S, N);
        }
        m_prepared = false;
        m_S.reset();
        m_N.reset();
        const uint32_t flags = m_compat ? PFAAI_FLAG_REF_COMPAT : 0u;
        std::thread ids;
        bool ids_async = !m_prepAhead;
        std::exception_ptr ids_err;  // initJAC's exception, rethrown on this thread
        if (!m_prepAhead) {
            try {
                ids = std::thread([this, &ids_err, t0, ms_since] {
                    try {
                        m_JAC = m_ds.initJAC();
                        m_msIds = ms_since(t0);
                    } catch (...) {
                        ids_err = std::current_exception();
                    }
                });
            } catch (const std::system_error&) {
                ids_async = false;
                m_JAC = m_ds.initJAC();
            }
        }
        int rc = PFAAI_RC_OK;
        std::string err;
        try {
            if (m_ctx.size() == 1) {
                rc = pfaai_compute(ctx(), flags, m_AJIdev.data(), S.get(), N.get());
                if (rc) err = pfaai_last_error(ctx());
            } else {
                computeMulti(flags, S.get(), N.get());
            }
        } catch (...) {
            if (ids_async) ids.join();
            throw;
        }
        m_msCompute = ms_since(t0);
        if (ids_async) ids.join();
        const auto t_fill = std::chrono::steady_clock::now();
        if (ids_err) std::rethrow_exception(ids_err);
        if (rc) throw HipError(rc, err);
        if (m_JAC.size() != n) throw HipError(PFAAI_RC_INVALID, "initJAC size differs from the engine's pair count");
        const bool qt_ids = m_mode == PFAAI_MODE_QT && !m_compat;
        const int64_t nT = m_ds.tgtSetSize();
        detail::par_range((int64_t)n, [&](int64_t lo, int64_t hi) {
            for (int64_t i = lo; i < hi; ++i) {
                if (qt_ids) {  // correct QT ids = the E ids (query nT + q, target t); SURVEY 8a row Q
                    m_JAC[i].genomeA = static_cast<IdType>(nT + i / nT);
                    m_JAC[i].genomeB = static_cast<IdType>(i % nT);
                }
                m_JAC[i].S = S[i];
                m_JAC[i].N = N[i];
            }
        });
        m_msFill = ms_since(t_fill);
        if (m_ctx.size() == 1) {
            pfaai_last_stats(ctx(), &m_events, &m_msBuild, &m_msRows);
            pfaai_run_info(ctx(), &m_rowsKernel, nullptr);
            pfaai_run_walk(ctx(), &m_walk, &m_narrow);
        }
        return 0;  // PFAAI_OK
    }
    // algorithm_impl.hpp:309-322 (the kernel epilogue already divided S / N)
    int computeAJI() {
        join_prep();
        if (m_prepared || m_AJIdev.size() != m_JAC.size() || m_JAC.empty()) {
            if (!m_JAC.empty() && m_AJI.size() == m_JAC.size()) return 0;  // already moved out
            computeJAC();
        }
        if constexpr (std::is_same<ValueType, double>::value) {
            m_AJI.swap(m_AJIdev);  // the device's AJI as it landed (no 8 B-per-pair copy)
            m_AJIdev.clear();
        } else {
            m_AJI.assign(m_AJIdev.begin(), m_AJIdev.end());
        }
        return 0;
    }
    // algorithm_impl.hpp:325-329
    int run() {
        computeJAC();
        computeAJI();
        return 0;
    }
    // Output-tile streaming (pfaai_stream): the AJI vector
    // in JAC-index order written to `path` in the reference's cereal
    // vector<double> format (u64 count + doubles, as PREFIX_aji.bin), tile by
    // tile -- neither the host nor the device holds the whole output.  ALL and
    // QT modes.  Returns 0, or the engine / I/O error code.
    int streamAJI(const std::string& path, int64_t tile_pairs) {
        drop_prepared();
        int64_t rows = 0, pairs = 0;
        int rc = pfaai_shape(ctx(), &rows, &pairs);
        if (rc) throw HipError(rc, pfaai_last_error(ctx()));
        FILE* f = std::fopen(path.c_str(), "wb");
        if (!f) return PFAAI_RC_INVALID;
        const uint64_t n = (uint64_t)pairs;
        bool ok = std::fwrite(&n, 8, 1, f) == 1;
        auto sink = [](void* user, int64_t, int64_t, int64_t, int64_t count, const double* aji, const double*,
                       const int32_t*) -> int {
            return std::fwrite(aji, sizeof(double), (size_t)count, static_cast<FILE*>(user)) == (size_t)count
                       ? 0 : PFAAI_RC_INVALID;
        };
        rc = ok ? pfaai_stream(ctx(), 0, rows, tile_pairs, m_compat ? PFAAI_FLAG_REF_COMPAT : 0u, sink, f)
                : PFAAI_RC_INVALID;
        ok = std::fclose(f) == 0 && ok;
        if (rc) throw HipError(rc, pfaai_last_error(ctx()));
        pfaai_stream_events(ctx(), &m_events);
        return ok ? 0 : PFAAI_RC_INVALID;
    }
    // Dense output rows (pfaai_stream_matrix): printOutput's nQ x nT matrix
    // (main.cpp:143-154), mirror half included, tile by tile to
    // sink(user, row_begin, row_end, n_cols, block) -- the whole matrix is
    // never held.  Returns 0 or throws the engine error.
    int streamMatrix(int64_t tile_rows, pfaai_matrix_sink_fn sink, void* user) {
        drop_prepared();
        int64_t rows = 0;
        int rc = pfaai_shape(ctx(), &rows, nullptr);
        if (!rc) rc = pfaai_stream_matrix(ctx(), 0, rows, tile_rows, m_compat ? PFAAI_FLAG_REF_COMPAT : 0u, sink, user);
        if (rc) throw HipError(rc, pfaai_last_error(ctx()));
        pfaai_stream_events(ctx(), &m_events);
        return 0;
    }
    // (the accessors wait for the constructor's helper thread: it assigns m_JAC)
    const std::vector<JACType>& getJAC() const {
        wait_prep();
        return m_JAC;
    }
    const std::vector<ValueType>& getAJI() const {
        wait_prep();
        return m_AJI;
    }
    // the reference's debug listing (algorithm_impl.hpp:347-356; main.cpp
    // calls it when NDEBUG is not defined)
    void print_aji() const {
        wait_prep();
        std::printf("AJI Ouput : \n [(GP1, GP2,   SUM, NCP) ->  AJI]\n");
        for (std::size_t i = 0; i < m_JAC.size(); ++i)
            std::printf(" [%lld, %.17g -> %03.2f] \n",
                        (long long)m_ds.genomePairToIndex(m_JAC[i].genomeA, m_JAC[i].genomeB), (double)m_AJI[i],
                        (double)m_AJI[i]);
    }
    int64_t nEvents() const { return m_events; }
    // host-side times (ms) of the last computeJAC, from its start: initJAC
    // done (on its thread), the engine's compute + D2H done; and the JAC
    // tuple fill after both
    float msIds() const { return m_msIds; }
    // whether the last computeJAC found initJAC and its output pages made
    // during construction (msIds is then that helper thread's own time)
    bool preparedAhead() const { return m_prepAhead; }
    float msCompute() const { return m_msCompute; }
    float msFill() const { return m_msFill; }
    float msBuild() const { return m_msBuild; }
    float msRows() const { return m_msRows; }
    int mode() const { return m_mode; }
    // PFAAI_ROWS_* of the last run
    int rowsKernel() const { return m_rowsKernel; }
    // PFAAI_WALK_* of the last run, and whether its narrow rows ran beside it
    int walkForm() const { return m_walk; }
    bool narrowLaunch() const { return m_narrow != 0; }
    int nDevices() const { return (int)m_ctx.size(); }
    pfaai_ctx* context() const { return ctx(); }

  private:
    pfaai_ctx* ctx() const { return m_ctx.front().get(); }

    static constexpr int64_t kPrepPairs = (int64_t)1 << 26;  // 44 B a pair: <= 2.75 GiB of host outputs

    // S / N (filled by the device, never value-initialised) and the AJI
    // vector, asking for huge pages before their first touch
    void alloc_outputs(std::size_t n, std::unique_ptr<double[]>& S, std::unique_ptr<int32_t[]>& N) {
        S.reset(new double[n ? n : 1]);
        N.reset(new int32_t[n ? n : 1]);
        detail::advise_huge(S.get(), n * sizeof(double));
        detail::advise_huge(N.get(), n * sizeof(int32_t));
        m_AJIdev.clear();
        m_AJIdev.shrink_to_fit();
        m_AJIdev.reserve(n);  // (untouched: huge pages before the zero fill)
        detail::advise_huge(m_AJIdev.data(), n * sizeof(double));
        m_AJIdev.resize(n);
    }
    // the constructor's helper thread: initJAC, then the outputs allocated and
    // every page of S / N touched (the device's D2H then lands in mapped pages)
    void prepare_outputs() {
        const auto t0 = std::chrono::steady_clock::now();
        m_JAC = m_ds.initJAC();
        const std::size_t n = m_JAC.size();
        alloc_outputs(n, m_S, m_N);
        double* S = m_S.get();
        int32_t* N = m_N.get();
        // on 4 threads: this runs beside the upload's 16 copy threads, and the
        // job's CPU quota (16 on the pool's boxes) throttles every thread of
        // the process once the sum runs over it
        detail::par_range((int64_t)n, [&](int64_t lo, int64_t hi) {
            for (int64_t i = lo; i < hi; i += 512) S[i] = 0.0;  // one store a 4 KB page
            for (int64_t i = lo; i < hi; i += 1024) N[i] = 0;
        }, 4);
        m_msIds = (float)std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        m_prepared = true;
    }
    // the helper thread finished (its error, if any, is rethrown by join_prep)
    void wait_prep() const {
        if (m_prep.t.joinable()) m_prep.t.join();
    }
    void join_prep() {
        wait_prep();
        if (m_prepErr) {
            std::exception_ptr e = m_prepErr;
            m_prepErr = nullptr;
            m_prepared = false;
            std::rethrow_exception(e);
        }
    }
    void drop_prepared() {
        join_prep();
        if (!m_prepared) return;
        m_prepared = false;
        m_S.reset();
        m_N.reset();
        std::vector<JACType>().swap(m_JAC);
        std::vector<double>().swap(m_AJIdev);
    }

    void computeMulti(uint32_t flags, double* S, int32_t* N) {
        int64_t rows = 0, pairs = 0;
        pfaai_shape(ctx(), &rows, &pairs);
        const auto cut = split_rows(rows, (int)m_ctx.size(), m_mode == PFAAI_MODE_ALL);
        std::vector<int> rcs(m_ctx.size(), 0);
        std::vector<std::thread> th;
        for (std::size_t i = 0; i < m_ctx.size(); ++i)
            th.emplace_back([&, i] {
                rcs[i] = pfaai_compute_rows(m_ctx[i].get(), cut[i], cut[i + 1], flags, m_AJIdev.data(), S, N);
            });
        for (auto& t : th) t.join();
        m_events = 0;
        m_msBuild = m_msRows = 0.f;
        for (std::size_t i = 0; i < m_ctx.size(); ++i) {
            if (rcs[i]) throw HipError(rcs[i], pfaai_last_error(m_ctx[i].get()));
            if (cut[i + 1] == cut[i]) continue;
            int64_t e = 0;
            float b = 0.f, r = 0.f;
            pfaai_last_stats(m_ctx[i].get(), &e, &b, &r);
            pfaai_run_info(m_ctx[i].get(), &m_rowsKernel, nullptr);
            pfaai_run_walk(m_ctx[i].get(), &m_walk, &m_narrow);
            m_events += e;
            m_msBuild = std::max(m_msBuild, b);
            m_msRows = std::max(m_msRows, r);
        }
    }

    void upload() {
        const auto& T = m_ds.refT();
        pfaai_problem pb{};
        // a producer's genome-major lists (pfaai::DeviceE's `<p>_genomes`
        // ingest): the device builds F from them, refF() is never asked
        const GenomeMajorSource* gm = nullptr;
        if constexpr (std::is_polymorphic<DSIT>::value) gm = dynamic_cast<const GenomeMajorSource*>(&m_ds);
        if (gm && gm->genomeMajorOff() && gm->genomeMajorTet()) {
            pb.G_off = gm->genomeMajorOff()->data();
            pb.G_tet = gm->genomeMajorTet()->data();
        }
        const bool g_only = pb.G_off != nullptr;
        static const std::vector<typename std::decay_t<decltype(m_ds.refF())>::value_type> kNoF;
        const auto& F = g_only ? kNoF : m_ds.refF();
        const int64_t nf = (int64_t)F.size();
        if constexpr (detail::has_genome_major<DSIT>::value) {
            if (!g_only && (!m_ds.refGTet().empty() || nf == 0)) {
                pb.G_off = m_ds.refGOff().data();
                pb.G_tet = m_ds.refGTet().data();
            }
        }
        if (!g_only && (nf > 0 || !pb.G_off)) {  // F in the reference's layout -> the ABI's columns
            const auto& Lc = m_ds.refLc();
            m_Lp.assign(PFAAI_NTETRAMERS + 1, 0);
            for (int t = 0; t < PFAAI_NTETRAMERS; ++t) m_Lp[t + 1] = m_Lp[t] + (int64_t)Lc[t];
            m_Fp.resize(nf);
            m_Fg.resize(nf);
            detail::par_range(nf, [&](int64_t lo, int64_t hi) {
                for (int64_t i = lo; i < hi; ++i) {
                    m_Fp[i] = F[i].first;
                    m_Fg[i] = F[i].second;
                }
            });
            pb.n_f = nf;
            pb.Lp = m_Lp.data();
            pb.F_prot = m_Fp.data();
            pb.F_genome = m_Fg.data();
        }
        const int64_t P = (int64_t)T.rows(), C = (int64_t)T.cols();
        m_T.resize(P * C);
        for (int64_t p = 0; p < P; ++p)
            for (int64_t g = 0; g < C; ++g) m_T[p * C + g] = T(p, g);
        pb.mode = m_mode;
        pb.n_prot = (int32_t)P;
        pb.t_cols = (int32_t)C;
        pb.T = m_T.data();
        if (m_mode == PFAAI_MODE_ALL) {
            pb.n_ids = (int32_t)m_ds.tgtSetSize();
        } else if (m_mode == PFAAI_MODE_QSUB) {
            const int32_t n = (int32_t)m_ds.tgtSetSize();
            pb.n_ids = n;
            pb.n_qry = (int32_t)m_ds.qrySetSize();
            pb.n_tgt = n - pb.n_qry;
            m_isq.resize(n);
            m_qidx.assign(n, -1);
            m_trank.assign(n, -1);
            for (int32_t g = 0; g < n; ++g) {  // mapQueryId = genome index map (ds_impl.hpp:264)
                m_isq[g] = m_ds.isQryGenome(g) ? 1 : 0;
                (m_isq[g] ? m_qidx[g] : m_trank[g]) = (int32_t)m_ds.mapQueryId(g);
            }
            pb.is_q = m_isq.data();
            pb.q_index = m_qidx.data();
            pb.t_rank = m_trank.data();
        } else {
            pb.n_tgt = (int32_t)m_ds.tgtSetSize();
            pb.n_qry = (int32_t)m_ds.qrySetSize();
            pb.n_ids = pb.n_tgt + pb.n_qry;
            m_isq.assign(pb.n_ids, 0);
            for (int32_t g = pb.n_tgt; g < pb.n_ids; ++g) m_isq[g] = 1;
            pb.is_q = m_isq.data();
        }
        for (auto& c : m_ctx) {
            const int rc = pfaai_load(c.get(), &pb);
            if (rc) throw HipError(rc, pfaai_last_error(c.get()));
        }
        // the devices hold their own copies now
        std::vector<int64_t>().swap(m_Lp);
        std::vector<int32_t>().swap(m_Fp);
        std::vector<int32_t>().swap(m_Fg);
        std::vector<int32_t>().swap(m_T);
    }

    const DSIT& m_ds;
    int m_mode;
    bool m_compat;
    std::vector<detail::CtxPtr> m_ctx;  // one per device; [0] drives single-device runs
    std::vector<int64_t> m_Lp;
    std::vector<int32_t> m_Fp, m_Fg, m_T, m_qidx, m_trank;
    std::vector<uint8_t> m_isq;
    std::vector<JACType> m_JAC;
    std::vector<double> m_AJIdev;
    float m_msIds = 0.f, m_msCompute = 0.f, m_msFill = 0.f;
    std::vector<ValueType> m_AJI;
    int64_t m_events = 0;
    float m_msBuild = 0.f, m_msRows = 0.f;
    int32_t m_rowsKernel = -1;
    int32_t m_walk = PFAAI_WALK_NONE, m_narrow = 0;
    // the constructor's output preparation (prepare_outputs)
    std::unique_ptr<double[]> m_S;
    std::unique_ptr<int32_t[]> m_N;
    bool m_prepared = false, m_prepAhead = false;
    std::exception_ptr m_prepErr;
    struct Joiner {  // joined before the members above are destroyed (a throwing constructor included)
        std::thread t;
        ~Joiner() {
            if (t.joinable()) t.join();
        }
    };
    mutable Joiner m_prep;  // (joined by the const accessors too)
};

}  // namespace pfaai

// the producer half of the drop-in: pfaai::DeviceE<DS> (it uses the adapter's
// helpers above, and the adapter takes its lists through GenomeMajorSource)
#include "pfaai_dropin.hpp"
