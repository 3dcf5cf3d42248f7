// pfaai_hip.hpp -- C++ adapter with the reference's ParFAAIImpl surface over
// the C ABI of libpfaai_hip.so.
//
// Drop-in for  ParFAAIImpl<IdType, ValueType, DSIT>
//              (reference include/pfaai/algorithm_impl.hpp:38-357):
//   explicit ParFAAIHipImpl(const DSIT&);  int run();  int computeJAC();
//   int computeAJI();  const std::vector<JACType>& getJAC() const;
//   const std::vector<ValueType>& getAJI() const;
// DSIT is any type with the reference's DataStructInterface accessors
// (interface.hpp:200-328): refLp(), refLc(), refF() (elements with .first/
// .second), refT() (operator()(p, g), rows(), cols()), initJAC(),
// nGenomePairs(), qrySetSize(), tgtSetSize(), isQryGenome(), mapQueryId(),
// plus the JACType typedef -- the reference's own ParFAAIData /
// ParFAAIQSubData / ParFAAIQryTgtData qualify unchanged, and so do the host
// classes of parfastaai_amd/host/datastruct.hpp.  The mode is deduced from the
// DSIT (pfaai_mode_of<DSIT>) or passed explicitly.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <thread>
#include <stdexcept>
#include <string>
#include <vector>

#include "pfaai_hip.h"

namespace pfaai {

struct HipError : std::runtime_error {
    int code;
    HipError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

template <typename IdType, typename ValueType, typename DSIT>
class ParFAAIHipImpl {
  public:
    using JACType = typename DSIT::JACType;

    // mode: PFAAI_MODE_ALL / QSUB / QT (the three reference DSIT classes)
    explicit ParFAAIHipImpl(const DSIT& ds, int mode, int device = 0, bool ref_compat = false)
        : m_ds(ds), m_mode(mode), m_compat(ref_compat) {
        int rc = pfaai_create(&m_ctx, device);
        if (rc) throw HipError(rc, "pfaai_create failed (no visible MI355X?)");
        upload();
    }
    // Multi-GPU (one process, one context per device, one host thread per
    // context): rows are split by the row-cost model of parfastaai_amd/shard.py
    // and every device writes its rows' JAC span of the shared host arrays
    // (pfaai_compute_rows); ALL and QT -- QSUB runs on devices[0].
    ParFAAIHipImpl(const DSIT& ds, int mode, const std::vector<int>& devices, bool ref_compat = false)
        : m_ds(ds), m_mode(mode), m_compat(ref_compat) {
        if (devices.empty()) throw HipError(PFAAI_ERR_INVALID, "no device");
        int rc = pfaai_create(&m_ctx, devices[0]);
        if (rc) throw HipError(rc, "pfaai_create failed (no visible MI355X?)");
        for (std::size_t i = 1; i < devices.size() && mode != PFAAI_MODE_QSUB; ++i) {
            pfaai_ctx* x = nullptr;
            rc = pfaai_create(&x, devices[i]);
            if (rc) throw HipError(rc, "pfaai_create failed for device " + std::to_string(devices[i]));
            m_extra.push_back(x);
        }
        upload();
    }
    ~ParFAAIHipImpl() {
        pfaai_destroy(m_ctx);
        for (pfaai_ctx* x : m_extra) pfaai_destroy(x);
    }
    ParFAAIHipImpl(const ParFAAIHipImpl&) = delete;
    ParFAAIHipImpl& operator=(const ParFAAIHipImpl&) = delete;

    // algorithm_impl.hpp:281-306
    int computeJAC() {
        m_JAC = m_ds.initJAC();
        if (m_mode == PFAAI_MODE_QT && !m_compat) {
            // correct QT ids = the E ids (query nT + q, target t); SURVEY 8a row Q
            const int64_t nT = m_ds.tgtSetSize();
            for (std::size_t i = 0; i < m_JAC.size(); ++i) {
                m_JAC[i].genomeA = static_cast<IdType>(nT + (int64_t)i / nT);
                m_JAC[i].genomeB = static_cast<IdType>((int64_t)i % nT);
            }
        }
        const std::size_t n = m_JAC.size();
        std::vector<double> S(n);
        std::vector<int32_t> N(n);
        m_AJIdev.resize(n);
        const uint32_t flags = m_compat ? PFAAI_FLAG_REF_COMPAT : 0u;
        if (m_extra.empty()) {
            int rc = pfaai_compute(m_ctx, flags, m_AJIdev.data(), S.data(), N.data());
            if (rc) throw HipError(rc, pfaai_last_error(m_ctx));
        } else {
            computeMulti(flags, S.data(), N.data());
        }
        for (std::size_t i = 0; i < n; ++i) {
            m_JAC[i].S = S[i];
            m_JAC[i].N = N[i];
        }
        if (m_extra.empty()) pfaai_last_stats(m_ctx, &m_events, &m_msBuild, &m_msRows);
        return 0;  // PFAAI_OK
    }
    // algorithm_impl.hpp:309-322 (the kernel epilogue already divided S / N)
    int computeAJI() {
        if (m_AJIdev.size() != m_JAC.size() || m_JAC.empty()) computeJAC();
        m_AJI.assign(m_AJIdev.begin(), m_AJIdev.end());
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
        int64_t rows = 0, pairs = 0;
        int rc = pfaai_shape(m_ctx, &rows, &pairs);
        if (rc) throw HipError(rc, pfaai_last_error(m_ctx));
        FILE* f = std::fopen(path.c_str(), "wb");
        if (!f) return PFAAI_ERR_INVALID;
        const uint64_t n = (uint64_t)pairs;
        bool ok = std::fwrite(&n, 8, 1, f) == 1;
        auto sink = [](void* user, int64_t, int64_t, int64_t, int64_t count, const double* aji, const double*,
                       const int32_t*) -> int {
            return std::fwrite(aji, sizeof(double), (size_t)count, static_cast<FILE*>(user)) == (size_t)count
                       ? 0 : PFAAI_ERR_INVALID;
        };
        rc = ok ? pfaai_stream(m_ctx, 0, rows, tile_pairs, m_compat ? PFAAI_FLAG_REF_COMPAT : 0u, sink, f)
                : PFAAI_ERR_INVALID;
        ok = std::fclose(f) == 0 && ok;
        if (rc) throw HipError(rc, pfaai_last_error(m_ctx));
        pfaai_stream_events(m_ctx, &m_events);
        return ok ? 0 : PFAAI_ERR_INVALID;
    }
    const std::vector<JACType>& getJAC() const { return m_JAC; }
    const std::vector<ValueType>& getAJI() const { return m_AJI; }
    int64_t nEvents() const { return m_events; }
    float msBuild() const { return m_msBuild; }
    float msRows() const { return m_msRows; }

    int nDevices() const { return 1 + (int)m_extra.size(); }

  private:
    // contiguous row blocks balanced by the row-cost model (shard.py:split_rows)
    static std::vector<int64_t> splitRows(int64_t n, int parts, bool all_vs_all) {
        std::vector<int64_t> cut{0};
        const double k = 0.75 * (double)n;  // shard.FIXED_COST_FRACTION
        auto before = [&](int64_t a) {
            return all_vs_all ? (double)a * k + (double)a * n - (double)a * (a + 1) / 2.0 : (double)a;
        };
        const double total = before(n);
        for (int r = 1; r < parts; ++r) {
            int64_t lo = cut.back(), hi = n;
            const double target = total * r / parts;
            while (lo < hi) {
                const int64_t mid = (lo + hi) / 2;
                if (before(mid) < target) lo = mid + 1; else hi = mid;
            }
            cut.push_back(lo);
        }
        cut.push_back(n);
        return cut;
    }
    void computeMulti(uint32_t flags, double* S, int32_t* N) {
        int64_t rows = 0, pairs = 0;
        pfaai_shape(m_ctx, &rows, &pairs);
        std::vector<pfaai_ctx*> ctx{m_ctx};
        ctx.insert(ctx.end(), m_extra.begin(), m_extra.end());
        const auto cut = splitRows(rows, (int)ctx.size(), m_mode == PFAAI_MODE_ALL);
        std::vector<int> rcs(ctx.size(), 0);
        std::vector<std::thread> th;
        for (std::size_t i = 0; i < ctx.size(); ++i)
            th.emplace_back([&, i] {
                rcs[i] = pfaai_compute_rows(ctx[i], cut[i], cut[i + 1], flags, m_AJIdev.data(), S, N);
            });
        for (auto& t : th) t.join();
        m_events = 0;
        m_msBuild = m_msRows = 0.f;
        for (std::size_t i = 0; i < ctx.size(); ++i) {
            if (rcs[i]) throw HipError(rcs[i], pfaai_last_error(ctx[i]));
            if (cut[i + 1] == cut[i]) continue;
            int64_t e = 0;
            float b = 0.f, r = 0.f;
            pfaai_last_stats(ctx[i], &e, &b, &r);
            m_events += e;
            m_msBuild = std::max(m_msBuild, b);
            m_msRows = std::max(m_msRows, r);
        }
    }

    void upload() {
        const auto& Lp32 = m_ds.refLp();
        const auto& Lc = m_ds.refLc();
        const auto& F = m_ds.refF();
        const auto& T = m_ds.refT();
        const int64_t nf = (int64_t)F.size();
        m_Lp.assign(PFAAI_NTETRAMERS + 1, 0);
        for (int t = 0; t < PFAAI_NTETRAMERS; ++t) m_Lp[t + 1] = m_Lp[t] + (int64_t)Lc[t];
        (void)Lp32;
        m_Fp.resize(nf);
        m_Fg.resize(nf);
        for (int64_t i = 0; i < nf; ++i) {
            m_Fp[i] = F[i].first;
            m_Fg[i] = F[i].second;
        }
        const int64_t P = (int64_t)T.rows(), C = (int64_t)T.cols();
        m_T.resize(P * C);
        for (int64_t p = 0; p < P; ++p)
            for (int64_t g = 0; g < C; ++g) m_T[p * C + g] = T(p, g);
        pfaai_problem pb{};
        pb.mode = m_mode;
        pb.n_prot = (int32_t)P;
        pb.t_cols = (int32_t)C;
        pb.n_f = nf;
        pb.Lp = m_Lp.data();
        pb.F_prot = m_Fp.data();
        pb.F_genome = m_Fg.data();
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
        int rc = pfaai_load(m_ctx, &pb);
        if (rc) throw HipError(rc, pfaai_last_error(m_ctx));
        for (pfaai_ctx* x : m_extra)
            if ((rc = pfaai_load(x, &pb))) throw HipError(rc, pfaai_last_error(x));
    }

    const DSIT& m_ds;
    int m_mode;
    bool m_compat;
    pfaai_ctx* m_ctx = nullptr;
    std::vector<pfaai_ctx*> m_extra;  // further devices (multi-GPU constructor)
    std::vector<int64_t> m_Lp;
    std::vector<int32_t> m_Fp, m_Fg, m_T, m_qidx, m_trank;
    std::vector<uint8_t> m_isq;
    std::vector<JACType> m_JAC;
    std::vector<double> m_AJIdev;
    std::vector<ValueType> m_AJI;
    int64_t m_events = 0;
    float m_msBuild = 0.f, m_msRows = 0.f;
};

}  // namespace pfaai
