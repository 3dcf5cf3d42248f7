// pfaai_dropin.hpp -- the producer half of the drop-in:
// pfaai::DeviceE<DS> wraps each of the reference's DataStructInterface
// classes (ParFAAIData / ParFAAIQSubData / ParFAAIQryTgtData, ds_impl.hpp)
// so that construct() (interface.hpp:306-327) no longer spends its time
// where the engine does not need it.  Included by pfaai_hip.hpp.
//
//   constructE   (ds_helper.hpp:362-421 + psort.hpp:27-53, 86 % of the
//                reference's wall time at C2): not built -- the engine never
//                reads E (refE()).
//   constructL / constructF / constructT (ds_helper.hpp:46-162 over the
//                SQLite UNION ALL + ORDER BY of scp_db.hpp:161-262, 10-17 s
//                at C2; VERDICT r05 missing #2): the `<p>_genomes` lists read
//                over per-protein connections on all threads
//                (parfastaai_amd/host/scp_db.hpp load_single_g, the CLI's
//                ingest, with its exact orientation check against the
//                `<p>_tetras` blobs); Lc, Lp and T follow from the lists, and
//                the engine builds F on the device from them (the G-only
//                load: the benchmarked k_rows_pl form).  F in the
//                reference's layout is assembled on the host only if someone
//                asks for it (refF()), so refLc / refLp / refF / refT keep
//                their meaning.
//
// The fast path applies to the single-DB classes (all-vs-all, -q), whose DB
// interface names its file (getDBPath, scp_db.hpp:100); a query-vs-target
// DB interface does not expose its query file, so ParFAAIQryTgtData keeps
// the reference's own L / F / T construction (and still skips E).  Any
// disagreement -- a DB whose two orientations differ, protein or genome
// order unlike the reference's metadata, a read error -- also falls back
// to the reference's construction, so the produced arrays are the
// reference's in every case.
#pragma once
#include <omp.h>

#include <atomic>
#include <cstdint>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <utility>
#include <vector>

#include "../parfastaai_amd/host/scp_db.hpp"
#include "pfaai_hip.hpp"  // (includes this header at its end: either order works)

namespace pfaai {

template <class DS>
class DeviceE : public DS, public GenomeMajorSource {
  public:
    using IdPairType = typename DS::IdPairType;
    using IdType = std::remove_cv_t<std::remove_reference_t<decltype(std::declval<IdPairType&>().first)>>;
    using ErrT = decltype(std::declval<DS&>().constructE());

    // the reference classes' constructors: (DB interface, DB metadata, ...)
    template <class DBI, class Meta, class... Rest>
    DeviceE(const DBI& db, const Meta& meta, Rest&&... rest) : DS(db, meta, std::forward<Rest>(rest)...) {
        if constexpr (!detail::has_union_genomes<DS>::value) {
            m_path = db.getDBPath();
            m_proteins = &meta.proteinSet;
            m_genomes = &meta.genomeSet;
            m_try = true;
        }
    }
    ~DeviceE() override {
        if (m_warm.joinable()) m_warm.join();
        release_parked_contexts();  // a prewarmed context no engine adopted
    }

    ErrT constructL() override {
        if (!m_try) return DS::constructL();
        // the HIP runtime's first initialisation and device 0's context
        // (the one-argument engine's) beside the SQLite read; the engine
        // adopts it (prewarm_context)
        try {
            m_warm = std::thread([] { prewarm_context(0); });
        } catch (const std::system_error&) {
        }
        const bool ok = ingest();
        if (m_warm.joinable()) m_warm.join();  // parked before the engine is made
        if (!ok) return DS::constructL();
        this->m_initFlags["L"] = true;
        return (this->m_errorCode = ErrT{});
    }
    ErrT constructF() override {
        if (!m_fast) return DS::constructF();
        this->m_initFlags["F"] = true;  // built on demand (refF) or on the device
        return ErrT{};
    }
    ErrT constructT() override {
        if (!m_fast) return DS::constructT();
        this->m_initFlags["T"] = true;  // from the list lengths (ingest)
        return ErrT{};
    }
    // the engine never reads E
    ErrT constructE() override { return ErrT{}; }

    // F in the reference's layout, (tetramer, protein, genome) order
    // (ds_helper.hpp:126-162), assembled from the lists on first use
    const std::vector<IdPairType>& refF() const override {
        if (m_fast) std::call_once(m_fOnce, [this] { const_cast<DeviceE*>(this)->assembleF(); });
        return DS::refF();
    }
    const std::vector<int64_t>* genomeMajorOff() const override { return m_fast ? &m_gOff : nullptr; }
    const std::vector<int32_t>* genomeMajorTet() const override { return m_fast ? &m_gTet : nullptr; }
    // whether construct() took the `<p>_genomes` ingest
    bool fastIngest() const { return m_fast; }

  private:
    bool ingest() {
        pfaai_host::DBMetaData hm;
        pfaai_host::LoadedArrays arr;
        std::string err;
        if (pfaai_host::load_single_g(m_path, hm, arr, err) != 0) return false;
        // the same protein and genome numbering as the reference's metadata
        // (db_helper.hpp:86-106, 195-215)
        if (hm.proteinSet != *m_proteins || hm.genomeSet != *m_genomes) return false;
        const int64_t P = (int64_t)hm.proteinSet.size(), G = (int64_t)hm.genomeSet.size();
        const int64_t nT = (int64_t)pfaai_host::kNTetramers;
        // Lc[t] = lists holding t (constructLc, ds_helper.hpp:82-110), per-thread counts
        const int nth = std::max(1, omp_get_max_threads());
        std::vector<std::vector<IdType>> part((std::size_t)nth);
        const std::vector<int32_t>& tet = arr.G_tet;
        const int64_t n = (int64_t)tet.size();
#pragma omp parallel num_threads(nth)
        {
            const int t = omp_get_thread_num(), k = omp_get_num_threads();
            std::vector<IdType>& c = part[(std::size_t)t];
            c.assign((std::size_t)nT, 0);
            for (int64_t i = n * t / k; i < n * (t + 1) / k; ++i) ++c[(std::size_t)tet[(std::size_t)i]];
        }
        this->m_Lc.assign((std::size_t)nT, 0);
        for (const auto& c : part)
            if (!c.empty())
                for (int64_t t = 0; t < nT; ++t) this->m_Lc[(std::size_t)t] += c[(std::size_t)t];
        // Lp = exclusive prefix of Lc (parallelPrefixSum, ds_helper.hpp:112-122)
        this->m_Lp.assign((std::size_t)nT, 0);
        IdType run = 0;
        for (int64_t t = 0; t < nT; ++t) {
            this->m_Lp[(std::size_t)t] = run;
            run += this->m_Lc[(std::size_t)t];
        }
        // T(p, g) = tetramers of protein p in genome g (constructT, ds_helper.hpp:46-79)
        for (int64_t p = 0; p < P; ++p)
            for (int64_t g = 0; g < G; ++g)
                this->m_T((std::size_t)p, (std::size_t)g) = (IdType)arr.T((std::size_t)p, (std::size_t)g);
        m_gOff = std::move(arr.G_off);
        m_gTet = std::move(arr.G_tet);
        m_P = P;
        m_G = G;
        m_fast = true;
        return true;
    }
    // counting placement by tetramer, protein-major then genome-major, so a
    // block's entries land in (protein, genome) order
    void assembleF() {
        std::vector<int64_t> cur((std::size_t)pfaai_host::kNTetramers);
        for (std::size_t t = 0; t < cur.size(); ++t) cur[t] = (int64_t)this->m_Lp[t];
        auto& F = this->m_F;
        F.assign(m_gTet.size(), IdPairType{});
        for (int64_t p = 0; p < m_P; ++p)
            for (int64_t g = 0; g < m_G; ++g) {
                const int64_t k = g * m_P + p;
                for (int64_t i = m_gOff[(std::size_t)k]; i < m_gOff[(std::size_t)k + 1]; ++i) {
                    IdPairType& e = F[(std::size_t)cur[(std::size_t)m_gTet[(std::size_t)i]]++];
                    e.first = (IdType)p;
                    e.second = (IdType)g;
                }
            }
    }

    std::string m_path;
    const std::vector<std::string>* m_proteins = nullptr;
    const std::vector<std::string>* m_genomes = nullptr;
    bool m_try = false, m_fast = false;
    int64_t m_P = 0, m_G = 0;
    std::vector<int64_t> m_gOff;
    std::vector<int32_t> m_gTet;
    mutable std::once_flag m_fOnce;
    std::thread m_warm;
};

}  // namespace pfaai
