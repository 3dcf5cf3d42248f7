// datastruct.hpp -- host mirror of the reference's three DataStructInterface
// modes (ds_impl.hpp), holding the loader's arrays and the mode's index maps.
// They expose exactly the accessors pfaai::ParFAAIHipImpl (include/
// pfaai_hip.hpp) and printOutput need, with the reference's names.
#pragma once
#include <sys/mman.h>

#include <algorithm>
#include <cstdint>
#include <string>
#include <system_error>
#include <thread>
#include <unordered_map>
#include <vector>

#include "scp_db.hpp"

namespace pfaai_host {

struct JACTuple {  // JACTuple<int, double>, interface.hpp:61-75
    int32_t genomeA, genomeB;
    double S;
    int32_t N;
    // no zero-fill on construction: initJAC writes every field, in parallel
    // (a vector of n value-initialised tuples is a serial 24n-byte memset)
    JACTuple() {}
    JACTuple(int32_t a, int32_t b, double s, int32_t n) : genomeA(a), genomeB(b), S(s), N(n) {}
};

// transparent huge pages for an untouched allocation (see pfaai::detail::advise_huge)
inline void advise_huge(const void* p, std::size_t bytes) {
    const auto a = (reinterpret_cast<std::uintptr_t>(p) + (((std::uintptr_t)1 << 21) - 1)) & ~(((std::uintptr_t)1 << 21) - 1);
    const auto e = reinterpret_cast<std::uintptr_t>(p) + bytes;
    if (e > a + ((std::uintptr_t)1 << 21)) (void)madvise(reinterpret_cast<void*>(a), e - a, MADV_HUGEPAGE);
}

// fn(lo, hi) over [0, n) on up to 4 threads (>= 64k items each): initJAC runs
// beside the upload's copy threads (the job's CPU quota is 16 on the pool's boxes)
// A slice whose thread cannot be created (std::system_error) runs on the
// calling thread; the threads that did start are always joined.
template <class Fn>
void par_items(int64_t n, Fn fn) {
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>({4, (int64_t)std::thread::hardware_concurrency(), n >> 16}));
    std::vector<std::thread> th;
    th.reserve(nt);
    int started = 1;
    try {
        for (; started < nt; ++started) {
            const int t = started;
            th.emplace_back([&, t] { fn(n * t / nt, n * (t + 1) / nt); });
        }
    } catch (const std::system_error&) {
    }
    fn(0, n / nt);
    for (int t = started; t < nt; ++t) fn(n * t / nt, n * (t + 1) / nt);
    for (auto& x : th) x.join();
}

class DataBase {
  public:
    using JACType = JACTuple;
    DataBase(DBMetaData meta, LoadedArrays arr) : m_meta(std::move(meta)), m_arr(std::move(arr)) {
        if (m_arr.Lc.empty()) m_arr.Lc.assign(kNTetramers, 0);  // G path: F is built on the device
        m_Lp.assign(kNTetramers, 0);
        int32_t run = 0;
        for (int t = 0; t < kNTetramers; ++t) {  // parallelPrefixSum, ds_helper.hpp:112-122
            m_Lp[t] = run;
            run += m_arr.Lc[t];
        }
    }
    const std::vector<int32_t>& refLc() const { return m_arr.Lc; }
    const std::vector<int32_t>& refLp() const { return m_Lp; }
    const std::vector<DPair>& refF() const { return m_arr.F; }
    const DMatrix& refT() const { return m_arr.T; }
    // genome-major `<p>_genomes` lists (G path; empty on the F path)
    const std::vector<int64_t>& refGOff() const { return m_arr.G_off; }
    const std::vector<int32_t>& refGTet() const { return m_arr.G_tet; }
    const DBMetaData& meta() const { return m_meta; }

  protected:
    DBMetaData m_meta;
    LoadedArrays m_arr;
    std::vector<int32_t> m_Lp;
};

// ParFAAIData (ds_impl.hpp:38-151)
class AllData : public DataBase {
  public:
    using DataBase::DataBase;
    int64_t n() const { return (int64_t)m_meta.genomeSet.size(); }
    const std::vector<std::string>& refQuerySet() const { return m_meta.genomeSet; }
    const std::vector<std::string>& refTargetSet() const { return m_meta.genomeSet; }
    int64_t qrySetSize() const { return n(); }
    int64_t tgtSetSize() const { return n(); }
    int64_t nGenomePairs() const { return n() * (n() - 1) / 2; }
    bool isQryGenome(int32_t) const { return true; }
    int32_t mapQueryId(int32_t g) const { return g; }
    int32_t mapTargetId(int32_t g) const { return g; }
    // pair k of row a (columns a+1..n-1) sits at n a - a (a + 1) / 2 + b - a - 1
    // (ds_impl.hpp:83-86); each thread finds its first pair's row by
    // bisection and walks on
    std::vector<JACType> initJAC() const {
        std::vector<JACType> j(nGenomePairs());
        advise_huge(j.data(), j.size() * sizeof(JACType));
        const int64_t nn = n();
        auto first = [nn](int64_t a) { return nn * a - a * (a + 1) / 2; };
        par_items((int64_t)j.size(), [&](int64_t lo, int64_t hi) {
            int64_t a0 = 0, a1 = nn - 1;  // the row holding pair lo: first(a) <= lo < first(a + 1)
            while (a0 < a1) {
                const int64_t m = (a0 + a1 + 1) / 2;
                if (first(m) <= lo) a0 = m; else a1 = m - 1;
            }
            int32_t a = (int32_t)a0, b = (int32_t)(a0 + 1 + lo - first(a0));
            for (int64_t k = lo; k < hi; ++k) {
                j[k] = JACType{a, b, 0.0, 0};
                if (b == nn - 1) { ++a; b = a + 1; } else { ++b; }
            }
        });
        return j;
    }
};

// ParFAAIQSubData (ds_impl.hpp:158-337)
class QSubData : public DataBase {
  public:
    QSubData(DBMetaData meta, LoadedArrays arr, std::vector<std::string> qry)
        : DataBase(std::move(meta), std::move(arr)), m_qry(std::move(qry)) {
        const int32_t n = (int32_t)m_meta.genomeSet.size();
        std::unordered_map<std::string, int32_t> qpos;
        for (std::size_t i = 0; i < m_qry.size(); ++i) qpos.emplace(m_qry[i], (int32_t)i);
        m_isq.assign(n, 0);
        m_map.assign(n, 0);
        m_qlook.assign(m_qry.size(), 0);
        for (int32_t ix = 0, jx = 0; ix < n; ++ix) {
            auto it = qpos.find(m_meta.genomeSet[ix]);
            if (it != qpos.end()) {
                m_isq[ix] = 1;
                m_qlook[it->second] = ix;
                m_map[ix] = it->second;
            } else {
                m_tlook.push_back(ix);
                m_map[ix] = jx++;
            }
        }
    }
    const std::vector<std::string>& refQuerySet() const { return m_qry; }
    const std::vector<std::string>& refTargetSet() const { return m_meta.genomeSet; }
    int64_t qrySetSize() const { return (int64_t)m_qry.size(); }
    int64_t tgtSetSize() const { return (int64_t)m_meta.genomeSet.size(); }
    int64_t nTgt() const { return tgtSetSize() - qrySetSize(); }
    int64_t nGenomePairs() const { return qrySetSize() * nTgt() + qrySetSize() * (qrySetSize() - 1) / 2; }
    bool isQryGenome(int32_t g) const { return m_isq[g]; }
    int32_t mapQueryId(int32_t g) const { return m_map[g]; }
    int32_t mapTargetId(int32_t g) const { return g; }
    std::vector<JACType> initJAC() const {
        std::vector<JACType> j(nGenomePairs(), JACType{0, 0, 0.0, 0});
        const int64_t qt = qrySetSize() * nTgt();
        par_items(qt, [&](int64_t lo, int64_t hi) {
            for (int64_t i = lo; i < hi; ++i) {
                j[i].genomeA = m_qlook[i / nTgt()];
                j[i].genomeB = m_tlook[i % nTgt()];
            }
        });
        int32_t a = 0, b = 1;
        for (int64_t i = qt; i < (int64_t)j.size(); ++i) {
            j[i].genomeA = m_qlook[a];
            j[i].genomeB = m_qlook[b];
            if (b == qrySetSize() - 1) { ++a; b = a + 1; } else { ++b; }
        }
        return j;
    }

  private:
    std::vector<std::string> m_qry;
    std::vector<uint8_t> m_isq;
    std::vector<int32_t> m_map, m_qlook, m_tlook;
};

// ParFAAIQryTgtData (ds_impl.hpp:343-490): targets 0..nT-1, queries nT..
class QTData : public DataBase {
  public:
    using DataBase::DataBase;
    const std::vector<std::string>& refQuerySet() const { return m_meta.qyGenomeSet; }
    const std::vector<std::string>& refTargetSet() const { return m_meta.genomeSet; }
    int64_t qrySetSize() const { return (int64_t)m_meta.qyGenomeSet.size(); }
    int64_t tgtSetSize() const { return (int64_t)m_meta.genomeSet.size(); }
    int64_t nGenomePairs() const { return qrySetSize() * tgtSetSize(); }
    int64_t nUnionGenomes() const { return qrySetSize() + tgtSetSize(); }  // ds_impl.hpp:370
    bool isQryGenome(int32_t g) const { return g >= tgtSetSize(); }
    int32_t mapQueryId(int32_t g) const { return g < tgtSetSize() ? g : (int32_t)(g - tgtSetSize()); }
    int32_t mapTargetId(int32_t g) const { return mapQueryId(g); }
    // the reference's ids (i/nT, nQ + i%nT), ds_impl.hpp:434-436
    std::vector<JACType> initJAC() const {
        std::vector<JACType> j(nGenomePairs());
        advise_huge(j.data(), j.size() * sizeof(JACType));
        const int64_t nT = tgtSetSize(), nQ = qrySetSize();
        par_items((int64_t)j.size(), [&](int64_t lo, int64_t hi) {
            for (int64_t i = lo; i < hi; ++i) j[i] = JACType{(int32_t)(i / nT), (int32_t)(nQ + i % nT), 0.0, 0};
        });
        return j;
    }
};

}  // namespace pfaai_host
