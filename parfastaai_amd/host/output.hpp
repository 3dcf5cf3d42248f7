// output.hpp -- the reference's output formats, produced in parallel.
//
//  * CSV (printOutput, main.cpp:133-175): dense nQ x nT AJI matrix filled
//    from the JAC tuples (mirrored when isSubset and genomeB is a query),
//    header `sep + join(targets, sep)`, rows `name sep join(values, sep)`.
//    Doubles are printed like fmt 10's `{}`: shortest round-trip digits,
//    fixed notation iff -4 <= exp10 < 16, integral values without ".0".
//    Rows are formatted by all OpenMP threads into per-row buffers and
//    written in order (the reference formats single-threaded).
//  * --bin: cereal BinaryOutputArchive of std::vector<JACTuple<int,double>>
//    and std::vector<double> (the golden-vector format of the reference's
//    tests, interface.hpp:72-74), plus the dense DMatrix<double>.
#pragma once
#include <omp.h>

#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <string>
#include <vector>

namespace pfaai_host {

// fmt 10 `{}` of a double.  Returns the number of chars written to out
// (>= 32 bytes available).
inline int fmt_double(double v, char* out) {
    if (std::isnan(v)) { std::memcpy(out, "nan", 3); return 3; }
    if (std::isinf(v)) {
        if (v < 0) { std::memcpy(out, "-inf", 4); return 4; }
        std::memcpy(out, "inf", 3);
        return 3;
    }
    char tmp[40];
    auto r = std::to_chars(tmp, tmp + sizeof(tmp), v, std::chars_format::scientific);  // shortest digits
    *r.ptr = '\0';
    int o = 0;
    const char* q = tmp;
    if (*q == '-') out[o++] = *q++;
    char dig[24];
    int nd = 0;
    while (*q && *q != 'e') {
        if (*q != '.') dig[nd++] = *q;
        ++q;
    }
    const int e = std::atoi(q + 1);
    if (nd == 1 && dig[0] == '0') {  // +-0
        out[o++] = '0';
        return o;
    }
    if (e >= -4 && e < 16) {
        if (e >= 0) {
            for (int k = 0; k <= e; ++k) out[o++] = k < nd ? dig[k] : '0';
            if (nd > e + 1) {
                out[o++] = '.';
                for (int k = e + 1; k < nd; ++k) out[o++] = dig[k];
            }
        } else {
            out[o++] = '0';
            out[o++] = '.';
            for (int k = 0; k < -e - 1; ++k) out[o++] = '0';
            for (int k = 0; k < nd; ++k) out[o++] = dig[k];
        }
    } else {
        out[o++] = dig[0];
        if (nd > 1) {
            out[o++] = '.';
            for (int k = 1; k < nd; ++k) out[o++] = dig[k];
        }
        out[o++] = 'e';
        int ae = e;
        if (ae < 0) { out[o++] = '-'; ae = -ae; } else { out[o++] = '+'; }
        if (ae < 10) out[o++] = '0';
        char eb[8];
        int ne = std::snprintf(eb, sizeof(eb), "%d", ae);
        std::memcpy(out + o, eb, ne);
        o += ne;
    }
    return o;
}

// printOutput's dense fill (main.cpp:143-154)
template <typename DS, typename JAC>
std::vector<double> dense_matrix(const DS& ds, const std::vector<JAC>& jac, const std::vector<double>& aji,
                                 bool isSubset) {
    const int64_t nq = ds.qrySetSize(), nt = ds.tgtSetSize();
    std::vector<double> M((std::size_t)(nq * nt), 0.0);
    if (!isSubset) {  // QT: the reference's ids (ref-compat) land off their row when nQ > nT: flat,
                      // bounds-checked, and in JAC order there (later pairs overwrite, as main.cpp:149 does)
#pragma omp parallel for schedule(static) if (nq <= nt)
        for (int64_t i = 0; i < (int64_t)jac.size(); ++i) {
            const int64_t f = (int64_t)ds.mapQueryId(jac[i].genomeA) * nt + ds.mapTargetId(jac[i].genomeB);
            if (f >= 0 && f < nq * nt) M[(std::size_t)f] = aji[i];
        }
        return M;
    }
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)jac.size(); ++i) {
        const int32_t a = jac[i].genomeA, b = jac[i].genomeB;
        M[(std::size_t)ds.mapQueryId(a) * nt + ds.mapTargetId(b)] = aji[i];
        if (ds.isQryGenome(b)) M[(std::size_t)ds.mapQueryId(b) * nt + ds.mapTargetId(a)] = aji[i];
    }
    return M;
}

// printOutput's CSV (main.cpp:156-174), written block of rows by block of
// rows: header at open, then rows() any number of times in row order (every
// OpenMP thread formats rows into its own buffer; they are written in order).
class CsvWriter {
  public:
    CsvWriter(const std::string& path, const std::vector<std::string>& cols, const std::string& sep)
        : m_f(std::fopen(path.c_str(), "w")), m_sep(sep), m_nc((int64_t)cols.size()) {
        if (!m_f) return;
        std::string head = sep;
        for (std::size_t j = 0; j < cols.size(); ++j) {
            if (j) head += sep;
            head += cols[j];
        }
        head += '\n';
        m_ok = std::fwrite(head.data(), 1, head.size(), m_f) == head.size();
    }
    ~CsvWriter() { close(); }
    bool ok() const { return m_f && m_ok; }
    // rows [r0, r1) named names[r], values M[(r - r0) * n_cols + c]
    bool rows(const std::vector<std::string>& names, const double* M, int64_t r0, int64_t r1) {
        if (!ok()) return false;
        const int64_t block = 256;  // rows formatted per parallel batch, then written in order
        for (int64_t b0 = r0; b0 < r1; b0 += block) {
            const int64_t b1 = std::min(r1, b0 + block);
            if ((int64_t)m_buf.size() < b1 - b0) m_buf.resize(b1 - b0);
#pragma omp parallel for schedule(dynamic, 1)
            for (int64_t r = b0; r < b1; ++r) {
                std::string& s = m_buf[r - b0];
                s.clear();
                s.reserve(names[r].size() + m_nc * 20 + 2);
                s += names[r];
                s += m_sep;
                char tmp[48];
                const double* row = M + (std::size_t)(r - r0) * m_nc;
                for (int64_t c = 0; c < m_nc; ++c) {
                    if (c) s += m_sep;
                    s.append(tmp, fmt_double(row[c], tmp));
                }
                s += '\n';
            }
            for (int64_t r = b0; r < b1; ++r)
                m_ok = m_ok && std::fwrite(m_buf[r - b0].data(), 1, m_buf[r - b0].size(), m_f) == m_buf[r - b0].size();
        }
        return m_ok;
    }
    bool close() {
        if (!m_f) return m_ok;
        m_ok = std::fclose(m_f) == 0 && m_ok;
        m_f = nullptr;
        return m_ok;
    }

  private:
    FILE* m_f;
    std::string m_sep;
    int64_t m_nc;
    bool m_ok = false;
    std::vector<std::string> m_buf;
};

inline int write_csv(const std::string& path, const std::vector<std::string>& rows,
                     const std::vector<std::string>& cols, const std::vector<double>& M, const std::string& sep) {
    CsvWriter w(path, cols, sep);
    w.rows(rows, M.data(), 0, (int64_t)rows.size());
    return w.close() ? 0 : 1;
}

// cereal: std::vector<JACTuple<int,double>> (20-B packed records) / vector<double>
template <typename JAC>
inline int write_bin(const std::string& prefix, const std::vector<JAC>& jac, const std::vector<double>& aji,
                     const std::vector<double>& M, int64_t rows, int64_t cols) {
    auto put = [](FILE* f, const void* p, std::size_t n) { return n == 0 || std::fwrite(p, 1, n, f) == n; };  // (empty vectors: data() may be null)
    bool ok = true;
    if (FILE* f = std::fopen((prefix + "_jac.bin").c_str(), "wb")) {
        uint64_t n = jac.size();
        ok &= put(f, &n, 8);
        for (const auto& x : jac) {
            ok &= put(f, &x.genomeA, 4) && put(f, &x.genomeB, 4) && put(f, &x.S, 8) && put(f, &x.N, 4);
        }
        std::fclose(f);
    } else {
        ok = false;
    }
    if (FILE* f = std::fopen((prefix + "_aji.bin").c_str(), "wb")) {
        uint64_t n = aji.size();
        ok &= put(f, &n, 8) && put(f, aji.data(), 8 * n);
        std::fclose(f);
    } else {
        ok = false;
    }
    if (FILE* f = std::fopen((prefix + "_aji_matrix.bin").c_str(), "wb")) {  // DMatrix<double>
        uint64_t h[3] = {(uint64_t)rows, (uint64_t)cols, (uint64_t)(rows * cols)};
        ok &= put(f, h, 24) && put(f, M.data(), 8 * M.size());
        std::fclose(f);
    } else {
        ok = false;
    }
    return ok ? 0 : 1;
}

}  // namespace pfaai_host
