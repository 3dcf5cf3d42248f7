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
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)jac.size(); ++i) {
        const int32_t a = jac[i].genomeA, b = jac[i].genomeB;
        M[(std::size_t)ds.mapQueryId(a) * nt + ds.mapTargetId(b)] = aji[i];
        if (isSubset && ds.isQryGenome(b)) M[(std::size_t)ds.mapQueryId(b) * nt + ds.mapTargetId(a)] = aji[i];
    }
    return M;
}

inline int write_csv(const std::string& path, const std::vector<std::string>& rows,
                     const std::vector<std::string>& cols, const std::vector<double>& M, const std::string& sep) {
    FILE* f = std::fopen(path.c_str(), "w");
    if (!f) return 1;
    std::string head = sep;
    for (std::size_t j = 0; j < cols.size(); ++j) {
        if (j) head += sep;
        head += cols[j];
    }
    head += '\n';
    std::fwrite(head.data(), 1, head.size(), f);
    const int64_t nr = (int64_t)rows.size(), nc = (int64_t)cols.size();
    const int64_t block = 256;  // rows formatted per parallel batch, then written in order
    std::vector<std::string> buf(block);
    for (int64_t r0 = 0; r0 < nr; r0 += block) {
        const int64_t r1 = std::min(nr, r0 + block);
#pragma omp parallel for schedule(dynamic, 1)
        for (int64_t r = r0; r < r1; ++r) {
            std::string& s = buf[r - r0];
            s.clear();
            s.reserve(rows[r].size() + nc * 20 + 2);
            s += rows[r];
            s += sep;
            char tmp[48];
            for (int64_t c = 0; c < nc; ++c) {
                if (c) s += sep;
                s.append(tmp, fmt_double(M[(std::size_t)r * nc + c], tmp));
            }
            s += '\n';
        }
        for (int64_t r = r0; r < r1; ++r) std::fwrite(buf[r - r0].data(), 1, buf[r - r0].size(), f);
    }
    return std::fclose(f) == 0 ? 0 : 1;
}

// cereal: std::vector<JACTuple<int,double>> (20-B packed records) / vector<double>
template <typename JAC>
inline int write_bin(const std::string& prefix, const std::vector<JAC>& jac, const std::vector<double>& aji,
                     const std::vector<double>& M, int64_t rows, int64_t cols) {
    auto put = [](FILE* f, const void* p, std::size_t n) { return std::fwrite(p, 1, n, f) == n; };
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
