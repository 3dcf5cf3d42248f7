"""Reference file formats: cereal binary archives and the AJI CSV matrix.

cereal BinaryOutputArchive (little endian, no padding), as the reference's
fixtures and tests use it:
  std::vector<T>        uint64 n, then n packed records
  DPair<int,int>        (first, second) int32          utils.hpp:204-225
  ETriple<int>          (proteinIndex, genomeA, genomeB) interface.hpp:92-121
  JACTuple<int,double>  (genomeA i32, genomeB i32, S f64, N i32) = 20 B
                                                       interface.hpp:61-75
  DMatrix<int>          uint64 rows, uint64 cols, vector<int> utils.hpp:240-288

CSV: printOutput (main.cpp:133-175) writes `sep + join(targets, sep)` then one
line per query `name sep join(values, sep)`; values use fmt 10's `{}` for
double = shortest round-trip text, fixed notation iff -4 <= exp10 < 16,
integral values without ".0".
"""
from __future__ import annotations

import gzip
import io
import os
import struct

import numpy as np

JAC_DTYPE = np.dtype([("genomeA", "<i4"), ("genomeB", "<i4"), ("S", "<f8"), ("N", "<i4")], align=False)
assert JAC_DTYPE.itemsize == 20


def _open(path):
    path = os.fspath(path)
    if path.endswith(".gz"):
        return gzip.open(path, "rb")
    if not os.path.exists(path) and os.path.exists(path + ".gz"):
        return gzip.open(path + ".gz", "rb")
    return open(path, "rb")


def _read_bytes(path) -> bytes:
    with _open(path) as f:
        return f.read()


def _vec(buf: bytes, offset: int, dtype) -> tuple[np.ndarray, int]:
    (n,) = struct.unpack_from("<Q", buf, offset)
    offset += 8
    dt = np.dtype(dtype)
    arr = np.frombuffer(buf, dtype=dt, count=n, offset=offset).copy()
    return arr, offset + n * dt.itemsize


def read_vec_i32(path) -> np.ndarray:
    """std::vector<int> (Lc, Lp, e_size, gpe_starts ...)."""
    return _vec(_read_bytes(path), 0, "<i4")[0]


def read_vec_f64(path) -> np.ndarray:
    """std::vector<double> (AJI)."""
    return _vec(_read_bytes(path), 0, "<f8")[0]


def read_f_array(path) -> np.ndarray:
    """std::vector<DPair<int,int>> -> (n, 2) int32 [protein, genome]."""
    buf = _read_bytes(path)  # the vector length counts pairs, not ints
    (n,) = struct.unpack_from("<Q", buf, 0)
    return np.frombuffer(buf, dtype="<i4", count=2 * n, offset=8).reshape(n, 2).copy()


def read_e_array(path) -> np.ndarray:
    """std::vector<ETriple<int>> -> (n, 3) int32 [protein, genomeA, genomeB]."""
    buf = _read_bytes(path)
    (n,) = struct.unpack_from("<Q", buf, 0)
    return np.frombuffer(buf, dtype="<i4", count=3 * n, offset=8).reshape(n, 3).copy()


def read_matrix_i32(path) -> np.ndarray:
    """DMatrix<int> -> (rows, cols) int32."""
    buf = _read_bytes(path)
    rows, cols, n = struct.unpack_from("<QQQ", buf, 0)
    assert n == rows * cols
    return np.frombuffer(buf, dtype="<i4", count=n, offset=24).reshape(rows, cols).copy()


def read_jac(path) -> np.ndarray:
    """std::vector<JACTuple<int,double>> -> structured array (genomeA, genomeB, S, N)."""
    return _vec(_read_bytes(path), 0, JAC_DTYPE)[0]


def write_vec(path, arr: np.ndarray) -> None:
    arr = np.ascontiguousarray(arr)
    n = arr.shape[0]
    with open(path, "wb") as f:
        f.write(struct.pack("<Q", n))
        f.write(arr.tobytes())


def write_jac(path, ga, gb, S, N) -> None:
    rec = np.empty(len(S), dtype=JAC_DTYPE)
    rec["genomeA"], rec["genomeB"], rec["S"], rec["N"] = ga, gb, S, N
    write_vec(path, rec)


def write_matrix_f64(path, m: np.ndarray) -> None:
    """DMatrix<double> cereal layout (rows, cols, vector<double>)."""
    m = np.ascontiguousarray(m, dtype="<f8")
    with open(path, "wb") as f:
        f.write(struct.pack("<QQQ", m.shape[0], m.shape[1], m.size))
        f.write(m.tobytes())


# ---------------------------------------------------------------------------
# CSV (main.cpp:156-174)
# ---------------------------------------------------------------------------

def fmt_double(x: float) -> str:
    """fmt 10 `{}` of a double: shortest round-trip; Python's repr uses the
    same digits and the same fixed/scientific switch; fmt drops the ".0"."""
    s = repr(float(x))
    if s.endswith(".0"):
        s = s[:-2]
    return s


def csv_text(row_names, col_names, matrix: np.ndarray, sep: str = ",") -> str:
    out = io.StringIO()
    out.write(sep + sep.join(col_names) + "\n")
    for name, row in zip(row_names, matrix):
        out.write(name + sep + sep.join(fmt_double(v) for v in row.tolist()) + "\n")
    return out.getvalue()


def read_csv_matrix(path, sep: str = ","):
    """-> (row_names, col_names, float64 matrix) of a printOutput CSV."""
    with _open(path) as f:
        lines = f.read().decode().splitlines()
    cols = lines[0].split(sep)[1:]
    rows, vals = [], []
    for ln in lines[1:]:
        parts = ln.split(sep)
        rows.append(parts[0])
        vals.append([float(v) for v in parts[1:]])
    return rows, cols, np.array(vals, dtype=np.float64).reshape(len(rows), len(cols))
