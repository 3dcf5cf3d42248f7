"""ctypes wrapper of the CPU oracle (oracle/pfaai_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, always as the checker / baseline -- never by the
product package (parfastaai_amd/ must not import this module).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.environ.get("PFAAI_ORACLE_LIB", os.path.join(HERE, "_build", "libpfaai_oracle.so"))  # (tools/sanitize.py)


class Mode(ctypes.Structure):
    _fields_ = [
        ("mode", ctypes.c_int32), ("n_ids", ctypes.c_int32), ("n_prot", ctypes.c_int32),
        ("t_cols", ctypes.c_int32), ("n_qry", ctypes.c_int32), ("n_tgt", ctypes.c_int32),
        ("compat", ctypes.c_int32), ("pad_", ctypes.c_int32),
        ("is_q", ctypes.c_void_p), ("q_index", ctypes.c_void_p), ("t_rank", ctypes.c_void_p),
        ("q_lookup", ctypes.c_void_p), ("t_lookup", ctypes.c_void_p),
    ]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            import subprocess
            subprocess.run(["make", "-C", HERE], check=True, capture_output=True)
        L = ctypes.CDLL(LIB)
        vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32
        L.oracle_n_pairs.restype, L.oracle_n_pairs.argtypes = i64, [vp]
        L.oracle_count_e.restype, L.oracle_count_e.argtypes = i64, [vp, vp, vp, vp]
        L.oracle_build_sorted_e.restype, L.oracle_build_sorted_e.argtypes = i64, [vp, vp, vp, vp, vp, i64]
        L.oracle_ref_run.restype = i64
        L.oracle_ref_run.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
        L.oracle_dense_rows.restype = i64
        L.oracle_dense_rows.argtypes = [vp, vp, vp, vp, vp, i32, i32, vp, vp]
        L.oracle_init_jac.restype, L.oracle_init_jac.argtypes = None, [vp, vp, vp]
        L.oracle_full_rows.restype = i64
        L.oracle_full_rows.argtypes = [vp, vp, vp, vp, vp, i64, i64, vp, vp, vp]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class Problem:
    """Arrays + mode description, built from a parfastaai_amd DataStruct-like
    problem dict (mode, n_ids, n_prot, Lp, F_prot, F_genome, T, ...)."""

    def __init__(self, prob: dict, compat: bool = False, q_lookup=None, t_lookup=None):
        self.Lp = np.ascontiguousarray(prob["Lp"], dtype=np.int64)
        self.Fp = np.ascontiguousarray(prob["F_prot"], dtype=np.int32)
        self.Fg = np.ascontiguousarray(prob["F_genome"], dtype=np.int32)
        self.T = np.ascontiguousarray(prob["T"], dtype=np.int32)
        n_ids = prob["n_ids"]
        self.is_q = np.ascontiguousarray(prob.get("is_q", np.ones(n_ids, np.uint8)), dtype=np.uint8)
        self.q_index = np.ascontiguousarray(prob.get("q_index", np.full(n_ids, -1, np.int32)), dtype=np.int32)
        self.t_rank = np.ascontiguousarray(prob.get("t_rank", np.full(n_ids, -1, np.int32)), dtype=np.int32)
        mode = prob["mode"]
        n_qry = prob.get("n_qry", n_ids)
        n_tgt = prob.get("n_tgt", 0)
        if mode == 1:
            if q_lookup is None:
                q_lookup = np.zeros(n_qry, np.int32)
                sel = np.nonzero(self.is_q)[0]
                q_lookup[self.q_index[sel]] = sel
            if t_lookup is None:
                sel = np.nonzero(self.is_q == 0)[0]
                t_lookup = np.zeros(n_tgt, np.int32)
                t_lookup[self.t_rank[sel]] = sel
        self.q_lookup = np.ascontiguousarray(q_lookup if q_lookup is not None else np.zeros(1, np.int32), dtype=np.int32)
        self.t_lookup = np.ascontiguousarray(t_lookup if t_lookup is not None else np.zeros(1, np.int32), dtype=np.int32)
        self.mode = Mode(mode=mode, n_ids=n_ids, n_prot=self.T.shape[0], t_cols=self.T.shape[1],
                         n_qry=n_qry if mode != 0 else n_ids, n_tgt=n_tgt, compat=int(compat),
                         is_q=_p(self.is_q), q_index=_p(self.q_index), t_rank=_p(self.t_rank),
                         q_lookup=_p(self.q_lookup), t_lookup=_p(self.t_lookup))

    def n_pairs(self):
        return lib().oracle_n_pairs(ctypes.byref(self.mode))

    def count_e(self):
        return lib().oracle_count_e(ctypes.byref(self.mode), _p(self.Lp), _p(self.Fp), _p(self.Fg))

    def sorted_e(self):
        ne = self.count_e()
        out = np.empty((max(ne, 1), 3), dtype=np.int32)
        got = lib().oracle_build_sorted_e(ctypes.byref(self.mode), _p(self.Lp), _p(self.Fp), _p(self.Fg), _p(out), ne)
        assert got == ne
        return out[:ne]

    def init_jac(self):
        n = self.n_pairs()
        ga, gb = np.empty(n, np.int32), np.empty(n, np.int32)
        lib().oracle_init_jac(ctypes.byref(self.mode), _p(ga), _p(gb))
        return ga, gb

    def ref_run(self):
        """-> dict(S, N, AJI, genomeA, genomeB, n_events) in JAC order."""
        n = self.n_pairs()
        S, N, A = np.empty(n), np.empty(n, np.int32), np.empty(n)
        ga, gb = np.empty(n, np.int32), np.empty(n, np.int32)
        ne = lib().oracle_ref_run(ctypes.byref(self.mode), _p(self.Lp), _p(self.Fp), _p(self.Fg), _p(self.T),
                                  _p(S), _p(N), _p(A), _p(ga), _p(gb))
        if ne < 0:
            raise RuntimeError(f"oracle_ref_run failed: {ne}")
        return dict(S=S, N=N, AJI=A, genomeA=ga, genomeB=gb, n_events=ne)

    def dense_rows(self, row_lo, row_hi):
        """Appendix-A restatement for genome ids [row_lo, row_hi) as rows:
        -> (S, N) of shape (rows, n_ids), n_events."""
        nr, ni = row_hi - row_lo, self.mode.n_ids
        S = np.zeros((nr, ni)); N = np.zeros((nr, ni), np.int32)
        ne = lib().oracle_dense_rows(ctypes.byref(self.mode), _p(self.Lp), _p(self.Fp), _p(self.Fg), _p(self.T),
                                     row_lo, row_hi, _p(S), _p(N))
        return S, N, ne

    def full_rows(self, row_lo, row_hi, S, N, AJI):
        """Appendix A over output rows [row_lo, row_hi) (mode 0: genomes;
        mode 2: query rows), written into S / N / AJI (views of the JAC-order
        arrays starting at the rows' first JAC index; corrected semantics).
        OpenMP over rows.  -> |E| of the rows."""
        for a, dt in ((S, np.float64), (N, np.int32), (AJI, np.float64)):
            assert a.dtype == dt and a.flags.c_contiguous
        ne = lib().oracle_full_rows(ctypes.byref(self.mode), _p(self.Lp), _p(self.Fp), _p(self.Fg), _p(self.T),
                                    row_lo, row_hi, _p(S), _p(N), _p(AJI))
        if ne < 0:
            raise RuntimeError(f"oracle_full_rows failed: {ne}")
        return ne
