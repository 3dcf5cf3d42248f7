"""ParFAAIImpl mirror on the MI355X engine.

Same public surface as the reference's consumer class ParFAAIImpl
(algorithm_impl.hpp:38-357): ``run()``, ``computeJAC()``, ``computeAJI()``,
``getJAC()``, ``getAJI()``, all returning PFAAI_OK (0) like the reference
(algorithm_impl.hpp:281-329).  Every call goes through libpfaai_hip.so; the
JAC genome ids are the mode's initJAC ids (ds_impl.hpp:99-114, 278-305,
428-439).
"""
from __future__ import annotations

import numpy as np

from . import _capi
from .formats import JAC_DTYPE

PFAAI_OK = 0


class ParFAAIImpl:
    def __init__(self, ds, device: int = 0, ref_compat: bool = False, engine: _capi.Engine | None = None):
        self.ds = ds
        self.ref_compat = bool(ref_compat)
        self.engine = engine or _capi.Engine(device)
        self.engine.load(**ds.problem())
        self.n_rows, self.n_pairs = self.engine.shape()
        assert self.n_pairs == ds.nGenomePairs()
        self._jac = None
        self._aji = None
        self._aji_dev = None
        self.stats = {}

    @property
    def flags(self):
        return _capi.FLAG_REF_COMPAT if self.ref_compat else 0

    # algorithm_impl.hpp:281-306
    def computeJAC(self) -> int:
        aji, S, N = self.engine.compute(self.flags)
        ga, gb = self.ds.initJAC(self.ref_compat)
        jac = np.empty(self.n_pairs, dtype=JAC_DTYPE)
        jac["genomeA"], jac["genomeB"], jac["S"], jac["N"] = ga, gb, S, N
        self._jac = jac
        self._aji_dev = aji  # the kernel's epilogue already divided S / N
        self.stats = self.engine.stats()
        return PFAAI_OK

    # algorithm_impl.hpp:309-322
    def computeAJI(self) -> int:
        if self._jac is None:
            self.computeJAC()
        self._aji = self._aji_dev
        return PFAAI_OK

    # algorithm_impl.hpp:325-329
    def run(self) -> int:
        self.computeJAC()
        self.computeAJI()
        return PFAAI_OK

    def getJAC(self) -> np.ndarray:
        return self._jac

    def getAJI(self) -> np.ndarray:
        return self._aji

    def n_events(self) -> int:
        """|E| counted by the scatter kernel (countTetramerTuples total)."""
        return int(self.stats.get("n_events", -1))

    def output_matrix(self) -> np.ndarray:
        """printOutput's dense AJI matrix (main.cpp:143-154)."""
        jac = self.getJAC()
        return self.ds.output_matrix(jac["genomeA"], jac["genomeB"], self.getAJI())

    def row_counts(self, row: int) -> np.ndarray:
        """Integer intersection counts c(p, A=row genome, B) from the device
        (pfaai_debug_row_counts)."""
        n_ids = self.ds.problem()["n_ids"]
        return self.engine.debug_row_counts(row, self.ds.n_prot, n_ids)
