"""Host-side mirror of the reference's data-structure contract.

DataStructInterface (interface.hpp:200-328) and its three modes
(ds_impl.hpp): the arrays Lc / Lp / F / T plus the mode's index maps.  These
classes hold host numpy arrays (from the SQLite loader, a fixture or the
synthetic generator) and describe them to the HIP engine through
``problem()``; the hot path itself runs in libpfaai_hip.so.

Names follow the reference (refLc, refF, nGenomePairs, genomePairToIndex,
initJAC, mapQueryId ...) so code and tests read like its own.
"""
from __future__ import annotations

import numpy as np

from . import _capi

NTETRAMERS = _capi.NTETRAMERS


def lp_from_lc(Lc: np.ndarray) -> np.ndarray:
    """Exclusive prefix of Lc with the total appended: int64[160001]
    (parallelPrefixSum, ds_helper.hpp:112-122, widened to 64 bit)."""
    Lc = np.asarray(Lc, dtype=np.int64)
    assert Lc.shape == (NTETRAMERS,)
    Lp = np.zeros(NTETRAMERS + 1, dtype=np.int64)
    np.cumsum(Lc, out=Lp[1:])
    return Lp


class DataStruct:
    """Common part of DataStructInterface (interface.hpp:200-328)."""

    mode = -1

    def __init__(self, Lc, F, T, protein_set=None):
        F = np.asarray(F)
        self.F_prot = np.ascontiguousarray(F[:, 0], dtype=np.int32) if F.ndim == 2 else None
        self.F_genome = np.ascontiguousarray(F[:, 1], dtype=np.int32) if F.ndim == 2 else None
        self.Lc = np.asarray(Lc, dtype=np.int32)
        self.Lp = lp_from_lc(self.Lc)
        self.T = np.ascontiguousarray(T, dtype=np.int32)
        self.n_prot = self.T.shape[0]
        self.protein_set = list(protein_set) if protein_set is not None else [f"P{i}" for i in range(self.n_prot)]
        assert self.Lp[-1] == len(self.F_genome), "Lc does not match |F|"

    G_off = None  # optional genome-major view (the `<p>_genomes` blobs)
    G_tet = None

    def with_genome_major(self, G_off, G_tet):
        """Attach the genome-major tetramer lists ((genome, protein)-major CSR)."""
        self.G_off = np.ascontiguousarray(G_off, dtype=np.int64)
        self.G_tet = np.ascontiguousarray(G_tet, dtype=np.int32)
        return self

    def _g(self):
        return {} if self.G_off is None else dict(G_off=self.G_off, G_tet=self.G_tet)

    @classmethod
    def from_split(cls, Lp, F_prot, F_genome, T, *args, **kw):
        """Build from int64 Lp[160001] and separate F columns (no copies of F)."""
        obj = cls.__new__(cls)
        obj.F_prot = np.ascontiguousarray(F_prot, dtype=np.int32)
        obj.F_genome = np.ascontiguousarray(F_genome, dtype=np.int32)
        obj.Lp = np.ascontiguousarray(Lp, dtype=np.int64)
        obj.Lc = np.diff(obj.Lp).astype(np.int32)
        obj.T = np.ascontiguousarray(T, dtype=np.int32)
        obj.n_prot = obj.T.shape[0]
        protein_set = kw.pop("protein_set", None)
        obj.protein_set = list(protein_set) if protein_set is not None else [f"P{i}" for i in range(obj.n_prot)]
        obj._init_mode(*args, **kw)
        return obj

    # reference accessors (interface.hpp:246-250)
    def refLc(self):
        return self.Lc

    def refLp(self):
        return self.Lp[:-1].astype(np.int32)

    def refF(self):
        return np.stack([self.F_prot, self.F_genome], axis=1)

    def refT(self):
        return self.T

    def nTetramers(self):
        return NTETRAMERS

    def problem(self) -> dict:
        raise NotImplementedError

    def output_matrix(self, ga, gb, aji) -> np.ndarray:
        """printOutput's dense fill (main.cpp:143-154).  The cell index is
        the row-major DMatrix offset row * nT + col, as the reference's
        unchecked operator() computes it: with the quirky -r ids and more
        queries than targets a column can pass nT and the write lands in a
        later row (always inside the matrix for nQ >= nT); writes happen in
        JAC order, so the last one to a cell wins."""
        M = np.zeros((self.qrySetSize(), self.tgtSetSize()), dtype=np.float64)
        mq = self._map_query(ga).astype(np.int64)
        mt = self._map_target(gb).astype(np.int64)
        flat = mq * self.tgtSetSize() + mt
        if len(flat) and (mt.max() >= self.tgtSetSize() or flat.max() >= M.size):
            if flat.max() >= M.size:
                raise IndexError("output cell past the end of the matrix")
            # last write wins: keep each cell's final JAC index
            last = np.zeros(M.size, np.int64) - 1
            np.maximum.at(last, flat, np.arange(len(flat)))
            sel = last >= 0
            M.flat[np.nonzero(sel)[0]] = np.asarray(aji)[last[sel]]
        else:
            M[mq, mt] = aji
        if self.is_subset_output:
            sel = self._is_qry(gb)
            M[self._map_query(gb[sel]), self._map_target(ga[sel])] = aji[sel]
        return M


class ParFAAIData(DataStruct):
    """All-vs-all (ds_impl.hpp:38-151)."""

    mode = _capi.MODE_ALL
    is_subset_output = True

    def __init__(self, Lc, F, T, genome_set=None, protein_set=None):
        super().__init__(Lc, F, T, protein_set)
        self._init_mode(genome_set)

    def _init_mode(self, genome_set=None):
        n = self.T.shape[1] if genome_set is None else len(genome_set)
        self.genome_set = list(genome_set) if genome_set is not None else [f"G{i}" for i in range(n)]
        self.n_genomes = n

    def refQuerySet(self):
        return self.genome_set

    def refTargetSet(self):
        return self.genome_set

    def qrySetSize(self):
        return self.n_genomes

    def tgtSetSize(self):
        return self.n_genomes

    def nGenomePairs(self):
        return self.n_genomes * (self.n_genomes - 1) // 2

    def genomePairToIndex(self, a, b):
        return self.n_genomes * a + b - (a + 2) * (a + 1) // 2

    def isQryGenome(self, g):
        return True

    def isValidPair(self, a, b):
        return a < b

    def countGenomePairs(self, nq, nt):
        return nq * (nq - 1) // 2

    def initJAC(self, ref_compat=False):
        a, b = np.triu_indices(self.n_genomes, 1)
        return a.astype(np.int32), b.astype(np.int32)

    def _map_query(self, g):
        return g

    def _map_target(self, g):
        return g

    def _is_qry(self, g):
        return np.ones(len(g), dtype=bool)

    def problem(self):
        return dict(mode=self.mode, n_ids=self.n_genomes, n_prot=self.n_prot, Lp=self.Lp,
                    F_prot=self.F_prot, F_genome=self.F_genome, T=self.T, **self._g())


class ParFAAIQSubData(DataStruct):
    """Query subset of one DB, ``-q`` (ds_impl.hpp:158-337)."""

    mode = _capi.MODE_QSUB
    is_subset_output = True

    def __init__(self, Lc, F, T, genome_set, qry_genome_set, protein_set=None):
        super().__init__(Lc, F, T, protein_set)
        self._init_mode(genome_set, qry_genome_set)

    def _init_mode(self, genome_set, qry_genome_set):
        self.genome_set = list(genome_set)
        self.qry_genome_set = list(qry_genome_set)
        n = self.n_genomes = len(self.genome_set)
        nq = self.n_qry = len(self.qry_genome_set)
        self.n_tgt = n - nq
        qpos = {name: i for i, name in enumerate(self.qry_genome_set)}  # ds_impl.hpp:203-207
        self.is_q = np.zeros(n, dtype=np.uint8)
        self.q_index = np.full(n, -1, dtype=np.int32)
        self.t_rank = np.full(n, -1, dtype=np.int32)
        self.genome_index_map = np.zeros(n, dtype=np.int32)
        self.qry_lookup = np.zeros(nq, dtype=np.int32)
        self.tgt_lookup = np.zeros(self.n_tgt, dtype=np.int32)
        jx = 0
        for ix, name in enumerate(self.genome_set):  # ds_impl.hpp:210-223
            if name in qpos:
                self.is_q[ix] = 1
                self.q_index[ix] = qpos[name]
                self.qry_lookup[qpos[name]] = ix
                self.genome_index_map[ix] = qpos[name]
            else:
                self.t_rank[ix] = jx
                self.tgt_lookup[jx] = ix
                self.genome_index_map[ix] = jx
                jx += 1

    def refQuerySet(self):
        return self.qry_genome_set

    def refTargetSet(self):
        return self.genome_set

    def qrySetSize(self):
        return self.n_qry

    def tgtSetSize(self):
        return self.n_genomes

    def nGenomePairs(self):
        return self.n_qry * self.n_tgt + self.n_qry * (self.n_qry - 1) // 2

    def isQryGenome(self, g):
        return bool(self.is_q[g])

    def isValidPair(self, a, b):
        return bool((self.is_q[a] and self.is_q[b] and a < b) or (self.is_q[a] and not self.is_q[b] and a != b))

    def countGenomePairs(self, nq, nt):
        return nq * nt + nq * (nq - 1) // 2

    def initJAC(self, ref_compat=False):
        nq, nt = self.n_qry, self.n_tgt
        i = np.arange(nq * nt, dtype=np.int64)
        ga = [self.qry_lookup[i // nt]] if nt else [np.zeros(0, np.int32)]
        gb = [self.tgt_lookup[i % nt]] if nt else [np.zeros(0, np.int32)]
        a, b = np.triu_indices(nq, 1)
        ga.append(self.qry_lookup[a])
        gb.append(self.qry_lookup[b])
        return np.concatenate(ga).astype(np.int32), np.concatenate(gb).astype(np.int32)

    def _map_query(self, g):
        return self.genome_index_map[g]

    def _map_target(self, g):
        return g

    def _is_qry(self, g):
        return self.is_q[g].astype(bool)

    def problem(self):
        return dict(mode=self.mode, n_ids=self.n_genomes, n_prot=self.n_prot, Lp=self.Lp,
                    F_prot=self.F_prot, F_genome=self.F_genome, T=self.T, n_qry=self.n_qry,
                    n_tgt=self.n_tgt, is_q=self.is_q, q_index=self.q_index, t_rank=self.t_rank, **self._g())


class ParFAAIQryTgtData(DataStruct):
    """Query DB vs target DB, ``-r`` (ds_impl.hpp:343-490).

    Genome ids in F: targets 0..nT-1, queries nT..nT+nQ-1
    (scp_db.hpp:518-519).  T has nT + nQ columns."""

    mode = _capi.MODE_QT
    is_subset_output = False

    def __init__(self, Lc, F, T, tgt_genome_set, qry_genome_set, protein_set=None):
        super().__init__(Lc, F, T, protein_set)
        self._init_mode(tgt_genome_set, qry_genome_set)

    def _init_mode(self, tgt_genome_set, qry_genome_set):
        self.tgt_genome_set = list(tgt_genome_set)
        self.qry_genome_set = list(qry_genome_set)
        self.n_tgt = len(self.tgt_genome_set)
        self.n_qry = len(self.qry_genome_set)
        n = self.n_ids = self.n_tgt + self.n_qry
        self.is_q = np.zeros(n, dtype=np.uint8)
        self.is_q[self.n_tgt:] = 1
        self.genome_index_map = np.concatenate([np.arange(self.n_tgt), np.arange(self.n_qry)]).astype(np.int32)

    def refQuerySet(self):
        return self.qry_genome_set

    def refTargetSet(self):
        return self.tgt_genome_set

    def qrySetSize(self):
        return self.n_qry

    def tgtSetSize(self):
        return self.n_tgt

    def nGenomePairs(self):
        return self.n_qry * self.n_tgt

    def isQryGenome(self, g):
        return bool(self.is_q[g])

    def isValidPair(self, a, b):
        return bool(self.is_q[a] and not self.is_q[b])

    def countGenomePairs(self, nq, nt):
        return nq * nt

    def initJAC(self, ref_compat=False):
        """ds_impl.hpp:428-439.  The reference stores (i/nT, nQ + i%nT), which
        are not the E ids; with ref_compat=False the E ids
        (nT + i/nT, i%nT) are returned."""
        i = np.arange(self.n_qry * self.n_tgt, dtype=np.int64)
        if ref_compat:
            return (i // self.n_tgt).astype(np.int32), (self.n_qry + i % self.n_tgt).astype(np.int32)
        return (self.n_tgt + i // self.n_tgt).astype(np.int32), (i % self.n_tgt).astype(np.int32)

    def _map_query(self, g):
        return self.genome_index_map[g]

    def _map_target(self, g):
        return self.genome_index_map[g]

    def _is_qry(self, g):
        return self.is_q[g].astype(bool)

    def problem(self):
        return dict(mode=self.mode, n_ids=self.n_ids, n_prot=self.n_prot, Lp=self.Lp,
                    F_prot=self.F_prot, F_genome=self.F_genome, T=self.T, n_qry=self.n_qry,
                    n_tgt=self.n_tgt, is_q=self.is_q, **self._g())
