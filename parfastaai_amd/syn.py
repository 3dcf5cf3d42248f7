"""Synthetic SCP/tetramer databases (SURVEY.md §8d "SYN" spec).

``generate()`` returns the arrays of a DataStructInterface (Lp, F, T) built by
tools/syn_gen.c (deterministic, OpenMP); ``write_db()`` writes the same
database as a FastAAI SQLite file with the reference's schema (for the CLI,
the loader and the reference binary).  Bench / test infrastructure.
"""
from __future__ import annotations

import ctypes
import os
import sqlite3

import numpy as np

from .datastruct import NTETRAMERS

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tools", "_build", "libpfaai_syn.so")
DEFAULT_SEED = 20250213


class SynParams(ctypes.Structure):
    _fields_ = [
        ("anc_seed", ctypes.c_uint64), ("genome_seed", ctypes.c_uint64),
        ("n_genomes", ctypes.c_int32), ("n_prot", ctypes.c_int32), ("clade_size", ctypes.c_int32),
        ("n_clades", ctypes.c_int32), ("clade_mod", ctypes.c_int32), ("n_random", ctypes.c_int32),
        ("keep_permille", ctypes.c_int32), ("has_permille", ctypes.c_int32),
    ]


_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError(f"{LIB} missing: run __graft_entry__.build()")
        L = ctypes.CDLL(LIB)
        vp = ctypes.c_void_p
        L.syn_counts.restype, L.syn_counts.argtypes = ctypes.c_int64, [vp, vp]
        L.syn_fill.restype, L.syn_fill.argtypes = ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp]
        L.syn_genome_set.restype, L.syn_genome_set.argtypes = ctypes.c_int32, [vp, ctypes.c_int32, ctypes.c_int32, vp]
        _lib = L
    return _lib


def params(n_genomes, n_prot=100, seed=DEFAULT_SEED, genome_seed=None, clade_size=20, n_clades=0,
           clade_mod=False, n_random=5, keep=0.9, has=0.98) -> SynParams:
    return SynParams(anc_seed=seed, genome_seed=seed if genome_seed is None else genome_seed,
                     n_genomes=n_genomes, n_prot=n_prot, clade_size=clade_size, n_clades=n_clades,
                     clade_mod=int(clade_mod), n_random=n_random, keep_permille=int(round(keep * 1000)),
                     has_permille=int(round(has * 1000)))


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def generate(n_genomes, n_prot=100, **kw) -> dict:
    """-> dict(Lp int64[160001], F_prot, F_genome int32[|F|], T int32[P, G],
    G_off int64[G*P+1], G_tet int32[|F|], genome_set, protein_set): F ordered
    exactly as the reference's loader would produce it from the equivalent
    SQLite DB, G = the genome-major `<p>_genomes` sets ((genome, protein)-major
    CSR)."""
    prm = params(n_genomes, n_prot, **kw)
    L = _load()
    T = np.zeros((n_prot, n_genomes), dtype=np.int32)
    nf = L.syn_counts(ctypes.byref(prm), _p(T))
    Lp = np.zeros(NTETRAMERS + 1, dtype=np.int64)
    Fp = np.empty(nf, dtype=np.int32)
    Fg = np.empty(nf, dtype=np.int32)
    G_off = np.zeros(n_genomes * n_prot + 1, dtype=np.int64)
    G_tet = np.empty(max(nf, 1), dtype=np.int32)
    rc = L.syn_fill(ctypes.byref(prm), _p(T), _p(Lp), _p(Fp), _p(Fg), _p(G_off), _p(G_tet))
    if rc:
        raise RuntimeError("syn_fill failed")
    return dict(Lp=Lp, F_prot=Fp, F_genome=Fg, T=T, G_off=G_off, G_tet=G_tet[:nf],
                genome_set=genome_names(n_genomes), protein_set=protein_names(n_prot), params=prm)


def genome_names(n, prefix="syn"):
    return [f"{prefix}_{i:06d}.fna.gz" for i in range(n)]


def protein_names(n):
    return [f"SYN{i:05d}.1" for i in range(n)]


def write_db(path, n_genomes, n_prot=100, genome_prefix="syn", **kw) -> dict:
    """Write a FastAAI-schema SQLite DB (same tables as the reference's test
    DBs: genome_metadata, scp_data, <acc>_tetras, <acc>_genomes)."""
    g = generate(n_genomes, n_prot, **kw)
    prm = g["params"]
    L = _load()
    if os.path.exists(path):
        os.remove(path)
    con = sqlite3.connect(path)
    gnames = genome_names(n_genomes, genome_prefix)
    pnames = protein_names(n_prot)
    con.execute("CREATE TABLE 'genome_metadata' (genome_name TEXT, genome_id INTEGER PRIMARY KEY, "
                "genome_length INTEGER, genome_class INTEGER, SCP_count INTEGER)")
    con.execute("CREATE TABLE 'scp_data' (genome_id INTEGER, SCP_acc TEXT, SCP_score REAL, tetra_count INTEGER)")
    T = g["T"]
    con.executemany("INSERT INTO genome_metadata VALUES (?,?,?,?,?)",
                    [(gnames[i], i, 0, 0, int((T[:, i] > 0).sum())) for i in range(n_genomes)])
    # scp_data ordered by (protein, genome): the first appearance of protein p
    # in `SELECT DISTINCT scp_acc FROM scp_data` is p (db_helper.hpp:195-215)
    con.executemany("INSERT INTO scp_data VALUES (?,?,?,?)",
                    [(gi, pnames[p], 0.0, int(T[p, gi])) for p in range(n_prot) for gi in range(n_genomes)
                     if T[p, gi] > 0])
    buf = np.empty(1024, dtype=np.int32)
    Lp, Fp, Fg = g["Lp"], g["F_prot"], g["F_genome"]
    tet_of = np.repeat(np.arange(NTETRAMERS, dtype=np.int64), np.diff(Lp))
    for p, acc in enumerate(pnames):
        con.execute(f"CREATE TABLE '{acc}_tetras' (tetramer INTEGER PRIMARY KEY, genomes BLOB)")
        con.execute(f"CREATE TABLE '{acc}_genomes' (genome_id INTEGER PRIMARY KEY, tetramers BLOB)")
        rows = []
        for gi in range(n_genomes):
            n = L.syn_genome_set(ctypes.byref(prm), gi, p, _p(buf))
            if n > 0:
                rows.append((gi, buf[:n].astype("<i4").tobytes()))
        con.executemany(f"INSERT INTO '{acc}_genomes' VALUES (?,?)", rows)
        sel = np.nonzero(Fp == p)[0]
        t = tet_of[sel]
        gg = Fg[sel]
        starts = np.flatnonzero(np.r_[True, t[1:] != t[:-1]]) if len(t) else np.zeros(0, np.int64)
        ends = np.r_[starts[1:], len(t)]
        con.executemany(f"INSERT INTO '{acc}_tetras' VALUES (?,?)",
                        [(int(t[s]), gg[s:e].astype("<i4").tobytes()) for s, e in zip(starts, ends)])
    con.commit()
    con.close()
    g["genome_set"] = gnames
    return g


def write_db_sets(path, sets, n_genomes, n_prot, genome_prefix="syn"):
    """A FastAAI-schema SQLite DB from explicit memberships: sets[(genome,
    protein)] = the genome's tetramer ids in that protein (any order; stored
    sorted).  Same tables and row orders as write_db (for hand-built cases
    such as pairs that share no tetramer)."""
    if os.path.exists(path):
        os.remove(path)
    T = np.zeros((n_prot, n_genomes), np.int64)
    for (gi, p), ts in sets.items():
        T[p, gi] = len(set(ts))
    con = sqlite3.connect(path)
    gnames = genome_names(n_genomes, genome_prefix)
    pnames = protein_names(n_prot)
    con.execute("CREATE TABLE 'genome_metadata' (genome_name TEXT, genome_id INTEGER PRIMARY KEY, "
                "genome_length INTEGER, genome_class INTEGER, SCP_count INTEGER)")
    con.execute("CREATE TABLE 'scp_data' (genome_id INTEGER, SCP_acc TEXT, SCP_score REAL, tetra_count INTEGER)")
    con.executemany("INSERT INTO genome_metadata VALUES (?,?,?,?,?)",
                    [(gnames[i], i, 0, 0, int((T[:, i] > 0).sum())) for i in range(n_genomes)])
    con.executemany("INSERT INTO scp_data VALUES (?,?,?,?)",
                    [(gi, pnames[p], 0.0, int(T[p, gi])) for p in range(n_prot) for gi in range(n_genomes)
                     if T[p, gi] > 0])
    for p, acc in enumerate(pnames):
        con.execute(f"CREATE TABLE '{acc}_tetras' (tetramer INTEGER PRIMARY KEY, genomes BLOB)")
        con.execute(f"CREATE TABLE '{acc}_genomes' (genome_id INTEGER PRIMARY KEY, tetramers BLOB)")
        by_t = {}
        rows = []
        for gi in range(n_genomes):
            ts = sorted(set(sets.get((gi, p), ())))
            if ts:
                rows.append((gi, np.asarray(ts, "<i4").tobytes()))
            for t in ts:
                by_t.setdefault(t, []).append(gi)
        con.executemany(f"INSERT INTO '{acc}_genomes' VALUES (?,?)", rows)
        con.executemany(f"INSERT INTO '{acc}_tetras' VALUES (?,?)",
                        [(t, np.asarray(gs, "<i4").tobytes()) for t, gs in sorted(by_t.items())])
    con.commit()
    con.close()
    return dict(genome_set=gnames, T=T)


def qt_merge(gt: dict, gq: dict) -> dict:
    """QT problem arrays from a target and a query SYN DB (generate() dicts)
    joined as the reference's QT loader does (scp_db.hpp:450-528): per
    (tetramer, protein) block present in both, target genomes then query
    genomes + n_tgt; T side by side; the genome-major lists concatenated
    (entries whose block is absent from F are ignored by the engine).  The
    linear C merge of tools/syn_gen.c (tests/helpers.py:qt_syn is the numpy
    statement of the same join)."""
    L = _load()
    vp = ctypes.c_void_p
    L.syn_qt_merge.restype = ctypes.c_int64
    L.syn_qt_merge.argtypes = [vp, vp, vp, vp, vp, vp, ctypes.c_int32, vp, vp, vp]
    nT = gt["T"].shape[1]
    Lp = np.zeros(NTETRAMERS + 1, dtype=np.int64)
    args = [_p(gt["Lp"]), _p(gt["F_prot"]), _p(gt["F_genome"]), _p(gq["Lp"]), _p(gq["F_prot"]), _p(gq["F_genome"]), nT]
    n = L.syn_qt_merge(*args, _p(Lp), None, None)
    Fp = np.empty(max(n, 1), dtype=np.int32)
    Fg = np.empty(max(n, 1), dtype=np.int32)
    L.syn_qt_merge(*args, _p(Lp), _p(Fp), _p(Fg))
    G_off = np.concatenate([gt["G_off"], gq["G_off"][1:] + gt["G_off"][-1]])
    return dict(Lp=Lp, F_prot=Fp[:n], F_genome=Fg[:n], T=np.concatenate([gt["T"], gq["T"]], axis=1),
                G_off=G_off, G_tet=np.concatenate([gt["G_tet"], gq["G_tet"]]), n_tgt=nT, n_qry=gq["T"].shape[1])
