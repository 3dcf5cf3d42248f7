"""Edge cases of the HIP engine vs the oracle (GPU): column chunking (rows
wider than one LDS counter row), many proteins, empty genomes / proteins,
single-query subsets, QT with nQ != nT, both work-list paths."""
import numpy as np
import pytest

import oracle as O
from helpers import qt_syn
from parfastaai_amd import syn
from parfastaai_amd.datastruct import ParFAAIData, ParFAAIQSubData
from parfastaai_amd.impl import ParFAAIImpl

pytestmark = pytest.mark.gpu
GM = pytest.mark.parametrize("gm", [False, True], ids=["F-only", "genome-major"])


def _ds_all(g, gm):
    ds = ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"])
    return ds.with_genome_major(g["G_off"], g["G_tet"]) if gm else ds


def _check(engine, ds, compat=False, rows=None):
    impl = ParFAAIImpl(ds, ref_compat=compat, engine=engine)
    impl.run()
    pr = O.Problem(ds.problem(), compat=compat)
    jac = impl.getJAC()
    if rows is None:
        r = pr.ref_run()
        assert impl.n_events() == r["n_events"]
        assert np.array_equal(jac["N"], r["N"]) and np.array_equal(jac["S"], r["S"])
        assert np.array_equal(impl.getAJI(), r["AJI"])
    else:  # sampled rows against the dense restatement (large problems)
        assert impl.n_events() == pr.count_e()
        n = pr.mode.n_ids
        for lo in rows:
            S, N, _ = pr.dense_rows(lo, lo + 1)
            b = np.arange(lo + 1, n)
            k = ds.genomePairToIndex(lo, b)
            assert np.array_equal(jac["S"][k], S[0, b]) and np.array_equal(jac["N"][k], N[0, b])
    return impl


@GM
def test_column_chunks_all_vs_all(engine, gm):
    """N = 21 000 > 20 480 columns per LDS row: rows split into 2 chunks."""
    g = syn.generate(21000, 2, clade_size=50, n_random=1)
    _check(engine, _ds_all(g, gm), rows=[0, 1, 7, 400, 20479, 20480, 20999 - 1])


@GM
def test_many_proteins(engine, gm):
    g = syn.generate(40, 700, clade_size=4, n_random=2)
    _check(engine, _ds_all(g, gm))


@GM
def test_sparse_genomes_and_empty_proteins(engine, gm):
    # has=0.3: most (genome, protein) sets are empty; keep=0.5
    g = syn.generate(120, 30, clade_size=6, has=0.3, keep=0.5)
    _check(engine, _ds_all(g, gm))
    _check(engine, _ds_all(g, gm), compat=True)


@GM
def test_single_query_subset(engine, gm):
    g = syn.generate(50, 10, clade_size=5)
    ds = ParFAAIQSubData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"], g["genome_set"],
                                    [g["genome_set"][17]])
    if gm:
        ds.with_genome_major(g["G_off"], g["G_tet"])
    _check(engine, ds)
    _check(engine, ds, compat=True)


@GM
@pytest.mark.parametrize("nT,nQ", [(30, 7), (7, 30), (20, 20)])
def test_qt_rectangular(engine, gm, nT, nQ):
    ds = qt_syn(dict(n_tgt=nT, n_qry=nQ, n_prot=12, clade_size=5), genome_major=gm)
    _check(engine, ds)
    _check(engine, ds, compat=True)


@GM
def test_qt_wide_targets(engine, gm):
    """QT rows wider than one column chunk at KW = 5 (12 000 targets)."""
    ds = qt_syn(dict(n_tgt=12000, n_qry=16, n_prot=6, clade_size=20), genome_major=gm)
    _check(engine, ds)


def _genome_major(Lp, Fp, Fg, n_ids, P):
    """G_off / G_tet from F: the (genome, protein) lists of ascending tetramers."""
    t = np.repeat(np.arange(160000, dtype=np.int32), np.diff(Lp))
    key = Fg.astype(np.int64) * P + Fp
    order = np.argsort(key, kind="stable")  # F is tetramer-ordered: lists stay ascending
    G_off = np.zeros(n_ids * P + 1, dtype=np.int64)
    G_off[1:] = np.cumsum(np.bincount(key, minlength=n_ids * P))
    return G_off, t[order]


@pytest.mark.parametrize("k", [37, 38, 39, 40])
def test_run_at_end_of_F(engine, k):
    """The last run of F ends at |F| with |F| % 4 = 0..3: its final 16-B member
    loads cross the end of the array (padding must read as data, not zeros)."""
    g = syn.generate(61, 3, clade_size=6)
    Lp, Fp, Fg, T = g["Lp"], g["F_prot"], g["F_genome"], g["T"].copy()
    last = slice(Lp[159999], Lp[160000])  # replace tetramer 159999's block with one run of k genomes
    for p_, g_ in zip(Fp[last], Fg[last]):
        T[p_, g_] -= 1
    Fp = np.concatenate([Fp[: Lp[159999]], np.full(k, 2, np.int32)])
    Fg = np.concatenate([Fg[: Lp[159999]], np.arange(k, dtype=np.int32)])
    T[2, :k] += 1
    Lp = Lp.copy()
    Lp[160000] = len(Fp)
    ds = ParFAAIData.from_split(Lp, Fp, Fg, T)
    ds.with_genome_major(*_genome_major(Lp, Fp, Fg, 61, 3))
    _check(engine, ds)


def test_genome_without_tetramers(engine):
    """A genome with no entries at all (all its pairs have zero overlap)."""
    g = syn.generate(30, 6, clade_size=5)
    keep = g["F_genome"] != 12
    Lc = np.bincount(np.repeat(np.arange(160000), np.diff(g["Lp"]))[keep], minlength=160000)
    F = np.stack([g["F_prot"][keep], g["F_genome"][keep]], axis=1)
    T = g["T"].copy()
    T[:, 12] = 0
    ds = ParFAAIData(Lc, F, T)
    _check(engine, ds)
    _check(engine, ds, compat=True)
