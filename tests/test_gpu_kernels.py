"""Kernel-level GPU checks: the row kernels' exact small-integer division is
bit-identical to IEEE '/', and every selectable row-kernel variant
(PFAAI_ROWS_KERNEL, read by the diagnostics build's pfaai_run) reproduces the
oracle bit-exactly; the release build ignores every A/B switch."""
import os

import numpy as np
import pytest

import oracle as O
from parfastaai_amd import syn
from parfastaai_amd.datastruct import ParFAAIData
from parfastaai_amd.impl import ParFAAIImpl

pytestmark = pytest.mark.gpu


def test_exact_division(engine):
    # T entries are < 2^16 (checked at load): c <= 65535 and c <= d < 2^17,
    # the whole domain, 6.4e9 quotients
    assert engine.debug_div_check(65535, (1 << 17) - 1) == 0


@pytest.fixture(scope="module")
def syn_problem():
    g = syn.generate(300, 24, clade_size=10)
    ds = ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"]).with_genome_major(g["G_off"], g["G_tet"])
    ref = O.Problem(ds.problem()).ref_run()
    return ds, ref


@pytest.mark.parametrize("variant", ["pl", "pl512", "fused", "worklist"])
def test_row_kernel_variants(diag_engine, syn_problem, variant):
    ds, ref = syn_problem
    os.environ["PFAAI_ROWS_KERNEL"] = variant
    try:
        impl = ParFAAIImpl(ds, engine=diag_engine)
        impl.run()
        assert impl.engine.stats()["rows_kernel"] == variant
    finally:
        os.environ.pop("PFAAI_ROWS_KERNEL", None)
    jac = impl.getJAC()
    assert impl.n_events() == ref["n_events"]
    assert np.array_equal(jac["N"], ref["N"]) and np.array_equal(jac["S"], ref["S"])
    assert np.array_equal(impl.getAJI(), ref["AJI"])


def test_release_library_ignores_ab_switches(engine, syn_problem, monkeypatch):
    """Production kernel choice does not depend on the environment: the
    release library runs k_rows_pl with a bogus PFAAI_ROWS_KERNEL and a
    counter-word cap set, and gives the oracle's results."""
    ds, ref = syn_problem
    for k, v in (("PFAAI_ROWS_KERNEL", "bogus"), ("PFAAI_PL_KWMAX", "1"), ("PFAAI_PL_WINDOWS", "0"),
                 ("PFAAI_XCD_CHUNK", "3"), ("PFAAI_PL_PRIO", "0"), ("PFAAI_BLK_END_TILE", "7")):
        monkeypatch.setenv(k, v)
    impl = ParFAAIImpl(ds, engine=engine)
    assert impl.run() == 0
    assert impl.engine.stats()["rows_kernel"] == "pl"
    jac = impl.getJAC()
    assert np.array_equal(jac["N"], ref["N"]) and np.array_equal(jac["S"], ref["S"])
    assert np.array_equal(impl.getAJI(), ref["AJI"])


def _problem_from_triples(n, P, trip):
    """(protein, genome, tetramer) triples -> the loader's arrays (F by
    (tetramer, protein, genome), Lp, T[P][n], genome-major G)."""
    p, g, t = (np.asarray(x, np.int64) for x in trip)
    o = np.lexsort((g, p, t))
    Lp = np.zeros(160001, np.int64)
    np.cumsum(np.bincount(t, minlength=160000), out=Lp[1:])
    T = np.zeros((P, n), np.int32)
    np.add.at(T, (p, g), 1)
    og = np.lexsort((t, p, g))
    G_off = np.zeros(n * P + 1, np.int64)
    np.cumsum(np.bincount(g * P + p, minlength=n * P), out=G_off[1:])
    return dict(mode=0, n_ids=n, n_prot=P, Lp=Lp, F_prot=p[o].astype(np.int32), F_genome=g[o].astype(np.int32),
                T=T, G_off=G_off, G_tet=t[og].astype(np.int32))


def test_run_end_table_heavy_tetramer(engine):
    """k_blk_end with a tetramer held by every (genome, protein): its tile
    holds 600 000 F entries, past the granule table's 8 192 x 64, so that
    tile looks tetramers up by binary search while the others use the table;
    the all-vs-all rows (G_pos walks over the end table) equal the oracle."""
    rng = np.random.default_rng(11)
    n, P = 600, 1000
    gg, pp = np.meshgrid(np.arange(n), np.arange(P), indexing="ij")
    ts = np.concatenate([np.full((n, P, 1), 777), rng.integers(0, 160000, (n, P, 3)),
                         rng.integers(20000, 20040, (n, P, 1))], axis=2)
    ts.sort(axis=2)
    keep = np.ones(ts.shape, bool)
    keep[:, :, 1:] = ts[:, :, 1:] != ts[:, :, :-1]  # a set per (genome, protein)
    rep = lambda x: np.broadcast_to(x[:, :, None], ts.shape)[keep]  # noqa: E731
    pb = _problem_from_triples(n, P, (rep(pp), rep(gg), ts[keep]))
    engine.load(**pb)
    pr = O.Problem(pb)
    aji, S, N = engine.compute(0)
    st = engine.stats()
    assert st["rows_kernel"] == "pl"
    assert st["n_events"] == pr.count_e()
    for a in (0, 1, 299, n - 2):
        So, No, _ = pr.dense_rows(a, a + 1)
        b = np.arange(a + 1, n)
        k = n * a + b - (a + 2) * (a + 1) // 2
        assert np.array_equal(N[k], No[0, b]) and np.array_equal(S[k], So[0, b]), a
