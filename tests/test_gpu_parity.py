"""HIP engine parity (GPU): every result goes through libpfaai_hip.so and is
compared with the reference's golden vectors or the pinned CPU oracle.

Bar: integer counts / N / genome ids bit-exact; S and AJI bit-exact too
(fp64 sums in ascending protein order, IEEE division), which is stricter
than north_star's 1e-6 AJI tolerance (checked as well, AJI_TOL).
"""
import numpy as np
import pytest

import oracle as O
from helpers import ALL_FIXTURES, all_ds, gpath, jac_fixture, qsub_ds, qt_ds, syn_case
from parfastaai_amd import formats as fm
from parfastaai_amd import syn
from parfastaai_amd.datastruct import ParFAAIData, ParFAAIQSubData
from parfastaai_amd.impl import ParFAAIImpl

pytestmark = pytest.mark.gpu
AJI_TOL = 1e-6  # north_star float tolerance (we assert exact equality as well)


def _assert_jac(jac, aji, J, A):
    assert np.array_equal(jac["genomeA"], J["genomeA"])
    assert np.array_equal(jac["genomeB"], J["genomeB"])
    assert np.array_equal(jac["N"], J["N"])
    assert np.max(np.abs(aji - A)) < AJI_TOL
    assert np.array_equal(jac["S"], J["S"])
    assert np.array_equal(aji, A)


@pytest.mark.parametrize("prefix,jname", ALL_FIXTURES)
@pytest.mark.parametrize("compat", [True, False])
def test_hip_all_vs_all_fixtures(engine, prefix, jname, compat):
    impl = ParFAAIImpl(all_ds(prefix), ref_compat=compat, engine=engine)
    assert impl.run() == 0
    J, A = jac_fixture(jname)
    _assert_jac(impl.getJAC(), impl.getAJI(), J, A)


def test_hip_xantho_events(engine):
    impl = ParFAAIImpl(all_ds("xanthodb"), engine=engine)
    impl.run()
    assert impl.n_events() == fm.read_vec_i32(gpath("xanthodb_e_size.bin")).sum() == 2608722


def test_hip_query_subset_fixture(engine):
    impl = ParFAAIImpl(qsub_ds(), ref_compat=True, engine=engine)
    impl.run()
    J, A = jac_fixture("xdb_qry_subset")
    _assert_jac(impl.getJAC(), impl.getAJI(), J, A)


def test_hip_qt_fixture_ref_compat(engine):
    impl = ParFAAIImpl(qt_ds(), ref_compat=True, engine=engine)
    impl.run()
    J, A = jac_fixture("xdb_qt")
    _assert_jac(impl.getJAC(), impl.getAJI(), J, A)


def test_hip_qt_correct_vs_oracle(engine):
    ds = qt_ds()
    impl = ParFAAIImpl(ds, ref_compat=False, engine=engine)
    impl.run()
    r = O.Problem(ds.problem(), compat=False).ref_run()
    assert np.array_equal(impl.getJAC()["S"], r["S"]) and np.array_equal(impl.getAJI(), r["AJI"])


@pytest.mark.parametrize("prefix", ["xdb_subset1", "xdb_subset2"])
def test_hip_counts_equal_sorted_e_runs(engine, prefix):  # noqa: D103
    """Integer intersection counts c(p,a,b) == run-lengths of the reference's sorted E."""
    ds = all_ds(prefix)
    impl = ParFAAIImpl(ds, engine=engine)
    E = fm.read_e_array(gpath(prefix + "_sorted_e_array.bin"))
    n = ds.n_genomes
    for a in range(n):
        C = impl.row_counts(a)
        ref = np.zeros_like(C)
        sel = E[E[:, 1] == a]
        np.add.at(ref, (sel[:, 0], sel[:, 2]), 1)
        assert np.array_equal(C, ref)


def test_hip_qt_counts_equal_sorted_e_runs(engine):
    ds = qt_ds()
    impl = ParFAAIImpl(ds, engine=engine)
    E = fm.read_e_array(gpath("xdb_qt_sorted_e_array.bin"))
    for q in range(ds.n_qry):
        C = impl.row_counts(q)
        ref = np.zeros_like(C)
        sel = E[E[:, 1] == ds.n_tgt + q]
        np.add.at(ref, (sel[:, 0], sel[:, 2]), 1)
        assert np.array_equal(C, ref)


@pytest.mark.parametrize("gm", [False, True], ids=["F-only", "genome-major"])
@pytest.mark.parametrize("name", ["all48", "all32_sparse", "qsub40", "qt12"])
def test_hip_vs_reference_binary_outputs(engine, name, gm):
    ds, M_ref = syn_case(name, genome_major=gm)
    compat = name.startswith("qt")
    impl = ParFAAIImpl(ds, ref_compat=compat, engine=engine)
    impl.run()
    assert np.array_equal(impl.output_matrix(), M_ref)


def _syn_all(n, P, gm, **kw):
    g = syn.generate(n, P, **kw)
    ds = ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"], g["genome_set"])
    return ds.with_genome_major(g["G_off"], g["G_tet"]) if gm else ds


@pytest.mark.parametrize("gm", [False, True], ids=["F-only", "genome-major"])
@pytest.mark.parametrize("n,P,k", [(300, 100, 20), (130, 40, 7), (2, 3, 1)])
def test_hip_vs_oracle_synthetic(engine, n, P, k, gm):
    ds = _syn_all(n, P, gm, clade_size=k)
    impl = ParFAAIImpl(ds, engine=engine)
    impl.run()
    r = O.Problem(ds.problem()).ref_run()
    jac = impl.getJAC()
    assert impl.n_events() == r["n_events"]
    assert np.array_equal(jac["N"], r["N"]) and np.array_equal(jac["S"], r["S"])
    assert np.array_equal(impl.getAJI(), r["AJI"])


@pytest.mark.parametrize("gm", [False, True], ids=["F-only", "genome-major"])
def test_hip_unsorted_query_list_correct_mode(engine, gm):
    g = syn.generate(60, 12, clade_size=6)
    q = [g["genome_set"][i] for i in (50, 3, 17, 40, 8)]
    ds = ParFAAIQSubData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"], g["genome_set"], q)
    if gm:
        ds.with_genome_major(g["G_off"], g["G_tet"])
    impl = ParFAAIImpl(ds, engine=engine)
    impl.run()
    r = O.Problem(ds.problem(), compat=False).ref_run()
    assert np.array_equal(impl.getJAC()["S"], r["S"]) and np.array_equal(impl.getAJI(), r["AJI"])


def _zero_overlap_ds():
    # 3 genomes, 2 proteins; genome 2 shares no tetramer with genome 0
    blocks = {  # (tetramer, protein) -> genomes
        (5, 0): [0, 1], (9, 0): [1, 2], (11, 1): [0, 1], (20, 1): [2], (30, 0): [0],
    }
    t_l, p_l, g_l = [], [], []
    for (t, p), gs in sorted(blocks.items()):
        for g in gs:
            t_l.append(t); p_l.append(p); g_l.append(g)
    Lc = np.bincount(np.array(t_l), minlength=160000)
    F = np.stack([p_l, g_l], axis=1)
    T = np.zeros((2, 3), np.int32)
    for (t, p), gs in blocks.items():
        for g in gs:
            T[p, g] += 1
    return ParFAAIData(Lc, F, T)


@pytest.mark.parametrize("compat", [True, False])
def test_hip_zero_overlap_pair(engine, compat):
    """compat reproduces the reference's J of E[0]'s
    protein; the default writes 0."""
    ds = _zero_overlap_ds()
    impl = ParFAAIImpl(ds, ref_compat=compat, engine=engine)
    impl.run()
    r = O.Problem(ds.problem(), compat=compat).ref_run()
    jac = impl.getJAC()
    assert np.array_equal(jac["N"], r["N"]) and np.array_equal(jac["S"], r["S"])
    assert np.array_equal(impl.getAJI(), r["AJI"])
    k = ds.genomePairToIndex(0, 2)
    assert (jac["N"][k] == 1) == compat


@pytest.mark.parametrize("gm", [False, True], ids=["F-only", "genome-major"])
def test_hip_row_sharding_matches_full(engine, gm):
    """Rows split over 'ranks' (pfaai_run on row ranges) == one full run."""
    ds = _syn_all(257, 30, gm, clade_size=9)
    impl = ParFAAIImpl(ds, engine=engine)
    impl.run()
    full = impl.getAJI()
    n_rows, n_pairs = engine.shape()
    out = np.zeros(n_pairs)
    for rb, re in [(0, 3), (3, 90), (90, 256), (256, 257)]:
        first, count = engine.row_span(rb, re)
        if count == 0:
            continue
        d = engine.alloc(count * 8)
        try:
            engine.run(rb, re, 0, d - first * 8)
            engine.synchronize()
            out[first:first + count] = engine.d2h(d, count, np.float64)
        finally:
            engine.free(d)
    assert np.array_equal(out, full)


@pytest.mark.parametrize("gm", [False, True], ids=["F-only", "genome-major"])
def test_hip_c2_scale_properties(engine, gm):
    """Full C2-size run (SYN 2000 x 100): |E| equals the oracle's count,
    sampled rows equal the oracle exactly, AJI in [0, 1]."""
    ds = _syn_all(2000, 100, gm)
    impl = ParFAAIImpl(ds, engine=engine)
    impl.run()
    pr = O.Problem(ds.problem())
    assert impl.n_events() == pr.count_e()
    aji, jac = impl.getAJI(), impl.getJAC()
    assert np.all((aji >= 0) & (aji <= 1)) and np.all(jac["N"] >= 1) and np.all(jac["N"] <= 100)
    for lo in (0, 997, 1996):
        S, N, _ = pr.dense_rows(lo, lo + 4)
        for a in range(lo, lo + 4):
            b = np.arange(a + 1, 2000)
            k = ds.genomePairToIndex(a, b)
            assert np.array_equal(jac["S"][k], S[a - lo, b]) and np.array_equal(jac["N"][k], N[a - lo, b])
