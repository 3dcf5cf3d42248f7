"""Both orientations of the SCP membership reach the same kernels
(pfaai_build.hpp): F-only input (the reference's own DataStructInterface
classes hand over F) gets its genome-major lists G built on the device, and
G-only input (the CLI's `<p>_genomes` ingest) gets F built on the device --
either way pfaai_run launches k_rows_pl, and S / N / AJI / |E| are bit-exact
against the F + G load and the pinned oracle, in all three modes."""
import numpy as np
import pytest

import oracle as O
from helpers import ALL_FIXTURES, all_ds, jac_fixture, qsub_ds, qt_ds, qt_syn
from parfastaai_amd import _capi, syn
from parfastaai_amd.datastruct import ParFAAIData, ParFAAIQSubData
from parfastaai_amd.impl import ParFAAIImpl

pytestmark = pytest.mark.gpu


def _problems():
    g = syn.generate(700, 40, clade_size=12)
    yield "all", ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"]).with_genome_major(
        g["G_off"], g["G_tet"]).problem()
    g = syn.generate(500, 30, clade_size=10)
    q = [g["genome_set"][i] for i in range(3, 500, 11)]
    yield "qsub", ParFAAIQSubData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"], g["genome_set"], q
                                             ).with_genome_major(g["G_off"], g["G_tet"]).problem()
    yield "qt", qt_syn(dict(n_tgt=400, n_qry=90, n_prot=30, clade_size=9), genome_major=True).problem()


def _strip(pb, drop):
    out = dict(pb)
    for k in drop:
        out.pop(k, None)
    return out


@pytest.mark.parametrize("compat", [0, _capi.FLAG_REF_COMPAT], ids=["default", "ref-compat"])
def test_f_only_and_g_only_equal_f_plus_g(engine, compat):
    for name, pb in _problems():
        engine.load(**pb)
        # both given: the transposition sort proves G against F (QT: G of both DBs, checked by search)
        assert engine.load_info() == ("as_given" if name == "qt" else "g_checked"), name
        ref = engine.compute(compat)
        st = engine.stats()
        assert st["rows_kernel"] == "pl", name
        ne = O.Problem(pb, compat=bool(compat)).count_e() if name != "qt" else None
        if ne is not None:
            assert st["n_events"] == ne, name
        for drop in (("G_off", "G_tet"), ("Lp", "F_prot", "F_genome")):
            if name == "qt" and drop[0] == "Lp":
                continue  # QT G of both DBs != the joined F (covered below)
            engine.load(**_strip(pb, drop))
            # F only: G by the sort, list bounds from T (QT's T counts both DBs' full lists, not the
            # joined F: the general radix sort); G only: F by the sort
            want = "f_from_g" if drop[0] == "Lp" else ("legacy" if name == "qt" else "g_from_f")
            assert engine.load_info() == want, (name, drop)
            got = engine.compute(compat)
            st2 = engine.stats()
            assert st2["rows_kernel"] == "pl", (name, drop)
            assert st2["n_events"] == st["n_events"], (name, drop)
            for a, b in zip(got, ref):
                assert np.array_equal(a, b), (name, drop)


def test_qt_from_both_dbs_genome_lists(engine):
    """-r through the CLI's ingest: G holds every tetramer of both DBs, F is
    built from it on the device (a superset of the reference's inner-joined
    F); the extra runs hold no query-target pair, so S, N, AJI and |E| equal
    the joined-F run, ref-compat included."""
    from parfastaai_amd import syn as S
    kw = dict(n_prot=30, clade_size=9)
    ds = qt_syn(dict(n_tgt=300, n_qry=70, **kw), genome_major=True)
    pb = ds.problem()
    for compat in (0, _capi.FLAG_REF_COMPAT):
        engine.load(**pb)
        ref = engine.compute(compat)
        ne = engine.stats()["n_events"]
        engine.load(**_strip(pb, ("Lp", "F_prot", "F_genome")))
        got = engine.compute(compat)
        assert engine.stats()["rows_kernel"] == "pl"
        assert engine.stats()["n_events"] == ne
        for a, b in zip(got, ref):
            assert np.array_equal(a, b)


@pytest.mark.parametrize("prefix,jname", ALL_FIXTURES)
def test_reference_fixtures_f_only_run_pl(engine, prefix, jname):
    """The reference's F / Lc / T fixtures (F only, as its DataStruct classes
    hold them) run on k_rows_pl and reproduce its JAC / AJI bit for bit."""
    impl = ParFAAIImpl(all_ds(prefix), ref_compat=True, engine=engine)
    impl.run()
    assert impl.stats["rows_kernel"] == "pl"
    J, A = jac_fixture(jname)
    jac = impl.getJAC()
    assert np.array_equal(jac["N"], J["N"]) and np.array_equal(jac["S"], J["S"])
    assert np.array_equal(impl.getAJI(), A)


def test_qsub_and_qt_fixtures_f_only_run_pl(engine):
    for ds, name in ((qsub_ds(), "xdb_qry_subset"), (qt_ds(), "xdb_qt")):
        impl = ParFAAIImpl(ds, ref_compat=True, engine=engine)
        impl.run()
        assert impl.stats["rows_kernel"] == "pl"
        J, A = jac_fixture(name)
        assert np.array_equal(impl.getJAC()["S"], J["S"]) and np.array_equal(impl.getAJI(), A)
