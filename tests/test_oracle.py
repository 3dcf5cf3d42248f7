"""Pin the CPU oracle before trusting it (CPU only).

Every JAC/AJI/E golden vector the reference's own test-suite holds
(tests/pfaai_tests.cpp:173-683 of the reference) and the reference binary's
own outputs on synthetic DBs (tests/golden/ref_*.csv.gz) must be reproduced
bit-exactly by oracle/pfaai_oracle.c.
"""
import numpy as np
import pytest

import oracle as O
from helpers import ALL_FIXTURES, all_ds, gpath, jac_fixture, qsub_ds, qt_ds, syn_case, text, xantho_names
from parfastaai_amd import formats as fm


@pytest.mark.parametrize("prefix,jname", ALL_FIXTURES)
@pytest.mark.parametrize("compat", [True, False])
def test_oracle_all_vs_all_jac_aji(prefix, jname, compat):
    # reference: compute_JAC_AJI / compute_subset{1,2}_JAC_AJI (pfaai_tests.cpp:355-453)
    ds = all_ds(prefix)
    r = O.Problem(ds.problem(), compat=compat).ref_run()
    J, A = jac_fixture(jname)
    assert np.array_equal(r["genomeA"], J["genomeA"]) and np.array_equal(r["genomeB"], J["genomeB"])
    assert np.array_equal(r["N"], J["N"])
    assert np.array_equal(r["S"], J["S"])  # bit-exact (reference tolerance is 1e-7)
    assert np.array_equal(r["AJI"], A)  # exact, as pfaai_tests.cpp:383


@pytest.mark.parametrize("prefix", ["xdb_subset1", "xdb_subset2"])
def test_oracle_sorted_e(prefix):
    # construct_subset{1,2}_LFTE: sorted E == fixture (pfaai_tests.cpp:232-353)
    ds = all_ds(prefix)
    E = O.Problem(ds.problem()).sorted_e()
    assert np.array_equal(E, fm.read_e_array(gpath(prefix + "_sorted_e_array.bin")))


def test_oracle_xantho_e_size_and_extents():
    # |E| = sum of the per-thread E sizes; per-pair extents = sum_p c
    ds = all_ds("xanthodb")
    pr = O.Problem(ds.problem())
    esize = fm.read_vec_i32(gpath("xanthodb_e_size.bin"))
    assert pr.count_e() == esize.sum() == 2608722
    st = fm.read_vec_i32(gpath("xanthodb_gpe_starts.bin"))
    en = fm.read_vec_i32(gpath("xanthodb_gpe_ends.bin"))
    E = pr.sorted_e()
    # run lengths of E by (a, b) in JAC order
    key = E[:, 1].astype(np.int64) * 20 + E[:, 2]
    _, counts = np.unique(key, return_counts=True)
    assert np.array_equal(counts, en - st + 1)


def test_oracle_query_subset():
    # query_subset (pfaai_tests.cpp:455-494) + its CSV fixture
    ds = qsub_ds()
    r = O.Problem(ds.problem(), compat=True).ref_run()
    J, A = jac_fixture("xdb_qry_subset")
    assert np.array_equal(r["genomeA"], J["genomeA"]) and np.array_equal(r["genomeB"], J["genomeB"])
    assert np.array_equal(r["S"], J["S"]) and np.array_equal(r["N"], J["N"])
    assert np.array_equal(r["AJI"], A)
    M = ds.output_matrix(r["genomeA"], r["genomeB"], r["AJI"])
    txt = fm.csv_text(ds.refQuerySet(), ds.refTargetSet(), M)
    assert txt == text("qsub_test_output_matrix_wheader.csv")


def test_oracle_qt_ref_compat():
    # qt_compute_JAC_AJI (pfaai_tests.cpp:653-683): only the reference's
    # T-index quirk reproduces xdb_qt_jac.bin
    ds = qt_ds()
    r = O.Problem(ds.problem(), compat=True).ref_run()
    J, A = jac_fixture("xdb_qt")
    assert np.array_equal(r["genomeA"], J["genomeA"]) and np.array_equal(r["genomeB"], J["genomeB"])
    assert np.array_equal(r["S"], J["S"]) and np.array_equal(r["N"], J["N"])
    assert np.array_equal(r["AJI"], A)
    E = O.Problem(ds.problem()).sorted_e()
    assert np.array_equal(E, fm.read_e_array(gpath("xdb_qt_sorted_e_array.bin")))


def test_oracle_xantho_csv_bytes():
    ds = all_ds("xanthodb", xantho_names())
    r = O.Problem(ds.problem()).ref_run()
    M = ds.output_matrix(r["genomeA"], r["genomeB"], r["AJI"])
    assert fm.csv_text(ds.refQuerySet(), ds.refTargetSet(), M) == text("xanthodb_aji_matrix_wheader.csv")


@pytest.mark.parametrize("name", ["all48", "all32_sparse", "qsub40", "qt12", "qt8x12"])
def test_oracle_vs_reference_binary(name):
    ds, M_ref = syn_case(name)
    compat = name.startswith("qt")
    r = O.Problem(ds.problem(), compat=compat).ref_run()
    ga, gb = ds.initJAC(compat)
    M = ds.output_matrix(ga, gb, r["AJI"])
    assert np.array_equal(M, M_ref)


@pytest.mark.parametrize("name", ["all48", "qsub40", "qt12"])
def test_dense_restatement_matches_ref(name):
    """Appendix-A dense formulation == E/sort formulation (correct mode)."""
    ds, _ = syn_case(name)
    pr = O.Problem(ds.problem(), compat=False)
    r = pr.ref_run()
    S, N, ne = pr.dense_rows(0, pr.mode.n_ids)
    ga, gb = ds.initJAC(False)
    assert ne == r["n_events"]
    assert np.array_equal(S[ga, gb], r["S"])
    assert np.array_equal(N[ga, gb], r["N"])


@pytest.mark.parametrize("name", ["all48", "all32_sparse", "qt12", "syn300", "qt_syn"])
def test_full_rows_matches_ref(name):
    """oracle_full_rows (the whole-output digests' restatement, row windows,
    OpenMP over rows) == the E/sort restatement pinned above (correct mode),
    in JAC order, over uneven row windows."""
    from helpers import qt_syn
    from parfastaai_amd import syn
    from parfastaai_amd.datastruct import ParFAAIData

    if name == "syn300":
        g = syn.generate(300, 24, clade_size=10)
        ds = ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"])
    elif name == "qt_syn":
        ds = qt_syn(dict(n_tgt=120, n_qry=17, n_prot=12, clade_size=8))
    else:
        ds, _ = syn_case(name)
    pr = O.Problem(ds.problem(), compat=False)
    r = pr.ref_run()
    n = pr.n_pairs()
    S, N, A = np.full(n, -1.0), np.full(n, -1, np.int32), np.full(n, -1.0)
    rows = pr.mode.n_ids if pr.mode.mode == 0 else pr.mode.n_qry
    cuts = sorted({0, rows, *[min(rows, x) for x in (1, 7, rows // 3, rows // 2 + 5)]})
    ne = 0
    for lo, hi in zip(cuts[:-1], cuts[1:]):
        if pr.mode.mode == 0:
            f = pr.mode.n_ids * lo - (lo + 1) * lo // 2
            c = pr.mode.n_ids * hi - (hi + 1) * hi // 2 - f
        else:
            f, c = lo * pr.mode.n_tgt, (hi - lo) * pr.mode.n_tgt
        ne += pr.full_rows(lo, hi, S[f:f + c], N[f:f + c], A[f:f + c])
    assert ne == r["n_events"]
    assert np.array_equal(N, r["N"]) and np.array_equal(S, r["S"]) and np.array_equal(A, r["AJI"])
