"""pfaai_stream_matrix: printOutput's dense nQ x nT matrix (main.cpp:143-154)
produced tile by tile on the device (full rows, kModeFull: the mirror half of
ALL / QSUB is computed rather than copied) equals the matrix the reference
builds from the JAC tuples -- bit-exact for every tile height, row range, mode
and both division conventions, plus a case wide enough for column windows."""
import numpy as np
import pytest

from helpers import ALL_FIXTURES, all_ds, qsub_ds, qt_ds, qt_syn
from parfastaai_amd import _capi, syn
from parfastaai_amd.datastruct import ParFAAIData, ParFAAIQSubData

pytestmark = pytest.mark.gpu

COMPAT = [0, _capi.FLAG_REF_COMPAT]


def _dense(engine, ds, flags):
    aji = engine.compute(flags)[0]
    return ds.output_matrix(*ds.initJAC(bool(flags & _capi.FLAG_REF_COMPAT)), aji)


def _streamed(engine, r0, r1, tile_rows, flags):
    got = []

    def sink(rb, re, block):
        got.append((rb, re, block.copy()))

    ne = engine.stream_matrix(r0, r1, tile_rows, flags, sink)
    pos = r0
    for rb, re, _ in got:  # tiles in row order, covering [r0, r1) exactly
        assert rb == pos and re > rb
        pos = re
    assert pos == r1
    return (np.concatenate([b for _, _, b in got]) if got else np.zeros((0, 0))), len(got), ne


def _cases():
    g = syn.generate(600, 35, clade_size=11)
    yield "syn-all", ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"], g["genome_set"]
                                            ).with_genome_major(g["G_off"], g["G_tet"])
    g = syn.generate(450, 30, clade_size=10)
    q = [g["genome_set"][i] for i in range(2, 450, 13)]
    yield "syn-qsub", ParFAAIQSubData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"], g["genome_set"], q
                                                 ).with_genome_major(g["G_off"], g["G_tet"])
    yield "syn-qt", qt_syn(dict(n_tgt=350, n_qry=60, n_prot=30, clade_size=9), genome_major=True)
    yield "xanthodb-qsub", qsub_ds()
    yield "xdb_qt", qt_ds()


@pytest.mark.parametrize("flags", COMPAT, ids=["default", "ref-compat"])
def test_stream_matrix_equals_dense_fill(engine, flags):
    for name, ds in _cases():
        engine.load(**ds.problem())
        M = _dense(engine, ds, flags)
        rows = M.shape[0]
        for tr in (1, 7, rows):
            got, nt, _ = _streamed(engine, 0, rows, tr, flags)
            assert nt == -(-rows // tr), (name, tr)
            assert got.shape == M.shape, name
            assert np.array_equal(got, M, equal_nan=True), (name, tr)
        if rows > 10:  # a row range that is not a multiple of the tile
            got, _, _ = _streamed(engine, 3, rows - 2, 4, flags)
            assert np.array_equal(got, M[3:rows - 2], equal_nan=True), name


@pytest.mark.parametrize("prefix,_j", ALL_FIXTURES)
def test_stream_matrix_reference_fixtures(engine, prefix, _j):
    """The reference's ALL-mode golden DBs (tests/golden/<p>_*): symmetric
    matrix with a zero diagonal, == the dense fill of the JAC vector."""
    ds = all_ds(prefix)
    engine.load(**ds.problem())
    for flags in COMPAT:
        M = _dense(engine, ds, flags)
        got, _, _ = _streamed(engine, 0, M.shape[0], 5, flags)
        assert np.array_equal(got, M, equal_nan=True)
        assert np.array_equal(got, got.T, equal_nan=True)
        assert not np.diag(got).any()


def test_stream_matrix_sink_stop_and_range_errors(engine):
    g = syn.generate(200, 20, clade_size=8)
    ds = ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"], g["genome_set"])
    engine.load(**ds.problem())
    seen = []
    with pytest.raises(_capi.PfaaiError):
        engine.stream_matrix(0, 200, 16, 0, lambda rb, re, b: seen.append(rb) or True)
    assert seen == [0]  # stopped after the first tile
    for r0, r1 in ((-1, 5), (5, 201), (10, 5)):
        with pytest.raises(_capi.PfaaiError):
            engine.stream_matrix(r0, r1, 4, 0, lambda *a: None)
    _, nt, _ = _streamed(engine, 50, 50, 4, 0)
    assert nt == 0
    # QT with the reference's ids and nQ > nT: its rows collide, not streamable
    ds = qt_syn(dict(n_tgt=30, n_qry=50, n_prot=10, clade_size=5))
    engine.load(**ds.problem())
    with pytest.raises(_capi.PfaaiError):
        engine.stream_matrix(0, 50, 8, _capi.FLAG_REF_COMPAT, lambda *a: None)
    got, _, _ = _streamed(engine, 0, 50, 8, 0)
    assert np.array_equal(got, _dense(engine, ds, 0))


def _all_rows(aji, n, r0, r1):
    """Rows [r0, r1) of the ALL-mode dense fill from the JAC-order AJI vector
    (pair (a, b), a < b, at n*a + b - (a+2)(a+1)/2), mirror half included."""
    out = np.zeros((r1 - r0, n))
    for r in range(r0, r1):
        b = np.arange(r + 1, n)
        out[r - r0, b] = aji[n * r + b - (r + 2) * (r + 1) // 2]
        a = np.arange(0, r)
        out[r - r0, a] = aji[n * a + r - (a + 2) * (a + 1) // 2]
    return out


@pytest.mark.parametrize("mode", ["all", "qt"])
def test_stream_matrix_column_windows(diag_engine, monkeypatch, mode):
    """Rows wider than one k_rows_pl chunk (column windows with a run table
    per window) in full-row mode: == the dense fill of pfaai_compute, and ==
    per-row chunks over one table (PFAAI_PL_WINDOWS=0, diagnostics build)."""
    engine = diag_engine
    if mode == "all":
        g = syn.generate(21000, 3, clade_size=50, n_random=1)
        ds = ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"], g["genome_set"]
                                    ).with_genome_major(g["G_off"], g["G_tet"])
        r0, r1 = 6990, 7130
    else:
        ds = qt_syn(dict(n_tgt=12000, n_qry=40, n_prot=4, clade_size=30, n_random=1), genome_major=True)
        r0, r1 = 0, 40
    engine.load(**ds.problem())
    for flags in COMPAT:
        monkeypatch.delenv("PFAAI_PL_WINDOWS", raising=False)
        if mode == "all":
            M = _all_rows(engine.compute(flags)[0], ds.n_genomes, r0, r1)
        else:
            M = _dense(engine, ds, flags)[r0:r1]
        got, nt, _ = _streamed(engine, r0, r1, 64, flags)
        assert engine.stats()["column_windows"]
        assert np.array_equal(got, M, equal_nan=True)
        monkeypatch.setenv("PFAAI_PL_WINDOWS", "0")
        got2, _, _ = _streamed(engine, r0, r1, 64, flags)
        assert np.array_equal(got2, M, equal_nan=True)
    monkeypatch.delenv("PFAAI_PL_WINDOWS", raising=False)
