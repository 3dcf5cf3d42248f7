"""Output-tile streaming (pfaai_stream), the
run-table reuse flag (PFAAI_FLAG_KEEP_RUNS) and F past 2^30 entries (where a
32-bit byte offset into F wraps), all through the C ABI on the GPU, bit-exact
against pfaai_compute and the CPU oracle."""
import numpy as np
import pytest

import oracle as O
from helpers import qt_syn
from parfastaai_amd import _capi, syn
from parfastaai_amd.datastruct import ParFAAIData, ParFAAIQSubData

pytestmark = pytest.mark.gpu


def _all_problem(n, p, **kw):
    g = syn.generate(n, p, **kw)
    ds = ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"])
    return ds.with_genome_major(g["G_off"], g["G_tet"]).problem()


def _collect(engine, rb, re, tile, flags):
    """-> (aji, S, N) over the rows' JAC span, tiles checked to arrive in order."""
    f0, cnt = engine.row_span(rb, re)
    aji = np.full(cnt, np.nan)
    S = np.full(cnt, np.nan)
    N = np.full(cnt, -1, np.int32)
    seen = []

    def sink(r0, r1, first, a, s, n):
        assert not seen or seen[-1][1] == r0, "tiles out of order"
        assert len(a) <= max(tile, engine.row_span(r0, r0 + 1)[1])
        seen.append((r0, r1))
        aji[first - f0: first - f0 + len(a)] = a
        if s is not None:
            S[first - f0: first - f0 + len(a)] = s
            N[first - f0: first - f0 + len(a)] = n
        return 0

    ne = engine.stream(rb, re, tile, flags, sink)
    assert seen[0][0] == rb and seen[-1][1] == re
    return aji, S, N, ne, len(seen)


@pytest.mark.parametrize("compat", [False, True], ids=["default", "ref-compat"])
def test_stream_all_equals_compute(engine, compat):
    pb = _all_problem(300, 30, clade_size=10)
    engine.load(**pb)
    flags = _capi.FLAG_REF_COMPAT if compat else 0
    aji, S, N = engine.compute(flags)
    # tiles of <= 997 pairs: ~45 tiles, the last rows several per tile
    a2, S2, N2, ne, nt = _collect(engine, 0, 300, 997, flags | _capi.FLAG_EMIT_JAC)
    assert nt > 20
    assert np.array_equal(a2, aji) and np.array_equal(S2, S) and np.array_equal(N2, N)
    assert ne == O.Problem(pb, compat=compat).count_e()
    # AJI only (no S/N), a row sub-range
    f0, cnt = engine.row_span(40, 211)
    a3, S3, _, _, _ = _collect(engine, 40, 211, 5000, flags)
    assert np.array_equal(a3, aji[f0:f0 + cnt]) and np.isnan(S3).all()


def test_stream_qt_equals_compute(engine):
    ds = qt_syn(dict(n_tgt=60, n_qry=25, n_prot=20, clade_size=6), genome_major=True)
    engine.load(**ds.problem())
    aji, S, N = engine.compute(0)
    a2, S2, N2, _, nt = _collect(engine, 0, 25, 130, _capi.FLAG_EMIT_JAC)
    assert nt == 13  # two 60-column rows per tile
    assert np.array_equal(a2, aji) and np.array_equal(S2, S) and np.array_equal(N2, N)


def test_stream_rejects_qsub_and_sink_stop(engine):
    pb = _all_problem(80, 10, clade_size=8)
    engine.load(**pb)
    calls = []
    with pytest.raises(_capi.PfaaiError) as ei:
        engine.stream(0, 80, 100, 0, lambda *a: calls.append(a[0]) or len(calls) == 2)
    assert ei.value.code == 7 and len(calls) == 2
    g = syn.generate(30, 5, clade_size=5)
    q = ParFAAIQSubData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"], g["genome_set"],
                                   [g["genome_set"][i] for i in (3, 9, 17)])
    engine.load(**q.problem())
    with pytest.raises(_capi.PfaaiError):
        engine.stream(0, 3, 100, 0, lambda *a: 0)


def test_keep_runs_matches_single_run(engine):
    """Rows computed in three pfaai_run calls, the later two reusing the run
    table, equal one run over all rows."""
    import torch

    pb = _all_problem(500, 40, clade_size=12)
    engine.load(**pb)
    aji, _, _ = engine.compute(0)
    _, npairs = engine.shape()
    out = torch.full((npairs,), -1.0, dtype=torch.float64, device="cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    for i, (rb, re) in enumerate([(0, 90), (90, 301), (301, 500)]):
        engine.run(rb, re, _capi.FLAG_KEEP_RUNS if i else 0, out.data_ptr(), stream=st)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), aji)
    n_runs, ms_build, _ = engine.timing(reset=True)
    assert n_runs >= 3


def test_keep_runs_across_table_kinds(engine):
    """All-vs-all rows read the u32 run-end table (k_blk_end), full rows the
    16-B run table (k_blk): PFAAI_FLAG_KEEP_RUNS must rebuild whenever the
    next run needs the other kind, in either order."""
    import torch

    n = 260
    pb = _all_problem(n, 30, clade_size=9)
    engine.load(**pb)
    aji, _, _ = engine.compute(0)
    dense = np.zeros((n, n))
    iu = np.triu_indices(n, 1)
    dense[iu] = aji
    dense = dense + dense.T
    _, npairs = engine.shape()
    tri = torch.full((npairs,), -1.0, dtype=torch.float64, device="cuda:0")
    full = torch.zeros((n * n,), dtype=torch.float64, device="cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    K, FR = _capi.FLAG_KEEP_RUNS, _capi.FLAG_FULL_ROWS
    engine.run(0, 100, 0, tri.data_ptr(), stream=st)            # builds the end table
    engine.run(0, 130, K | FR, full.data_ptr(), stream=st)      # needs the 16-B table
    engine.run(100, 200, K, tri.data_ptr(), stream=st)          # back to ends
    engine.run(130, n, K | FR, full.data_ptr(), stream=st)      # and 16-B again
    engine.run(200, n, K, tri.data_ptr(), stream=st)
    torch.cuda.synchronize()
    assert np.array_equal(tri.cpu().numpy(), aji)
    assert np.array_equal(full.cpu().numpy().reshape(n, n), dense)


@pytest.mark.timeout(600)
def test_f_beyond_2_30_entries(engine):
    """|F| > 2^30: member ids past byte offset 2^32 of F (SYN N = 38 000,
    |F| ~ 1.09e9); sampled rows streamed and checked against the oracle's
    dense restatement, |E| of those rows included."""
    n = 38000
    g = syn.generate(n, 100)
    nf = len(g["F_genome"])
    assert nf > (1 << 30), nf
    pb = dict(mode=_capi.MODE_ALL, n_ids=n, n_prot=100, Lp=g["Lp"], F_prot=g["F_prot"],
              F_genome=g["F_genome"], T=g["T"], G_off=g["G_off"], G_tet=g["G_tet"])
    engine.load(**pb)
    del g
    pr = O.Problem(pb)
    for lo, hi in [(0, 2), (20011, 20013), (n - 40, n - 37)]:
        f0, _ = engine.row_span(lo, hi)
        aji, S, N, ne, _ = _collect(engine, lo, hi, 1 << 20, _capi.FLAG_EMIT_JAC)
        So, No, neo = pr.dense_rows(lo, hi)
        assert ne == neo
        for a in range(lo, hi):
            b = np.arange(a + 1, n)
            k = n * a + b - (a + 2) * (a + 1) // 2 - f0
            assert np.array_equal(S[k], So[a - lo, b]) and np.array_equal(N[k], No[a - lo, b])
            assert np.array_equal(aji[k], np.where(N[k] > 0, S[k] / np.maximum(N[k], 1), 0.0))


@pytest.mark.parametrize("mode", ["all", "qsub", "qt"])
def test_column_windows_equal_row_chunks(diag_engine, monkeypatch, mode):
    """Rows wider than one k_rows_pl chunk: absolute column windows with a run
    table per window (default) == per-row chunks over one table
    (PFAAI_PL_WINDOWS=0, read by the diagnostics build only; itself pinned
    against the oracle in test_gpu_edges.py), S / N / AJI bit-exact,
    ref-compat included."""
    engine = diag_engine
    if mode == "all":
        pb = _all_problem(21000, 3, clade_size=50, n_random=1)
    elif mode == "qsub":
        g = syn.generate(11000, 4, clade_size=40, n_random=1)
        pick = list(range(5, 11000, 197))
        ds = ParFAAIQSubData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"], g["genome_set"],
                                        [g["genome_set"][i] for i in pick])
        pb = ds.with_genome_major(g["G_off"], g["G_tet"]).problem()
    else:
        pb = qt_syn(dict(n_tgt=12000, n_qry=40, n_prot=4, clade_size=30, n_random=1), genome_major=True).problem()
    engine.load(**pb)
    for flags in (0, _capi.FLAG_REF_COMPAT):
        monkeypatch.delenv("PFAAI_PL_WINDOWS", raising=False)
        a1, S1, N1 = engine.compute(flags)
        ne1 = engine.stats()["n_events"]
        monkeypatch.setenv("PFAAI_PL_WINDOWS", "0")
        a2, S2, N2 = engine.compute(flags)
        ne2 = engine.stats()["n_events"]
        assert ne1 == ne2
        assert np.array_equal(N1, N2) and np.array_equal(S1, S2) and np.array_equal(a1, a2)
        monkeypatch.delenv("PFAAI_PL_WINDOWS", raising=False)
        if mode != "qsub":  # streamed row tiles reuse the window tables (PFAAI_FLAG_KEEP_RUNS)
            rows = engine.shape()[0]
            a3, S3, N3, ne3, nt = _collect(engine, 0, rows, 3_000_000 if mode == "all" else 100_000,
                                           flags | _capi.FLAG_EMIT_JAC)
            assert nt > 1 and ne3 == ne1
            assert np.array_equal(a3, a1) and np.array_equal(S3, S1) and np.array_equal(N3, N1)


@pytest.mark.parametrize("case", ["all", "qt", "qt_edge"])
def test_window_spans_equal_window_launches(diag_engine, monkeypatch, case):
    """Round 6: column windows whose sub-runs hold only the row's partners
    (all-vs-all windows past the row's first column, every query-vs-target
    window) run as one WK 4 launch over (row, window) with the member codes
    and no window test, the all-vs-all diagonal windows as one WK 1 launch
    (pfaai_run_walk "spans") == round 5's launch per window over the window
    tables (PFAAI_PL_NOWK4=1, diagnostics build) == the oracle on sampled
    rows, S / N / AJI / |E| bit-exact, ref-compat included.  qt_edge: 20 480
    targets = exactly two windows, so the query ids (>= n_tgt) lie past the
    last window -- the tables stop at n_tgt, and no id indexes past them."""
    engine = diag_engine
    if case == "all":
        pb = _all_problem(21000, 3, clade_size=50, n_random=1)
        rows = [0, 10238, 10239, 10240, 15000, 20998]  # 10239: its columns start window 1
    else:
        n_tgt = 12000 if case == "qt" else 20480
        pb = qt_syn(dict(n_tgt=n_tgt, n_qry=40, n_prot=4, clade_size=30, n_random=1), genome_major=True).problem()
        rows = [n_tgt, n_tgt + 17, n_tgt + 39]
    engine.load(**pb)
    pr = O.Problem(pb)
    res = {}
    for flags in (0, _capi.FLAG_REF_COMPAT):
        monkeypatch.delenv("PFAAI_PL_NOWK4", raising=False)
        a1, S1, N1 = res[flags] = engine.compute(flags)
        st = engine.stats()
        assert st["walk"] == "spans", st
        monkeypatch.setenv("PFAAI_PL_NOWK4", "1")
        a2, S2, N2 = engine.compute(flags)
        assert engine.stats()["walk"] == "splitters"
        assert engine.stats()["n_events"] == st["n_events"]
        assert np.array_equal(N1, N2) and np.array_equal(S1, S2) and np.array_equal(a1, a2)
        monkeypatch.delenv("PFAAI_PL_NOWK4", raising=False)
    n = pb["n_ids"]
    _, S2, N2 = res[0]
    for a in rows:
        So, No, _ = pr.dense_rows(a, a + 1)
        if case == "all":
            b = np.arange(a + 1, n)
            k = n * a + b - (a + 2) * (a + 1) // 2
        else:
            n_tgt = pb["n_tgt"]
            b = np.arange(n_tgt)
            k = (a - n_tgt) * n_tgt + b
        assert np.array_equal(N2[k], No[0, b]) and np.array_equal(S2[k], So[0, b]), a


def test_compute_rows_two_contexts_fill_one_array(engine):
    """pfaai_compute_rows: two contexts (here both on device 0) each write
    their row block's JAC span of one host array; == pfaai_compute."""
    from parfastaai_amd.shard import split_rows

    pb = _all_problem(700, 30, clade_size=10)
    engine.load(**pb)
    ref_a, ref_S, ref_N = engine.compute(0)
    e2 = _capi.Engine(0)
    try:
        e2.load(**pb)
        n = len(ref_a)
        a = np.full(n, np.nan)
        S = np.full(n, np.nan)
        N = np.full(n, -1, np.int32)
        (r0, r1), (r2, r3) = split_rows(700, 2)
        for e, (rb, re) in ((engine, (r0, r1)), (e2, (r2, r3))):
            rc = e.lib.pfaai_compute_rows(e.ctx, rb, re, 0, a.ctypes.data, S.ctypes.data, N.ctypes.data)
            e._check(rc, "pfaai_compute_rows")
        assert np.array_equal(a, ref_a) and np.array_equal(S, ref_S) and np.array_equal(N, ref_N)
    finally:
        e2.close()


@pytest.mark.parametrize("order", ["sorted", "shuffled"])
def test_compute_rows_qsub_blocks_fill_one_array(engine, order):
    """Round 6: -q row blocks through pfaai_compute_rows --
    each block's cross cells by span, its query-query cells merged into the
    triangle cell by cell -- fill one array equal to pfaai_compute, for a
    query list in DB order and one shuffled (a pair's cell
    then lies in another block's rows), ref-compat included for the sorted
    list (with a shuffled one the reference's unswapped triangle index makes
    pairs collide on one cell, ds_impl.hpp:257-262: undefined there, single
    device included); three contexts on device 0 as in the CLI's --devices
    0,0,0."""
    g = syn.generate(900, 20, clade_size=10)
    rng = np.random.default_rng(11)
    pick = sorted(rng.choice(900, 61, replace=False).tolist())
    if order == "shuffled":
        rng.shuffle(pick)
    ds = ParFAAIQSubData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"], g["genome_set"],
                                    [g["genome_set"][i] for i in pick])
    pb = ds.with_genome_major(g["G_off"], g["G_tet"]).problem()
    engine.load(**pb)
    others = [_capi.Engine(0), _capi.Engine(0)]
    try:
        for e in others:
            e.load(**pb)
        for flags in (0, _capi.FLAG_REF_COMPAT) if order == "sorted" else (0,):
            ref_a, ref_S, ref_N = engine.compute(flags)
            n = len(ref_a)
            a = np.full(n, np.nan)
            S = np.full(n, np.nan)
            N = np.full(n, -7, np.int32)
            cuts = [0, 17, 40, 61]
            for e, rb, re in zip([engine] + others, cuts[:-1], cuts[1:]):
                e._check(e.lib.pfaai_compute_rows(e.ctx, rb, re, flags, a.ctypes.data, S.ctypes.data,
                                                  N.ctypes.data), "pfaai_compute_rows")
            assert np.array_equal(N, ref_N) and np.array_equal(S, ref_S) and np.array_equal(a, ref_a)
    finally:
        for e in others:
            e.close()


@pytest.mark.timeout(600)
def test_stream_tiles_switch_window_and_end_table(engine):
    """All-vs-all, 11 000 genomes (G_pos built): rows wider than one 10 240-
    column chunk run by column windows over window tables, the later rows in
    one chunk over the u32 run-end table -- each launch takes its own width,
    so streamed tiles switch table kinds within one load (PFAAI_FLAG_KEEP_RUNS
    must not hand a tile the other kind).  Equal to the single-launch run,
    which covers every row by windows, and to the oracle on sampled rows."""
    n, P = 11000, 12
    pb = _all_problem(n, P)
    engine.load(**pb)
    aji, S, N = engine.compute(0)
    a2, S2, N2, _, nt = _collect(engine, 0, n, 1 << 24, _capi.FLAG_EMIT_JAC)
    assert nt >= 3
    assert np.array_equal(a2, aji) and np.array_equal(S2, S) and np.array_equal(N2, N)
    pr = O.Problem(pb)
    for a in (0, 700, 900, 5000, n - 2):  # 700: wider than a chunk; 900: not
        So, No, _ = pr.dense_rows(a, a + 1)
        b = np.arange(a + 1, n)
        k = n * a + b - (a + 2) * (a + 1) // 2
        assert np.array_equal(N[k], No[0, b]) and np.array_equal(S[k], So[0, b]), a


@pytest.mark.parametrize("var", ["PFAAI_PL_T24", "PFAAI_PL_REV", "PFAAI_SORT_DIRECT"])
def test_diagnostic_variants_equal_release_form(diag_engine, monkeypatch, var):
    """The round-6 A/B variants of the diagnostics build compute what the
    release form computes, S / N / AJI / |E| bit for bit, on an all-vs-all
    windowed load and a query-vs-target one: 24-member span tasks
    (PFAAI_PL_T24), the further member rounds from the last lane pair down
    (PFAAI_PL_REV), the load sort's direct stores without the LDS reorder
    (PFAAI_SORT_DIRECT: the load is repeated under it).  Their timings are in
    profiles/r06/ab_t24.txt, ab_rev.txt and ab_sort_direct.txt."""
    engine = diag_engine
    if var == "PFAAI_SORT_DIRECT":  # the run-end sort: all-vs-all, both orientations, <= 20 480 genomes
        pbs = (_all_problem(3000, 20, clade_size=25, n_random=1),)
    else:
        pbs = (_all_problem(21000, 3, clade_size=50, n_random=1),
               qt_syn(dict(n_tgt=12000, n_qry=40, n_prot=4, clade_size=30, n_random=1), genome_major=True).problem())
    for pb in pbs:
        monkeypatch.delenv(var, raising=False)
        engine.load(**pb)
        a1, S1, N1 = engine.compute(0)
        e1 = engine.stats()["n_events"]
        monkeypatch.setenv(var, "1")
        if var == "PFAAI_SORT_DIRECT":
            engine.load(**pb)
        a2, S2, N2 = engine.compute(0)
        if var == "PFAAI_SORT_DIRECT":
            assert engine.stats()["walk"] == "gpos", engine.stats()
        assert engine.stats()["n_events"] == e1
        assert np.array_equal(N1, N2) and np.array_equal(S1, S2) and np.array_equal(a1, a2)
        monkeypatch.delenv(var, raising=False)
