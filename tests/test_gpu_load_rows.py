"""The run-end sort (pfaai_sort.hpp SrcFEnds: G_pos and G_end of the all-vs-all
walks from one two-pass sort of F) and the per-rank load
(pfaai_load_rows).

  * a rank that loads only its row block builds the walk data of those rows
    and its rows equal the same rows of a full load, bit for bit, through the
    benchmarked walk (pfaai_run_walk "gpos"), for every block of a 3-way and
    an 8-way split, in both input orientations that build G_pos (F and G,
    G only);
  * rows outside a G-only rank's block still run (run table + splitters);
    rows outside a both-given rank's block are refused -- its load checked
    only its own genomes' G lists against F;
  * the check of a both-given rank load refuses a G list of its block that
    differs from F's transpose, and accepts a block that does not contain it;
  * runs longer than a tile (a tetramer held by every genome), tiny problems
    (F shorter than one tile) and an empty block.
"""
import numpy as np
import pytest
import torch

from parfastaai_amd import _capi, syn
from parfastaai_amd.datastruct import ParFAAIData
from parfastaai_amd.shard import split_rows

pytestmark = pytest.mark.gpu


def _problem(n, P, **kw):
    g = syn.generate(n, P, **kw)
    return ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"]).with_genome_major(
        g["G_off"], g["G_tet"]).problem()


def _strip(pb, drop):
    return {k: v for k, v in pb.items() if k not in drop}


def _run(engine, rb, re, npairs):
    aji = torch.full((npairs,), -1.0, dtype=torch.float64, device="cuda:0")
    S = torch.full((npairs,), -1.0, dtype=torch.float64, device="cuda:0")
    N = torch.full((npairs,), -1, dtype=torch.int32, device="cuda:0")
    engine.run(rb, re, _capi.FLAG_EMIT_JAC, aji.data_ptr(), S.data_ptr(), N.data_ptr(),
               stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return aji.cpu().numpy(), S.cpu().numpy(), N.cpu().numpy()


@pytest.mark.parametrize("n,P,kw", [
    (1200, 30, dict(clade_size=12)),
    (37, 5, dict(clade_size=4)),              # |F| below one 4096-entry tile
])
@pytest.mark.parametrize("orient", ["both", "g_only"])
def test_rank_blocks_equal_full_load(engine, n, P, kw, orient):
    pb = _problem(n, P, **kw)
    if orient == "g_only":
        pb = _strip(pb, ("Lp", "F_prot", "F_genome"))
    engine.load(**pb)
    _, npairs = engine.shape()
    full = _run(engine, 0, n, npairs)
    assert engine.stats()["walk"] == "gpos"
    for parts in (3, 8):
        for rb, re in split_rows(n, parts):
            engine.load(rows=(rb, re), **pb)
            if re == rb:
                continue
            got = _run(engine, rb, re, npairs)
            assert engine.stats()["walk"] == "gpos", (rb, re)
            f, c = engine.row_span(rb, re)
            for x, y in zip(got, full):
                assert np.array_equal(x[f:f + c], y[f:f + c]), (parts, rb, re)
    # outside the block: G only runs them through the run table, both given refuses them
    # (the run-end sort takes two-pass keys; one-pass keys build and check every genome's walk data)
    two_pass = (n * P).bit_length() > 11
    rb, re = split_rows(n, 3)[1]
    engine.load(rows=(rb, re), **pb)
    if orient == "g_only" or not two_pass:
        got = _run(engine, 0, rb, npairs)
        assert engine.stats()["walk"] == ("splitters" if two_pass else "gpos")
        f, c = engine.row_span(0, rb)
        for x, y in zip(got, full):
            assert np.array_equal(x[f:f + c], y[f:f + c])
    else:
        with pytest.raises(_capi.PfaaiError):
            _run(engine, 0, rb, npairs)


def test_empty_block(engine):
    pb = _problem(300, 12, clade_size=6)
    engine.load(rows=(100, 100), **_strip(pb, ("Lp", "F_prot", "F_genome")))
    _, npairs = engine.shape()
    aji, _, _ = _run(engine, 0, 300, npairs)
    engine.load(**pb)
    ref, _, _ = _run(engine, 0, 300, npairs)
    assert np.array_equal(aji, ref)


def test_runs_longer_than_a_tile(engine):
    """A tetramer held by every genome in every protein: runs of n entries
    span several 4096-entry tiles of the run-end sort (their ends come from
    the next tiles' first tails)."""
    n, P = 9000, 3
    g = syn.generate(n, P, clade_size=30)
    # add a tetramer SYN uses nowhere to every (genome, protein) list
    G_off, G_tet = g["G_off"], g["G_tet"]
    t_add = int(np.setdiff1d(np.arange(160000), G_tet)[-1])
    lens = np.diff(G_off) + 1
    off = np.zeros(len(lens) + 1, np.int64)
    off[1:] = np.cumsum(lens)
    tet = np.empty(off[-1], np.int32)
    for k in range(len(lens)):
        tet[off[k]:off[k + 1]] = np.sort(np.r_[G_tet[G_off[k]:G_off[k + 1]], t_add])
    T = g["T"] + 1
    pbg = dict(mode=_capi.MODE_ALL, n_ids=n, n_prot=P, T=T, G_off=off, G_tet=tet)
    engine.load(**pbg)  # G only: F built on the device, then the run-end sort
    _, npairs = engine.shape()
    got = _run(engine, 0, n, npairs)
    assert engine.stats()["walk"] == "gpos"
    # the same problem through the run table (an empty walk block: no G_pos rows)
    engine.load(rows=(0, 0), **pbg)
    ref = _run(engine, 0, n, npairs)
    assert engine.stats()["walk"] == "splitters"
    for x, y in zip(got, ref):
        assert np.array_equal(x, y)
    assert (got[2] >= 1).all()  # every pair shares the added tetramer


def test_rank_check_refuses_a_bad_list_of_its_block(engine):
    n, P = 800, 20
    pb = _problem(n, P, clade_size=8)
    G_off, G_tet = pb["G_off"].copy(), pb["G_tet"].copy()
    gbad = 500
    k = gbad * P + 3
    lst = G_tet[G_off[k]:G_off[k + 1]]
    x = next(t for t in range(159999, 0, -1) if t not in set(lst.tolist()))
    lst[len(lst) // 2] = x
    G_tet[G_off[k]:G_off[k + 1]] = np.sort(lst)
    bad = dict(pb, G_tet=G_tet)
    with pytest.raises(_capi.PfaaiError):
        engine.load(**bad)
    with pytest.raises(_capi.PfaaiError):
        engine.load(rows=(400, 600), **bad)
    engine.load(rows=(0, 400), **bad)  # the block without genome 500: its lists are F's
    _, npairs = engine.shape()
    got = _run(engine, 0, 400, npairs)
    engine.load(**pb)
    ref = _run(engine, 0, 400, npairs)
    f, c = engine.row_span(0, 400)
    for x, y in zip(got, ref):
        assert np.array_equal(x[f:f + c], y[f:f + c])


@pytest.mark.parametrize("n,world,group", [(700, 3, 32), (3000, 8, 32), (2100, 5, 7)])
def test_cyclic_row_lists_assemble_to_the_whole_run(engine, n, world, group):
    """Round 6: a rank's block-cyclic share -- groups of
    rows dealt in snake order (shard.cyclic_rows) -- runs as ONE launch over
    its row list (pfaai_set_row_order), each rank into its own full-size
    array at the reference's JAC indices; the ranks' rows assemble to the
    single run bit for bit, S and N included, through the benchmarked walk
    (G_pos, the narrow 512-thread rows split off by genome)."""
    from parfastaai_amd.shard import cyclic_rows, row_segments
    pb = _problem(n, 30, clade_size=10)
    engine.load(**pb)
    rows, npairs = engine.shape()
    ref = [torch.full((npairs,), -1.0, dtype=dt, device="cuda:0") for dt in (torch.float64, torch.float64, torch.int32)]
    st = torch.cuda.current_stream().cuda_stream
    engine.run(0, rows, _capi.FLAG_EMIT_JAC, *(x.data_ptr() for x in ref), stream=st)
    got = [torch.full_like(x, -2) for x in ref]
    lists = cyclic_rows(rows, world, group)
    assert sorted(r for rl in lists for r in rl) == list(range(rows))
    # the sorted-E counts of a list's middle row (pfaai_debug_row_counts) follow the list too
    mid = {rl[len(rl) // 2]: engine.debug_row_counts(rl[len(rl) // 2], 30, n) for rl in lists}
    base = lambda a: n * a - a * (a + 1) // 2
    for rl in lists:
        engine.set_row_order(rl)
        assert np.array_equal(engine.debug_row_counts(len(rl) // 2, 30, n), mid[rl[len(rl) // 2]])
        part = [torch.full_like(x, -3) for x in ref]
        engine.run(0, len(rl), _capi.FLAG_EMIT_JAC, *(x.data_ptr() for x in part), stream=st)
        torch.cuda.synchronize()
        assert engine.stats()["walk"] == "gpos"
        for lo, hi in row_segments(rl):
            for g, p in zip(got, part):
                g[base(lo):base(hi)] = p[base(lo):base(hi)]
        with pytest.raises(_capi.PfaaiError):  # rows past the list
            engine.run(0, len(rl) + 1, 0, part[0].data_ptr(), stream=st)
        with pytest.raises(_capi.PfaaiError):  # span APIs refuse a row order
            engine.compute(0)
    engine.set_row_order(None)
    for g, r in zip(got, ref):
        assert torch.equal(g, r)
    with pytest.raises(_capi.PfaaiError):
        engine.set_row_order([5, 3])  # not ascending
    a2, _, _ = engine.compute(0)  # the id order is back
    assert np.array_equal(a2, ref[0].cpu().numpy())
