"""Multi-rank path on CPU (gloo, world_size 2): row-block split + gather.

Each rank computes its own row block (here with the CPU oracle as the
stand-in for the device, since this runs without a GPU -- the device leg of
the same split is tests/test_gpu_parity.py::test_hip_row_sharding_matches_full)
and rank 0 gathers with parfastaai_amd.shard.gather_rows; the gathered vector
must equal the single-process result exactly.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from parfastaai_amd.shard import FIXED_COST_FRACTION, NARROW_COLS, NARROW_COST_FACTOR, ROUND_TAIL, row_costs, split_rows

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, result_q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch
    import torch.distributed as dist

    import oracle as O
    from parfastaai_amd import syn
    from parfastaai_amd.datastruct import ParFAAIData
    from parfastaai_amd.shard import gather_rows, split_rows

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = syn.generate(n, 12, clade_size=5)  # identical on every rank
    ds = ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"])
    pr = O.Problem(ds.problem())
    blocks = split_rows(n, world)
    rb, re = blocks[rank]
    # this rank's rows: oracle dense rows -> JAC order (row a: b = a+1..n-1)
    S, N, _ = pr.dense_rows(rb, re)
    aji = [S[a - rb, a + 1:] / N[a - rb, a + 1:] for a in range(rb, re)]
    local = np.concatenate(aji) if aji else np.zeros(0)
    counts = [sum(n - 1 - a for a in range(b0, b1)) for b0, b1 in blocks]
    t = torch.zeros(max(counts), dtype=torch.float64)
    t[: len(local)] = torch.from_numpy(local)
    full = gather_rows(t, counts)
    if rank == 0:
        ref = pr.ref_run()["AJI"]
        result_q.put(bool(np.array_equal(full.numpy(), ref)))
    dist.destroy_process_group()


def _cyclic_worker(rank, world, port, n, steps, slots, result_q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch
    import torch.distributed as dist

    import oracle as O
    from parfastaai_amd import syn
    from parfastaai_amd.datastruct import ParFAAIData
    from parfastaai_amd.shard import SegmentGather, cyclic_rows, jac_segments

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = syn.generate(n, 12, clade_size=5)  # identical on every rank
    pr = O.Problem(ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"]).problem())
    lists = cyclic_rows(n, world, 7)
    segs = [jac_segments(n, rl) for rl in lists]
    npairs = n * (n - 1) // 2
    sg = SegmentGather(segs, npairs, slots=slots)
    S, N, _ = pr.dense_rows(0, n)  # (the device's stand-in: this rank writes only its rows)
    ok = True
    for i in range(steps):
        sg.begin(i)
        sg.buf.fill_(-1.0 - i)  # stale values must be overwritten by the rows' owners
        for a in lists[rank]:
            f = n * a - a * (a + 1) // 2
            sg.buf[f:f + n - 1 - a] = torch.from_numpy(S[a, a + 1:] / N[a, a + 1:] + i)
        sg.issue()
        if slots == 1:
            sg.wait()
    sg.wait()
    if rank == 0:
        ref = pr.ref_run()["AJI"]
        for k in range(min(slots, steps)):
            i = steps - 1 - k
            ok = ok and bool(np.array_equal(sg.result(slot=i % slots).numpy(), ref + i))
        result_q.put(ok)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,steps,slots", [(2, 1, 1), (3, 4, 2)])
def test_gloo_segment_gather_of_cyclic_rows(world, steps, slots):
    """shard.SegmentGather (the gather of block-cyclic row lists): every rank
    writes only its rows into its full-size array, the others' JAC segments
    arrive in rank 0's array by grouped send / recv, double-buffered over
    steps; rank 0's array equals the single-process AJI vector, each buffer
    set's own step."""
    port = _free_port()
    q = mp.get_context("spawn").SimpleQueue()
    ps = [mp.get_context("spawn").Process(target=_cyclic_worker, args=(r, world, port, 40, steps, slots, q))
          for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=300)
        assert p.exitcode == 0
    assert q.get() is True


@pytest.mark.parametrize("n,world,group", [(10000, 8, 32), (1000, 3, 32), (37, 5, 4), (5, 8, 32)])
def test_cyclic_rows_partition_and_balance(n, world, group):
    """shard.cyclic_rows: every row in exactly one rank's ascending list,
    groups of `group` consecutive rows, dealt in snake order; at 10k x 8 the
    ranks' row costs (row_costs) lie within 2 % of each other."""
    from parfastaai_amd.shard import cyclic_rows, row_segments
    lists = cyclic_rows(n, world, group)
    assert len(lists) == world
    assert sorted(r for rl in lists for r in rl) == list(range(n))
    for rl in lists:
        assert rl == sorted(rl)
        for lo, hi in row_segments(rl):
            assert lo % group == 0 and (hi - lo == group or hi == n or hi % group == 0)
    if n == 10000:
        c = row_costs(n)
        cost = [sum(c[r] for r in rl) for rl in lists]
        assert max(cost) / min(cost) < 1.02, cost


def test_split_rows_balanced():
    for n, w in [(10000, 8), (2000, 2), (7, 4), (3, 8)]:
        blocks = split_rows(n, w)
        assert blocks[0][0] == 0 and blocks[-1][1] == n
        assert all(blocks[i][1] == blocks[i + 1][0] for i in range(w - 1))
        c = row_costs(n)
        cost = [c[b0:b1].sum() for b0, b1 in blocks]
        if n >= 100 * w:
            assert max(cost) - min(cost) <= 2 * (FIXED_COST_FRACTION * n + n)  # within a row or two
    # the model: fixed + width, narrow rows (<= NARROW_COLS columns) scaled
    c = row_costs(5000)
    assert c[0] == FIXED_COST_FRACTION * 5000 + 4999
    assert c[-1] == NARROW_COST_FACTOR * FIXED_COST_FRACTION * 5000
    # cus: a cut a few rows into another round of 2 * cus workgroups moves back
    plain = split_rows(10000, 8)
    rounded = split_rows(10000, 8, cus=256)
    assert rounded[0][0] == 0 and rounded[-1][1] == 10000
    assert all(rounded[i][1] == rounded[i + 1][0] for i in range(7))
    for (b0, b1), (p0, p1) in zip(rounded, plain):
        m = b1 - b0
        if 10000 - b1 > NARROW_COLS + 1 and m > 512:
            assert not 0 < m % 512 <= ROUND_TAIL * 512, (b0, b1)
    assert rounded != plain  # (the 10k x 8 plain split leaves block 3 66 rows into a third round)
    assert split_rows(10, 3, cus=256) == split_rows(10, 3)
    # pure pair balance with fixed_cols = 0
    blocks = split_rows(10000, 8, fixed_cols=0)
    pairs = [sum(10000 - 1 - a for a in range(b0, b1)) for b0, b1 in blocks]
    assert max(pairs) - min(pairs) <= 10000
    assert split_rows(10, 3, all_vs_all=False) == [(0, 3), (3, 6), (6, 10)]


def test_gloo_world2_gather_equals_single():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, 90, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=10) is True


def _pipe_worker(rank, world, port, n, chunks, slots, steps, result_q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    from parfastaai_amd.shard import PipelinedGather, split_range, split_rows

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    base = lambda a: n * a - a * (a + 1) // 2  # JAC index of (a, a+1), ds_impl.hpp:83-86  # noqa: E731
    blocks = split_rows(n, world)
    sub = [split_range(b0, b1, chunks, n) for b0, b1 in blocks]
    counts = [[base(c1) - base(c0) for c0, c1 in s] for s in sub]
    pg = PipelinedGather(counts, dst=0, slots=slots)
    ok = True
    for step in range(steps):  # step i's "result": JAC index + i, buffer set i % slots
        pg.begin(step)
        for j, (c0, c1) in enumerate(sub[rank]):  # "compute" chunk j: its JAC indices
            pg.bufs[j][: counts[rank][j]] = torch.arange(base(c0), base(c1), dtype=torch.float64) + step
            pg.issue(j)
        if step >= slots - 1 and step % 2:  # drain now and then, as bench.py does only at the end
            pg.wait()
            full = pg.result()
            if rank == 0:
                ok = ok and bool(torch.equal(full, torch.arange(n * (n - 1) // 2, dtype=torch.float64) + step))
    pg.wait()
    for k in range(slots):  # the last step that used each buffer set
        last = max(i for i in range(steps) if i % slots == k)
        full = pg.result(k)
        if rank == 0:
            ok = ok and bool(torch.equal(full, torch.arange(n * (n - 1) // 2, dtype=torch.float64) + last))
    if rank == 0:
        result_q.put(ok)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,chunks,slots,steps", [(2, 3, 1, 1), (3, 1, 1, 1), (2, 1, 2, 5), (3, 2, 2, 4)])
def test_gloo_pipelined_gather_covers_jac_order(world, chunks, slots, steps):
    """bench.py's N > 1 steps: rank blocks (optionally cut into pipeline
    chunks) gathered asynchronously as soon as they are computed, double-
    buffered across steps (slots = 2: step i + 1 computes while step i's
    gather is in flight); rank 0's concatenation is each step's full
    JAC-ordered vector."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipe_worker, args=(r, world, port, 157, chunks, slots, steps, q))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=10) is True


def test_split_range_chunks():
    from parfastaai_amd.shard import split_range

    n = 10000
    for b0, b1 in split_rows(n, 8):
        sub = split_range(b0, b1, 4, n)
        assert sub[0][0] == b0 and sub[-1][1] == b1
        assert all(sub[i][1] == sub[i + 1][0] for i in range(3))
    assert split_range(10, 20, 3, 100, all_vs_all=False) == [(10, 13), (13, 16), (16, 20)]
