"""The multi-device group of the C ABI (pfaai_group_*: SURVEY 8b's
pfaai_create over a device list with the RCCL communicator inside; the
reference's distributeGenomePairs, algorithm_impl.hpp:100-120).

The GPU box has one device, so the group runs with one rank here: its
communicator is RCCL's (ncclCommInitAll over [0]), its load is the per-rank
load of the whole row range, its run writes the caller's device array in
place.  Checked: AJI, S and N equal a single context's run bit for bit (ALL
and QT), the blocks cover the rows, bad device lists are refused before
anything is created, a run before a load is refused.  The N > 1 gather
(grouped ncclSend / ncclRecv into device 0) runs only on a multi-GPU node:
its row blocks and spans are the ones bench.py's ranks use (tests/
test_adapter_split.py pins pfaai::split_rows to shard.split_rows).

Everything else of the N > 1 path runs here through a peer-gather group
whose members share the one GPU (pfaai_group_create_flags,
PFAAI_GROUP_PEER_GATHER): the concurrent per-member pfaai_load_rows, the
block buffers and their base-pointer offsets (blk - first * esz), the
per-member streams, and the gather into device-0 arrays (hipMemcpyPeerAsync
after each member's event in place of the ncclSend / ncclRecv pair) -- equal
to a single context bit for bit in ALL and QT, with 2, 3 and 5 members."""
import numpy as np
import pytest
import torch

from parfastaai_amd import _capi, syn
from parfastaai_amd.datastruct import ParFAAIData

pytestmark = pytest.mark.gpu


def _all_problem(n=400, P=20):
    g = syn.generate(n, P, clade_size=8)
    return ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"]).with_genome_major(
        g["G_off"], g["G_tet"]).problem()


def _outputs(npairs):
    aji = torch.full((npairs,), -1.0, dtype=torch.float64, device="cuda:0")
    S = torch.full((npairs,), -1.0, dtype=torch.float64, device="cuda:0")
    N = torch.full((npairs,), -1, dtype=torch.int32, device="cuda:0")
    return aji, S, N


def _engine_run(engine, pb):
    engine.load(**pb)
    rows, npairs = engine.shape()
    aji, S, N = _outputs(npairs)
    engine.run(0, rows, _capi.FLAG_EMIT_JAC, aji.data_ptr(), S.data_ptr(), N.data_ptr(),
               stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return aji.cpu().numpy(), S.cpu().numpy(), N.cpu().numpy()


@pytest.mark.parametrize("kind", ["all", "qt"])
def test_group_of_one_equals_a_context(engine, kind):
    if kind == "all":
        pb = _all_problem()
    else:
        nT, nQ, P = 300, 40, 15
        m = syn.qt_merge(syn.generate(nT, P, clade_size=6), syn.generate(nQ, P, clade_size=6, seed=7))
        is_q = np.zeros(nT + nQ, np.uint8)
        is_q[nT:] = 1
        pb = dict(mode=_capi.MODE_QT, n_ids=nT + nQ, n_prot=P, n_qry=nQ, n_tgt=nT, is_q=is_q, Lp=m["Lp"],
                  F_prot=m["F_prot"], F_genome=m["F_genome"], T=m["T"], G_off=m["G_off"], G_tet=m["G_tet"])
    ref = _engine_run(engine, pb)
    grp = _capi.Group([0])
    try:
        grp.load(**pb)
        rows, npairs = grp.shape()
        assert grp.blocks() == [(0, rows)]
        aji, S, N = _outputs(npairs)
        torch.cuda.synchronize()
        grp.run(_capi.FLAG_EMIT_JAC, aji.data_ptr(), S.data_ptr(), N.data_ptr())
        got = (aji.cpu().numpy(), S.cpu().numpy(), N.cpu().numpy())
        for x, y in zip(got, ref):
            assert np.array_equal(x, y)
        # AJI alone (no S / N)
        aji2 = torch.full((npairs,), -1.0, dtype=torch.float64, device="cuda:0")
        grp.run(0, aji2.data_ptr())
        assert np.array_equal(aji2.cpu().numpy(), ref[0])
    finally:
        grp.close()


def _qt_problem():
    nT, nQ, P = 300, 40, 15
    m = syn.qt_merge(syn.generate(nT, P, clade_size=6), syn.generate(nQ, P, clade_size=6, seed=7))
    is_q = np.zeros(nT + nQ, np.uint8)
    is_q[nT:] = 1
    return dict(mode=_capi.MODE_QT, n_ids=nT + nQ, n_prot=P, n_qry=nQ, n_tgt=nT, is_q=is_q, Lp=m["Lp"],
                F_prot=m["F_prot"], F_genome=m["F_genome"], T=m["T"], G_off=m["G_off"], G_tet=m["G_tet"])


@pytest.mark.parametrize("kind,members", [("all", 2), ("all", 3), ("all", 5), ("qt", 3)])
def test_peer_gather_group_on_one_gpu_equals_a_context(engine, kind, members):
    """The n > 1 group path with every member on device 0: rank loads of
    non-trivial blocks, block buffers, the gather at each block's JAC span."""
    pb = _all_problem(n=700, P=20) if kind == "all" else _qt_problem()
    ref = _engine_run(engine, pb)
    grp = _capi.Group([0] * members, peer_gather=True)
    try:
        grp.load(**pb)
        rows, npairs = grp.shape()
        blocks = grp.blocks()
        assert len(blocks) == members and blocks[0][0] == 0 and blocks[-1][1] == rows
        assert all(b > a for a, b in blocks), blocks  # every member has rows
        aji, S, N = _outputs(npairs)
        torch.cuda.synchronize()
        grp.run(_capi.FLAG_EMIT_JAC, aji.data_ptr(), S.data_ptr(), N.data_ptr())
        got = (aji.cpu().numpy(), S.cpu().numpy(), N.cpu().numpy())
        for x, y in zip(got, ref):
            assert np.array_equal(x, y)
        aji2 = torch.full((npairs,), -1.0, dtype=torch.float64, device="cuda:0")
        grp.run(0, aji2.data_ptr())  # AJI alone: the S / N block buffers are not touched
        assert np.array_equal(aji2.cpu().numpy(), ref[0])
    finally:
        grp.close()


def test_group_refuses_bad_device_lists_and_early_runs():
    ndev = torch.cuda.device_count()
    for devs in ([-1], [ndev], [0, 0]):
        with pytest.raises(_capi.PfaaiError) as e:
            _capi.Group(devs)
        assert e.value.code == 7  # PFAAI_RC_INVALID
    grp = _capi.Group([0])
    try:
        d = torch.zeros(4, dtype=torch.float64, device="cuda:0")
        with pytest.raises(_capi.PfaaiError):
            grp.run(0, d.data_ptr())  # nothing loaded
    finally:
        grp.close()
