"""The C QT join used at scale (parfastaai_amd.syn.qt_merge, tools/syn_gen.c)
equals the numpy statement of the reference's QT loader join
(tests/helpers.py:qt_syn, pinned against the reference's QT fixtures by
tests/test_gpu_parity.py)."""
import numpy as np
import pytest

from helpers import qt_syn
from parfastaai_amd import syn


@pytest.mark.parametrize("nT,nQ,P,K", [(60, 25, 20, 6), (7, 30, 5, 3), (40, 40, 12, 10)])
def test_qt_merge_equals_numpy_join(nT, nQ, P, K):
    ds = qt_syn(dict(n_tgt=nT, n_qry=nQ, n_prot=P, clade_size=K), genome_major=True)
    gt = syn.generate(nT, P, clade_size=K)
    gq = syn.generate(nQ, P, clade_size=K, genome_seed=syn.DEFAULT_SEED + 1, n_clades=(nT + K - 1) // K,
                      clade_mod=True)
    m = syn.qt_merge(gt, gq)
    pb = ds.problem()
    for k in ("Lp", "F_prot", "F_genome", "T", "G_off", "G_tet"):
        assert np.array_equal(m[k], pb[k]), k
    assert (m["n_tgt"], m["n_qry"]) == (nT, nQ)
