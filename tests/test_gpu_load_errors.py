"""pfaai_load rejects malformed input with PFAAI_ERR_INVALID (7) and a
message -- on small inputs and on inputs large enough (> 2^20 entries) that
the host-side checks run over several threads."""
import numpy as np
import pytest

from parfastaai_amd import _capi, syn

pytestmark = pytest.mark.gpu


def _pb(n, P, **kw):
    g = syn.generate(n, P, **kw)
    return dict(mode=_capi.MODE_ALL, n_ids=n, n_prot=P, Lp=g["Lp"], F_prot=g["F_prot"].copy(),
                F_genome=g["F_genome"].copy(), T=g["T"], G_off=g["G_off"], G_tet=g["G_tet"].copy())


@pytest.mark.parametrize("n,P", [(60, 8), (400, 100)], ids=["small", "threaded"])
def test_load_rejects_bad_input(engine, n, P):
    pb = _pb(n, P)
    nf = len(pb["F_genome"])
    if n == 400:
        assert nf > (1 << 21)  # several threads in par_for
    cases = []
    b = dict(pb); b["F_genome"] = pb["F_genome"].copy(); b["F_genome"][nf - 3] = n  # genome id out of range
    cases.append((b, "genome id"))
    b = dict(pb); b["F_prot"] = pb["F_prot"].copy(); b["F_prot"][nf // 2] = P  # protein id out of range
    cases.append((b, "protein id"))
    b = dict(pb); b["G_tet"] = pb["G_tet"].copy(); b["G_tet"][len(b["G_tet"]) - 2] = 160000
    cases.append((b, "G_tet"))
    # two members of one run swapped (late in F): unsorted
    Lp = pb["Lp"]
    t = int(np.flatnonzero(np.diff(Lp) >= 3)[-1])
    i = int(Lp[t])
    b = dict(pb); b["F_genome"] = pb["F_genome"].copy(); b["F_prot"] = pb["F_prot"].copy()
    b["F_genome"][[i, i + 1]] = b["F_genome"][[i + 1, i]]
    b["F_prot"][[i, i + 1]] = b["F_prot"][[i + 1, i]]
    if (b["F_prot"][i], b["F_genome"][i]) != (pb["F_prot"][i], pb["F_genome"][i]):
        cases.append((b, "sorted"))
    for bad, what in cases:
        with pytest.raises(_capi.PfaaiError) as ei:
            engine.load(**bad)
        assert ei.value.code == 7 and what in str(ei.value), (what, str(ei.value))
    engine.load(**pb)  # the good problem still loads and runs
    aji, _, _ = engine.compute(0)
    assert len(aji) == n * (n - 1) // 2 and np.all((aji >= 0) & (aji <= 1))


@pytest.mark.parametrize("n,P", [(60, 8), (400, 100)], ids=["small", "threaded"])
def test_load_rejects_bad_lp_and_g(engine, n, P):
    """Lp is checked (non-decreasing, so every interior entry <= n_f) before
    any F access; G lists must be strictly ascending sets of F's
    memberships (checked on the device against F)."""
    pb = _pb(n, P)
    nf = len(pb["F_genome"])
    cases = []
    b = dict(pb); b["Lp"] = pb["Lp"].copy(); b["Lp"][5] = nf + 1000  # interior past the end
    cases.append((b, "non-decreasing"))
    b = dict(pb); b["Lp"] = pb["Lp"].copy()
    t = int(np.flatnonzero(np.diff(b["Lp"]) > 0)[len(b["Lp"]) // 4 % 7])
    b["Lp"][t + 1], b["Lp"][t] = b["Lp"][t], b["Lp"][t + 1] + 1  # a descent
    cases.append((b, "non-decreasing"))
    G_off, G_tet = pb["G_off"], pb["G_tet"]
    k = int(np.flatnonzero(np.diff(G_off) >= 3)[-1])
    lo = int(G_off[k])
    b = dict(pb); b["G_tet"] = G_tet.copy(); b["G_tet"][[lo, lo + 1]] = b["G_tet"][[lo + 1, lo]]
    cases.append((b, "strictly ascending"))
    # a membership F does not hold: the last entry of a list moved to a free tetramer above it
    hi = int(G_off[k + 1]) - 1
    if G_tet[hi] + 1 < 160000:
        b = dict(pb); b["G_tet"] = G_tet.copy(); b["G_tet"][hi] += 1
        cases.append((b, "does not hold"))
    for bad, what in cases:
        with pytest.raises(_capi.PfaaiError) as ei:
            engine.load(**bad)
        assert ei.value.code == 7 and what in str(ei.value), (what, str(ei.value))
    engine.load(**pb)
    aji, _, _ = engine.compute(0)
    assert np.all((aji > 0) & (aji <= 1))
