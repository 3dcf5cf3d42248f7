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
