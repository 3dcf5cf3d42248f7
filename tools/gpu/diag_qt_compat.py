import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests")); sys.path.insert(0, os.path.join(os.getcwd(), "oracle"))
import numpy as np, torch
from helpers import qt_syn
from parfastaai_amd import _capi
import oracle as O
e = _capi.Engine(0)
ds = qt_syn(dict(n_tgt=400, n_qry=90, n_prot=30, clade_size=9), genome_major=True)
pb = ds.problem()
C = _capi.FLAG_REF_COMPAT
e.load(**pb); a1 = e.compute(C); a1b = e.compute(C)
print("F+G repeat equal:", all(np.array_equal(x, y) for x, y in zip(a1, a1b)))
f = dict(pb); f.pop("G_off"); f.pop("G_tet")
e.load(**f); a2 = e.compute(C)
pr = O.Problem(pb, compat=True)
ref = pr.ref_run()
for nm, a in (("F+G", a1), ("F-only", a2)):
    print(nm, "vs oracle S:", np.array_equal(a[1], ref["S"]), "N:", np.array_equal(a[2], ref["N"]), "AJI:", np.array_equal(a[0], ref["AJI"]))
d = np.flatnonzero(a1[0] != a2[0])
print("ndiff", len(d), d[:10])
for i in d[:5]:
    print(i, divmod(i, 400), a1[1][i], a1[2][i], a2[1][i], a2[2][i], ref["S"][i], ref["N"][i])
