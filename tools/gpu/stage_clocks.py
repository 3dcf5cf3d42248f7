"""k_rows_pl stage clocks at 10k (PFAAI_PL_CLK=1, diagnostics library:
`python tools/build_native.py --diag`, loaded through PFAAI_HIP_LIB): where the protein loop's
time goes, per stage, for the waves of the first 256 workgroups."""
import os

os.environ.setdefault("PFAAI_HIP_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))), "parfastaai_amd", "lib", "libpfaai_hip_diag.so"))
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from parfastaai_amd import _capi, syn  # noqa: E402
from parfastaai_amd.datastruct import ParFAAIData  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
g = syn.generate(n, 100)
ds = ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"]).with_genome_major(g["G_off"], g["G_tet"])
eng = _capi.Engine(0)
eng.load(**ds.problem())
rows, pairs = eng.shape()
d = eng.alloc(pairs * 8)
eng.run(0, rows, 0, d)  # warm
eng.debug_clocks(arm=True)
os.environ["PFAAI_PL_CLK"] = "1"
eng.timing(reset=True)
eng.run(0, rows, 0, d)
_, b, r = eng.timing(reset=True)
c = eng.debug_clocks().astype(np.float64)
names = ["T + S4a issue", "S3 tasks", "S2/S1 issue", "S5 normalise", "S4b round 1", "S4b rounds 2+/whole", "recycle+barrier"]
tot = c[:, :, :7].sum(axis=2)
print(f"row kernel {r:.3f} ms (clock variant); per wave-loop total: median {np.median(tot):.0f} cycles")
for j, nm in enumerate(names):
    x = c[:, :, j]
    print(f"  {nm:22s} share {x.sum() / tot.sum():6.3f}   wave0 {x[:, 0].mean():10.0f}   wave15 {x[:, 15].mean():10.0f}")
eng.free(d)
