"""Per-stage clock breakdown of k_rows_pl (diagnostics flag 0x1000).

    python tools/gpu/pl_stages.py --genomes 10000 [--ablate N]
Stage slots (cycles summed over proteins, per workgroup; mean over
workgroups): 0 T-issue  1 member-issue  2 prefetch-issue  3 S5 normalise
4 S4 atomics/rounds/whole  5 S3 tasks  6 barrier wait.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from parfastaai_amd import _capi, syn  # noqa: E402
from parfastaai_amd.datastruct import ParFAAIData  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--genomes", type=int, default=10000)
ap.add_argument("--prot", type=int, default=100)
ap.add_argument("--ablate", type=int, default=0)
ap.add_argument("--variant", type=int, default=12)
a = ap.parse_args()
g = syn.generate(a.genomes, a.prot)
ds = ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"])
ds.with_genome_major(g["G_off"], g["G_tet"])
eng = _capi.Engine(0)
eng.load(**ds.problem())
n_rows, n_pairs = eng.shape()
d = eng.alloc(n_pairs * 8)
sbuf = eng.alloc(max(n_pairs * 8, n_rows * 8 * 8 * 4))
nbuf = eng.alloc(n_pairs * 4)
os.environ["PFAAI_ROWS_OCC"] = str(a.variant)
eng.run(0, n_rows, 0, d)  # warm
os.environ["PFAAI_ABLATE"] = str(0x10 | a.ablate)
eng.timing(reset=True)
eng.run(0, n_rows, 0, d, d_S=sbuf, d_N=nbuf)
n, b, rr = eng.timing(reset=True)
t = eng.d2h(sbuf, n_rows * 8, np.float64).reshape(n_rows, 8)
t = t[t[:, 7] > 0]
names = ["T-issue", "member-issue", "prefetch", "S5 norm", "S4 atomics", "S3 tasks", "barrier"]
tot = t[:, :7].sum(axis=1)
print(f"rows kernel {rr:.3f} ms (with timers); workgroups {len(t)}; mean cycles/WG {tot.mean():.0f} "
      f"({tot.mean() / t[0, 7]:.0f} per protein)")
for k, nm in enumerate(names):
    print(f"  {nm:14s} {t[:, k].mean() / t[0, 7]:9.0f} cyc/protein  {100 * t[:, k].sum() / tot.sum():5.1f} %")
