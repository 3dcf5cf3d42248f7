"""Interleaved A/B of k_rows variants in one process (SYN all-vs-all).

    python tools/gpu/ab_rows.py --genomes 10000 --rounds 5 --variants PFAAI_ROWS_KERNEL=pl PFAAI_ROWS_KERNEL=fused
Each variant is an env setting read by pfaai_run (PFAAI_ROWS_KERNEL=pl|pl512|fused|worklist; PFAAI_ABLATE only
with the diagnostics library: PFAAI_HIP_LIB=parfastaai_amd/lib/libpfaai_hip_diag.so).
Prints per-variant median/min of build and row-kernel device times.
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
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--f-only", action="store_true")
ap.add_argument("--variants", nargs="+", default=["PFAAI_ROWS_KERNEL=pl", "PFAAI_ROWS_KERNEL=pl512"])
ap.add_argument("--rows", default=None, help="row range lo:hi (default: all rows)")
a = ap.parse_args()
g = syn.generate(a.genomes, a.prot)
ds = ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"])
if not a.f_only:
    ds.with_genome_major(g["G_off"], g["G_tet"])
eng = _capi.Engine(0)
eng.load(**ds.problem())
n_rows, n_pairs = eng.shape()
r0, r1 = (int(x) for x in a.rows.split(":")) if a.rows else (0, n_rows)
d = eng.alloc(n_pairs * 8)
res = {v: ([], []) for v in a.variants}
ref = None
for r in range(a.rounds + 1):
    for v in a.variants:
        for vv in a.variants:  # no setting leaks from one variant into the next
            for kv in vv.split(","):
                os.environ.pop(kv.split("=")[0], None)
        for kv in v.split(","):  # "K1=V1,K2=V2"
            k, val = kv.split("=")
            os.environ[k] = val
        eng.timing(reset=True)
        eng.run(r0, r1, 0, d)
        n, b, rr = eng.timing(reset=True)
        out = eng.d2h(d, n_pairs, np.float64)
        if ref is None:
            ref = out
        if "ABLATE" not in v:
            assert np.array_equal(out, ref), f"variant {v} differs"
        os.environ.pop("PFAAI_ABLATE", None)
        if r:
            res[v][0].append(b); res[v][1].append(rr)
for v, (b, rr) in res.items():
    if not b:
        continue
    print(f"{v:28s} build med {np.median(b):8.3f} min {np.min(b):8.3f} | rows med {np.median(rr):8.3f} min {np.min(rr):8.3f} ms")
eng.free(d)
