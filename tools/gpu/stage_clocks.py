"""Row-kernel stage clocks (diagnostics library: `python tools/build_native.py
--diag`, loaded through PFAAI_HIP_LIB): where the protein loop's time goes,
per stage, for the waves of the first 256 workgroups of the launch.

    python tools/gpu/stage_clocks.py [--genomes 10000] [--v2] [--rows lo:hi] [--qt 50000:1000]
k_rows_pl (PFAAI_PL_CLK) by default, k_rows_v2 (PFAAI_V2_CLK) with --v2.
"""
import argparse
import os

os.environ.setdefault("PFAAI_HIP_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))), "parfastaai_amd", "lib", "libpfaai_hip_diag.so"))
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from parfastaai_amd import _capi, syn  # noqa: E402
from parfastaai_amd.datastruct import ParFAAIData  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--genomes", type=int, default=10000)
ap.add_argument("--v2", action="store_true")
ap.add_argument("--rows", default=None, help="row range lo:hi (default: all rows)")
ap.add_argument("--la", action="store_true", help="stage names of k_rows_pl's lookahead form (narrow launches)")
ap.add_argument("--qt", default=None, help="targets:queries -- the query-vs-target (C4) shape of tools/gpu/qt_bench.py "
                "(window spans) instead of all-vs-all")
a = ap.parse_args()
eng = _capi.Engine(0)
if a.qt:
    nT, nQ = (int(x) for x in a.qt.split(":"))
    K = 20
    gt = syn.generate(nT, 100, clade_size=K)
    gq = syn.generate(nQ, 100, clade_size=K, genome_seed=syn.DEFAULT_SEED + 1, n_clades=(nT + K - 1) // K,
                      clade_mod=True)
    m = syn.qt_merge(gt, gq)
    del gt, gq
    is_q = np.zeros(nT + nQ, np.uint8)
    is_q[nT:] = 1
    eng.load(mode=_capi.MODE_QT, n_ids=nT + nQ, n_prot=100, n_qry=nQ, n_tgt=nT, is_q=is_q, Lp=m["Lp"],
             F_prot=m["F_prot"], F_genome=m["F_genome"], T=m["T"], G_off=m["G_off"], G_tet=m["G_tet"])
    del m
else:
    g = syn.generate(a.genomes, 100)
    ds = ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"]).with_genome_major(g["G_off"], g["G_tet"])
    eng.load(**ds.problem())
rows, pairs = eng.shape()
r0, r1 = (int(x) for x in a.rows.split(":")) if a.rows else (0, rows)
d = eng.alloc(pairs * 8)
if a.v2:
    os.environ["PFAAI_ROWS_KERNEL"] = "v2"
eng.run(r0, r1, 0, d)  # warm
eng.timing(reset=True)
eng.run(r0, r1, 0, d)
_, _, r_plain = eng.timing(reset=True)
eng.debug_clocks(arm=True)
os.environ["PFAAI_V2_CLK" if a.v2 else "PFAAI_PL_CLK_LA" if a.la else "PFAAI_PL_CLK"] = "1"
eng.run(r0, r1, 0, d)
_, b, r = eng.timing(reset=True)
c = eng.debug_clocks().astype(np.float64)
if a.v2:
    names = ["T issue + S3", "M/S2/S1 issue", "S5 normalise", "S4 prefetched", "S4 further rounds", "long runs",
             "barrier"]
elif a.la:
    names = ["S5 normalise", "S3 tasks", "S2/S1 issue", "T + next round-1 issue", "S4b round 1 (prefetched)",
             "S4b rounds 2+/whole", "recycle+barrier"]
else:
    names = ["S4a issue", "S3 tasks", "S2/S1 issue", "-", "S4b round 1", "S4b rounds 2+/whole + T issue",
             "recycle+barrier", "S5 normalise (first)"]
K = len(names)
used = c[:, 0, :K].sum(axis=1) > 0
c = c[used]
tot = c[:, :, :K].sum(axis=2)
print(f"{'k_rows_v2' if a.v2 else 'k_rows_pl'} rows [{r0}, {r1}): {r_plain:.3f} ms plain, {r:.3f} ms clock variant; "
      f"{used.sum()} workgroups sampled; per wave-loop total: median {np.median(tot):.0f} cycles")
for j, nm in enumerate(names):
    x = c[:, :, j]
    print(f"  {nm:22s} share {x.sum() / tot.sum():6.3f}   wave0 {x[:, 0].mean():10.0f}   wave15 {x[:, 15].mean():10.0f}"
          f"   max-wave {x.max(axis=1).mean():10.0f}")
if a.v2:
    print(f"  further rounds per wave-row: mean {c[:, :, 7].mean():.1f}  max {c[:, :, 7].max():.0f}")
eng.free(d)
