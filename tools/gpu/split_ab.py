"""A/B: the 10k all-vs-all as one launch vs a split -- the wide rows in one
k_rows_pl launch and the narrowest rows (<= 2048 columns) as a second launch
of the 512-thread WK 3 form (four workgroups per CU; diagnostics library,
PFAAI_ROWS_KERNEL=pl512 for the second run).  Wall time of the runs
(synchronized), medians over rounds, interleaved."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ.setdefault("PFAAI_HIP_LIB", os.path.join(ROOT, "parfastaai_amd", "lib", "libpfaai_hip_diag.so"))
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


def one():
    os.environ.pop("PFAAI_ROWS_KERNEL", None)
    eng.synchronize()
    t0 = time.perf_counter()
    eng.run(0, rows, 0, d)
    eng.synchronize()
    return (time.perf_counter() - t0) * 1e3


def split(cut):
    os.environ.pop("PFAAI_ROWS_KERNEL", None)
    eng.synchronize()
    t0 = time.perf_counter()
    eng.run(0, cut, 0, d)
    os.environ["PFAAI_ROWS_KERNEL"] = "pl512"
    eng.run(cut, rows, 0, d)
    eng.synchronize()
    os.environ.pop("PFAAI_ROWS_KERNEL", None)
    return (time.perf_counter() - t0) * 1e3


s2 = torch.cuda.Stream()


def split2(cut, kern):
    """the narrow rows on a second stream, concurrent with the wide launch"""
    os.environ.pop("PFAAI_ROWS_KERNEL", None)
    eng.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.run(0, cut, 0, d)
    if kern:
        os.environ["PFAAI_ROWS_KERNEL"] = kern
    eng.run(cut, rows, 0, d, stream=s2.cuda_stream)
    eng.synchronize()
    s2.synchronize()
    os.environ.pop("PFAAI_ROWS_KERNEL", None)
    return (time.perf_counter() - t0) * 1e3


cuts = [rows - 2048, rows - 1024]
res = {"one": []}
for c in cuts:
    res[f"split@{c}"] = []
    res[f"2stream@{c}/pl512"] = []
    res[f"2stream@{c}/pl"] = []
for r in range(7):
    res["one"].append(one())
    for c in cuts:
        res[f"split@{c}"].append(split(c))
        res[f"2stream@{c}/pl512"].append(split2(c, "pl512"))
        res[f"2stream@{c}/pl"].append(split2(c, None))
for k, v in res.items():
    print(f"{k:14s} median {np.median(v[1:]):.3f} ms  min {min(v[1:]):.3f}")
