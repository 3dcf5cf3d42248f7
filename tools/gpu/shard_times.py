"""Per-shard device times of the row kernel for split_rows(n, world) at 10k:
checks the row cost model of parfastaai_amd/shard.py on one GPU (each shard
run alone, as one rank of a world-size run would)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from parfastaai_amd import _capi, syn  # noqa: E402
from parfastaai_amd.datastruct import ParFAAIData  # noqa: E402
from parfastaai_amd.shard import split_rows  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
world = int(sys.argv[2]) if len(sys.argv) > 2 else 8
g = syn.generate(n, 100)
ds = ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"]).with_genome_major(g["G_off"], g["G_tet"])
eng = _capi.Engine(0, lib_path=os.environ.get("PFAAI_HIP_LIB"))  # (the diagnostics library for A/B switches)
eng.load(**ds.problem())
rows, pairs = eng.shape()
d = eng.alloc(pairs * 8)
eng.run(0, rows, 0, d)
fracs = [float(x) for x in os.environ.get("SHARD_FRACS", "").split(",") if x]
for label, kw in [("cost model", {}), ("pair balance", {"fixed_cols": 0})] + \
        [(f"fixed {f:.2f}n", {"fixed_cols": f * n}) for f in fracs]:
    blocks = split_rows(rows, world, **kw)
    ms = []
    for rb, re_ in blocks:
        t = []
        for _ in range(3):
            eng.timing(reset=True)
            eng.run(rb, re_, 0, d)
            _, b, r = eng.timing(reset=True)
            t.append(r)
        ms.append(float(np.median(t)))
    print(f"{label:12s} rows/shard {[b1 - b0 for b0, b1 in blocks]}")
    print(f"{label:12s} k_rows ms  {[round(x, 3) for x in ms]}  max {max(ms):.3f}  mean {np.mean(ms):.3f}")

# bench.py's pipeline chunks: a rank's block as 1, 2 or 4 k_rows launches
# (run table reused) -- the launch-tail cost of chunking the gather pipeline
from parfastaai_amd.shard import split_range  # noqa: E402

blocks = split_rows(rows, world)
for nch in (1, 2, 4):
    ms = []
    for rb, re_ in blocks:
        t = []
        for _ in range(3):
            eng.timing(reset=True)
            for j, (c0, c1) in enumerate(split_range(rb, re_, nch, rows)):
                eng.run(c0, c1, _capi.FLAG_KEEP_RUNS if j else 0, d)
            _, b, r = eng.timing(reset=True)
            t.append(b + r)
        ms.append(float(np.median(t)))
    print(f"chunks {nch}: k_blk + k_rows ms per shard {[round(x, 3) for x in ms]}  max {max(ms):.3f}")

# row cost profile: k_rows time of n/20-row blocks across the triangle, fitted
# as t = alpha * rows + beta * pairs -> the cost model's fixed part in column
# units (FIXED_COST_FRACTION * n = alpha / beta)
nb = 20
prof = []
for i in range(nb):
    rb, re_ = rows * i // nb, rows * (i + 1) // nb
    t = []
    for _ in range(3):
        eng.timing(reset=True)
        eng.run(rb, re_, _capi.FLAG_KEEP_RUNS, d)
        _, b, r = eng.timing(reset=True)
        t.append(r)
    npairs = sum(n - 1 - a for a in range(rb, re_))
    prof.append((re_ - rb, npairs, float(np.median(t))))
A = np.array([[r, p] for r, p, _ in prof], dtype=float)
y = np.array([t for _, _, t in prof])
(alpha, beta), *_ = np.linalg.lstsq(A, y, rcond=None)
print("row profile (rows, pairs, ms):", [(r, p, round(t, 3)) for r, p, t in prof])
print(f"fit: {alpha * 1e3:.3f} us per row + {beta * 1e6:.3f} ns per pair -> fixed = {alpha / beta:.0f} columns "
      f"= {alpha / beta / n:.3f} x n; residuals {[round(v, 3) for v in (A @ [alpha, beta] - y)]}")
eng.free(d)
