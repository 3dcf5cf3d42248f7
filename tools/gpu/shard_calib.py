"""Row-block balance of the N-way split, measured on one GPU (each block run
alone, as one rank would): the shard times of shard.split_rows, then a few
rounds of re-cutting by the measured cost (each block's measured time
spread over its rows in proportion to the model cost, the cuts moved to
equal shares), and the model's fit to the final cuts.

    python tools/gpu/shard_calib.py [n] [world] [rounds] [--cuts c1,c2,...;c1,c2,...]

--cuts: time these splits (each twice) instead of the re-cutting rounds.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from parfastaai_amd import _capi, syn  # noqa: E402
from parfastaai_amd.datastruct import ParFAAIData  # noqa: E402
from parfastaai_amd.shard import row_costs, split_rows  # noqa: E402

cut_sets = None
if "--cuts" in sys.argv:
    k = sys.argv.index("--cuts")
    cut_sets = [[int(x) for x in cs.split(",")] for cs in sys.argv[k + 1].split(";")]
    del sys.argv[k:k + 2]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
world = int(sys.argv[2]) if len(sys.argv) > 2 else 8
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
reps = 5
g = syn.generate(n, 100)
ds = ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"]).with_genome_major(g["G_off"], g["G_tet"])
eng = _capi.Engine(0)
eng.load(**ds.problem())
rows, pairs = eng.shape()
d = eng.alloc(pairs * 8)
eng.run(0, rows, 0, d)


def times(blocks):
    out = []
    for rb, re_ in blocks:
        t = []
        for _ in range(reps):
            eng.timing(reset=True)
            eng.run(rb, re_, 0, d)
            _, b, r = eng.timing(reset=True)
            t.append(b + r)
        out.append(float(np.median(t)))
    return out


def report(label, blocks, ms):
    print(json.dumps({"label": label, "rows": [b1 - b0 for b0, b1 in blocks], "cuts": [b0 for b0, _ in blocks[1:]],
                      "ms": [round(x, 4) for x in ms], "max": round(max(ms), 4), "mean": round(float(np.mean(ms)), 4),
                      "max_over_mean": round(max(ms) / float(np.mean(ms)), 4)}), flush=True)


if cut_sets:
    for rep in range(2):
        for cs in cut_sets:
            edges = [0] + cs + [rows]
            blocks = [(edges[i], edges[i + 1]) for i in range(len(edges) - 1)]
            report(f"cuts rep {rep}", blocks, times(blocks))
    eng.free(d)
    sys.exit(0)
blocks = split_rows(rows, world, cus=torch.cuda.get_device_properties(0).multi_processor_count)
ms = times(blocks)
report("model", blocks, ms)
w = row_costs(rows)  # the model's per-row cost
for it in range(rounds):
    # measured cost density: each block's time spread over its rows like the model's cost
    dens = np.empty(rows)
    for (b0, b1), t in zip(blocks, ms):
        dens[b0:b1] = w[b0:b1] * (t / w[b0:b1].sum())
    cum = np.concatenate([[0.0], np.cumsum(dens)])
    cuts = [int(np.searchsorted(cum, cum[-1] * r / world)) for r in range(1, world)]
    edges = [0] + cuts + [rows]
    blocks = [(edges[i], edges[i + 1]) for i in range(world)]
    ms = times(blocks)
    report(f"measured round {it + 1}", blocks, ms)
eng.free(d)
