"""One-GPU emulation of the 8-way row split of 10k all-vs-all, contiguous
blocks (shard.split_rows with the CU count, the shipped split) against
block-cyclic row lists (shard.cyclic_rows: 32-row groups dealt in snake
order, one launch per rank over its list through pfaai_set_row_order).
Each rank's work runs alone (device ms by HIP events around pfaai_run on
the rank's stream, median of --reps); the cyclic ranks' outputs, each into
its own full-size array, must assemble to the whole-matrix run bit for bit.
Prints one JSON line per form and repeat: device ms per rank, max, mean,
max/mean, sum / whole.

    python tools/gpu/shard_cyclic.py [n] [world] [--reps 5] [--group 32]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from parfastaai_amd import _capi, syn  # noqa: E402
from parfastaai_amd.datastruct import ParFAAIData  # noqa: E402
from parfastaai_amd.shard import cyclic_rows, row_segments, split_rows  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
n = int(args[0]) if args else 10000
world = int(args[1]) if len(args) > 1 else 8
reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 5
group = int(sys.argv[sys.argv.index("--group") + 1]) if "--group" in sys.argv else 32
g = syn.generate(n, 100)
ds = ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"]).with_genome_major(g["G_off"], g["G_tet"])
eng = _capi.Engine(0)
eng.load(**ds.problem())
rows, pairs = eng.shape()
cus = torch.cuda.get_device_properties(0).multi_processor_count
whole = torch.empty(pairs, dtype=torch.float64, device="cuda:0")
part = torch.empty(pairs, dtype=torch.float64, device="cuda:0")
st = torch.cuda.Stream()
eng.run(0, rows, 0, whole.data_ptr(), stream=st.cuda_stream)
torch.cuda.synchronize()


def timed(rb, re_, out):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    eng.run(rb, re_, 0, out.data_ptr(), stream=st.cuda_stream)
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def jac_spans(rlist):
    base = lambda a: n * a - a * (a + 1) // 2  # JAC index of (a, a + 1)
    return [(base(lo), base(hi)) for lo, hi in row_segments(rlist)]


contig = split_rows(rows, world, cus=cus)
cyc = cyclic_rows(rows, world, group)
assembled = torch.full((pairs,), -1.0, dtype=torch.float64, device="cuda:0")
for rep in range(2):
    eng.set_row_order(None)
    w_ms = float(np.median([timed(0, rows, whole) for _ in range(reps)]))
    ms = [float(np.median([timed(b0, b1, part) for _ in range(reps)])) for b0, b1 in contig]
    print(json.dumps({"label": "contiguous", "rep": rep, "rows": [b1 - b0 for b0, b1 in contig],
                      "ms": [round(x, 4) for x in ms], "max": round(max(ms), 4), "mean": round(float(np.mean(ms)), 4),
                      "max_over_mean": round(max(ms) / float(np.mean(ms)), 4), "whole_ms": round(w_ms, 4),
                      "sum_over_whole": round(sum(ms) / w_ms, 4)}), flush=True)
    ms = []
    for rl in cyc:
        eng.set_row_order(rl)
        ms.append(float(np.median([timed(0, len(rl), part) for _ in range(reps)])))
        if rep == 0:
            for f, l in jac_spans(rl):
                assembled[f:l] = part[f:l]
    eng.set_row_order(None)
    ok = bool(torch.equal(assembled, whole)) if rep == 0 else None
    print(json.dumps({"label": f"cyclic{group}", "rep": rep, "rows": [len(r) for r in cyc],
                      "ms": [round(x, 4) for x in ms], "max": round(max(ms), 4), "mean": round(float(np.mean(ms)), 4),
                      "max_over_mean": round(max(ms) / float(np.mean(ms)), 4), "whole_ms": round(w_ms, 4),
                      "sum_over_whole": round(sum(ms) / w_ms, 4), "assembled_bit_exact": ok}), flush=True)
    if rep == 0 and not ok:
        sys.exit(1)
