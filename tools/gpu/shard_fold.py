"""One-GPU emulation of the 8-way row split, contiguous blocks against folded
ones, 10k all-vs-all (each rank's work run alone, device time by HIP events
on the rank's stream, median of --reps):

  contiguous   rank r owns block r of shard.split_rows(n, 8, cus) (round 4's
               form: slowest 1.11-1.14 ms, the first block's two rounds of the
               widest rows)
  folded       rank r owns blocks r and 2W-1-r of a 2W-way cost split (one
               wide, one narrow), run as two pfaai_runs on two streams at once,
               so the narrow rows fill the CUs the wide block's last round
               leaves idle

Prints one JSON line per form and repeat: rows, device ms per rank, max,
mean, max/mean.

    python tools/gpu/shard_fold.py [n] [world] [--reps 5]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from parfastaai_amd import _capi, syn  # noqa: E402
from parfastaai_amd.datastruct import ParFAAIData  # noqa: E402
from parfastaai_amd.shard import split_rows  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
n = int(args[0]) if args else 10000
world = int(args[1]) if len(args) > 1 else 8
reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 5
g = syn.generate(n, 100)
ds = ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"]).with_genome_major(g["G_off"], g["G_tet"])
eng = _capi.Engine(0)
eng.load(**ds.problem())
rows, pairs = eng.shape()
cus = torch.cuda.get_device_properties(0).multi_processor_count
aji = torch.empty(pairs, dtype=torch.float64, device="cuda:0")
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
eng.run(0, rows, 0, aji.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()


def timed(blocks):
    """Device ms of the rank's blocks, each on its own stream, all at once."""
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    cur = torch.cuda.current_stream()
    e0.record(cur)
    ends = []
    for (rb, re_), st in zip(blocks, (sa, sb)):
        st.wait_event(e0)
        eng.run(rb, re_, 0, aji.data_ptr(), stream=st.cuda_stream)
        ev = torch.cuda.Event()
        ev.record(st)
        ends.append(ev)
    for ev in ends:
        cur.wait_event(ev)
    e1.record(cur)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


contig = [[b] for b in split_rows(rows, world, cus=cus)]
b2 = split_rows(rows, 2 * world, cus=cus)
folded = [[b2[r], b2[2 * world - 1 - r]] for r in range(world)]
for rep in range(2):
    for label, ranks in (("contiguous", contig), ("folded", folded)):
        ms = [float(np.median([timed(bl) for _ in range(reps)])) for bl in ranks]
        print(json.dumps({"label": label, "rep": rep, "rows": [[b1 - b0 for b0, b1 in bl] for bl in ranks],
                          "blocks": ranks, "ms": [round(x, 4) for x in ms], "max": round(max(ms), 4),
                          "mean": round(float(np.mean(ms)), 4), "max_over_mean": round(max(ms) / float(np.mean(ms)), 4),
                          "whole_ms": round(timed([(0, rows)]), 4)}), flush=True)
