"""The first pfaai_run after a load against the next ones (device time of
each, eng.timing), 10k all-vs-all: does the first carry a one-time cost?

    python tools/gpu/first_step.py [n] [--busy]

--busy: keep the GPU busy (torch matmuls, ~50 ms) right before each load, to
tell a clock ramp from a cold cache / TLB.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from parfastaai_amd import _capi, syn  # noqa: E402
from parfastaai_amd.datastruct import ParFAAIData  # noqa: E402

busy = "--busy" in sys.argv
args = [a for a in sys.argv[1:] if a != "--busy"]
n = int(args[0]) if args else 10000
g = syn.generate(n, 100)
ds = ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"]).with_genome_major(g["G_off"], g["G_tet"])
eng = _capi.Engine(0)
out = {"deferred_env": os.environ.get("HIP_ENABLE_DEFERRED_LOADING"), "busy": busy}
for rep in range(2):
    if busy:
        a = torch.randn(4096, 4096, device="cuda:0")
        for _ in range(40):
            a = a @ a
            a = a / a.norm()
        torch.cuda.synchronize()
    eng.load(**ds.problem())
    rows, pairs = eng.shape()
    d = eng.alloc(pairs * 8) if rep == 0 else d
    ts = []
    for _ in range(4):
        eng.timing(reset=True)
        eng.run(0, rows, 0, d)
        _, b, r = eng.timing(reset=True)
        ts.append(round(b + r, 3))
    out[f"load{rep}_runs_ms"] = ts
print(json.dumps(out), flush=True)
