#!/usr/bin/env python3
"""Interleaved A/B of the load's transposition-sort variants (diagnostics
library; SYN all-vs-all, F and G given: the checked run-end sort the bench
loads with).  Per variant and round: one pfaai_load (device span from
pfaai_load_timing) and one full pfaai_run whose AJI must equal the first
variant's bit for bit (the walk data G_pos / G_end the sort writes are what
the row kernel reads).

    PFAAI_HIP_LIB=parfastaai_amd/lib/libpfaai_hip_diag.so \\
        python tools/gpu/ab_sort.py --genomes 10000 --rounds 5 --variants - PFAAI_SORT_DIRECT=1
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genomes", type=int, default=10000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", nargs="+", default=["-", "PFAAI_SORT_DIRECT=1"],
                    help="NAME=VALUE environment settings per variant ('-': none)")
    a = ap.parse_args()
    import numpy as np
    import torch
    from parfastaai_amd import _capi, syn
    from parfastaai_amd.datastruct import ParFAAIData

    g = syn.generate(a.genomes, 100)
    pb = ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"]).with_genome_major(
        g["G_off"], g["G_tet"]).problem()
    eng = _capi.Engine(0, lib_path=os.environ.get("PFAAI_HIP_LIB"))
    names = [v.split("=")[0] for v in a.variants if v != "-"]
    res = {v: [] for v in a.variants}
    ref = None
    ok = True
    for _ in range(a.rounds):
        for v in a.variants:
            for n in names:
                os.environ.pop(n, None)
            if v != "-":
                k, val = v.split("=", 1)
                os.environ[k] = val
            eng.load(**pb)
            res[v].append(eng.load_timing()[2])
            rows, pairs = eng.shape()
            d = torch.empty(pairs, dtype=torch.float64, device="cuda:0")
            eng.run(0, rows, 0, d.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            h = d.cpu().numpy()
            if ref is None:
                ref = h
            else:
                ok &= bool(np.array_equal(h, ref))
    for n in names:
        os.environ.pop(n, None)
    for v in a.variants:
        x = np.array(res[v])
        print(f"{v:28s} load device ms  med {np.median(x):7.3f}  min {x.min():7.3f}  all {np.round(x, 3).tolist()}")
    print(json.dumps({"aji_equal_across_variants": ok, "path": eng.load_info()}))
    eng.close()
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
