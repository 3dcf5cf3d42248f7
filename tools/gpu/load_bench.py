#!/usr/bin/env python3
"""Load-time transposition benchmark: SYN N x P, pfaai_load repeated, the
device span of each load's F / G build (HIP events, pfaai_load_timing) and
the path taken (pfaai_load_info).  --orient both | f (F only: G built) |
g (G only: F built).  The library comes from PFAAI_HIP_LIB (the diagnostics
build reads the A/B switch PFAAI_TSORT_DB, the sort's digit width).

    python tools/gpu/load_bench.py --genomes 10000 --orient both --reps 3
    python tools/gpu/load_bench.py --parts 8      # each rank's load of an 8-way
                                                  # row split (pfaai_load_rows)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genomes", type=int, default=10000)
    ap.add_argument("--prot", type=int, default=100)
    ap.add_argument("--orient", choices=["both", "f", "g"], default="both")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--parts", type=int, default=1, help="per-rank loads of a K-way row split (pfaai_load_rows)")
    a = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime per process)
    from parfastaai_amd import _capi, syn
    from parfastaai_amd.datastruct import ParFAAIData

    t0 = time.perf_counter()
    g = syn.generate(a.genomes, a.prot)
    ds = ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"]).with_genome_major(g["G_off"], g["G_tet"])
    pb = ds.problem()
    drop = {"both": (), "f": ("G_off", "G_tet"), "g": ("Lp", "F_prot", "F_genome")}[a.orient]
    pb = {k: v for k, v in pb.items() if k not in drop}
    print(f"[load_bench] SYN {a.genomes} x {a.prot} |F| = {len(g['F_genome'])} in {time.perf_counter() - t0:.1f}s",
          file=sys.stderr, flush=True)
    eng = _capi.Engine(0, lib_path=os.environ.get("PFAAI_HIP_LIB"))
    from parfastaai_amd.shard import split_rows

    blocks = [None] if a.parts <= 1 else split_rows(a.genomes, a.parts)
    for blk in blocks:
        dev = []
        for _ in range(a.reps):
            eng.load(**pb, rows=blk)
            dev.append(round(eng.load_timing()[2], 3))
        print(json.dumps({"genomes": a.genomes, "prot": a.prot, "F": len(g["F_genome"]), "orient": a.orient,
                          "rows": list(blk) if blk else "all", "path": eng.load_info(), "device_ms": dev,
                          "tsort_db": os.environ.get("PFAAI_TSORT_DB")}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
