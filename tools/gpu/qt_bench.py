#!/usr/bin/env python3
"""Query-vs-target AJI (the reference's -r path, BASELINE config C4 shape) on
one MI355X: a target SYN DB of n_tgt genomes and a query SYN' DB of n_qry
new genomes (clade q mod C, seed + 1) joined as the reference's
QT loader does (parfastaai_amd.syn.qt_merge), QT mode with the corrected
semantics.  Times k_blk + k_rows_pl over all query rows
with the inputs resident (HIP events), re-checks sampled query rows against
the CPU oracle's dense restatement (S, N bit-exact), prints one JSON line.

    python tools/gpu/qt_bench.py --targets 50000 --queries 1000
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402  (one HIP runtime per process)


def log(m):
    print(f"[qt_bench] {m}", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--targets", type=int, default=50000)
    ap.add_argument("--queries", type=int, default=1000)
    ap.add_argument("--prot", type=int, default=100)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--check-rows", type=int, default=2)
    args = ap.parse_args()
    import oracle as O
    from parfastaai_amd import _capi, syn

    nT, nQ, P, K = args.targets, args.queries, args.prot, 20
    t0 = time.perf_counter()
    gt = syn.generate(nT, P, clade_size=K)
    gq = syn.generate(nQ, P, clade_size=K, genome_seed=syn.DEFAULT_SEED + 1, n_clades=(nT + K - 1) // K,
                      clade_mod=True)
    m = syn.qt_merge(gt, gq)
    del gt, gq
    n_f = len(m["F_genome"])
    log(f"QT SYN targets={nT} queries={nQ} P={P} |F|={n_f} in {time.perf_counter() - t0:.1f}s")
    is_q = np.zeros(nT + nQ, np.uint8)
    is_q[nT:] = 1
    pb = dict(mode=_capi.MODE_QT, n_ids=nT + nQ, n_prot=P, n_qry=nQ, n_tgt=nT, is_q=is_q, Lp=m["Lp"],
              F_prot=m["F_prot"], F_genome=m["F_genome"], T=m["T"], G_off=m["G_off"], G_tet=m["G_tet"])
    eng = _capi.Engine(0)
    t0 = time.perf_counter()
    eng.load(**pb)
    log(f"pfaai_load {time.perf_counter() - t0:.1f}s")
    n_rows, n_pairs = eng.shape()
    aji = torch.empty(n_pairs, dtype=torch.float64, device="cuda:0")
    S = torch.empty(n_pairs, dtype=torch.float64, device="cuda:0")
    N = torch.empty(n_pairs, dtype=torch.int32, device="cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    eng.run(0, n_rows, _capi.FLAG_EMIT_JAC, aji.data_ptr(), S.data_ptr(), N.data_ptr(), stream=st)
    torch.cuda.synchronize()
    n_events = eng.stats()["n_events"]
    eng.timing(reset=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.run(0, n_rows, 0, aji.data_ptr(), stream=st)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.steps
    n_runs, ms_build, ms_rows = eng.timing(reset=True)
    ms_build, ms_rows = ms_build / n_runs, ms_rows / n_runs
    pr = O.Problem(pb)
    ok = True
    Sh, Nh, Ah = S.cpu().numpy(), N.cpu().numpy(), aji.cpu().numpy()
    for q in np.linspace(0, nQ - 1, args.check_rows).astype(int):
        So, No, _ = pr.dense_rows(nT + int(q), nT + int(q) + 1)
        k = slice(int(q) * nT, (int(q) + 1) * nT)
        ok &= bool(np.array_equal(Sh[k], So[0, :nT]) and np.array_equal(Nh[k], No[0, :nT]))
        ok &= bool(np.array_equal(Ah[k], np.where(Nh[k] > 0, Sh[k] / np.maximum(Nh[k], 1), 0.0)))
    line = {
        "what": "query-vs-target AJI (-r, corrected semantics), BASELINE config C4 shape on 1 GPU",
        "targets": nT, "queries": nQ, "proteins": P, "F": n_f, "pairs": n_pairs, "events": n_events,
        "ms_per_step": round(wall * 1e3, 3), "pairs_per_s": round(n_pairs / wall, 1),
        "k_blk_ms": round(ms_build, 3), "k_rows_ms": round(ms_rows, 3),
        "events_per_s": round(n_events / (ms_rows * 1e-3), 1),
        "rows_check_vs_oracle_bit_exact": ok,
        "aji_range": [float(Ah.min()), float(Ah.max())],
    }
    print(json.dumps(line), flush=True)
    eng.close()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
