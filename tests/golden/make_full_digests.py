"""Whole-output digests of the BASELINE configs, computed by the CPU oracle.

    python tests/golden/make_full_digests.py [C2 C3 C4 ...]   (container side)

For each config the synthetic problem is generated exactly as the GPU tests
generate it (tools/syn_gen.c through parfastaai_amd.syn, deterministic), the
oracle's Appendix-A restatement (oracle/pfaai_oracle.c oracle_full_rows,
OpenMP over rows, pinned to the reference's E/sort restatement by
tests/test_oracle.py::test_full_rows_matches_ref, which is itself pinned to
every reference fixture) computes EVERY output pair, and the SHA-256 of the
full S (f64), N (i32) and AJI (f64) arrays in JAC order is written to
tests/golden/full_digests.json together with |E| and a digest of the
generated input arrays (so a mismatch on the GPU box can be told apart from
a generator difference).  The reference's own tests assert equality of the
entire JAC / AJI vectors (pfaai_tests.cpp:355-386); this is that assertion at
the sizes the benchmark uses, which the reference itself cannot run
(|E| > 2^31, ds_helper.hpp:209,365).

Configs (BASELINE.json configs[1..3]; corrected semantics -- on these DBs
every pair shares protein 0's core tetramers, so compat gives the same):
  C2  SYN 2 000 x 100 all-vs-all
  C3  SYN 10 000 x 100 all-vs-all
  C4  QT: target SYN 50 000 x 100, query SYN' 1 000 (seed + 1, clade q mod
      C), joined as the reference's QT loader (syn.qt_merge)
  C5  SYN 100 000 x 100 all-vs-all (5e9 pairs, 100 GB of S / N / AJI): the
      outputs never exist whole -- the oracle runs by row windows of at most
      WINDOW_PAIRS pairs and each window is fed, in JAC order, into one
      running SHA-256 per array (the same digests a whole-array hash gives);
      the GPU test feeds pfaai_stream's tiles into the same running hashes.
      The generated G arrays are dropped after the input digest (the oracle
      reads F and T only), so the container holds ~25 GB, not 35.

TEST INFRASTRUCTURE: runs the oracle as the checker; tests/test_gpu_configs.py
compares the device outputs with the committed digests.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "full_digests.json")

CONFIGS = {
    "C2": dict(kind="all", n=2000, P=100),
    "C3": dict(kind="all", n=10000, P=100),
    "C4": dict(kind="qt", nT=50000, nQ=1000, P=100, K=20),
    "C5": dict(kind="all", n=100000, P=100, streamed=True),
}
WINDOW_PAIRS = 125_000_000  # C5: pairs per oracle window (2.5 GB of S / N / AJI)


class RunningDigests:
    """One running SHA-256 per output array (S f64, N i32, AJI f64), fed with
    consecutive JAC-order pieces: equal to output_digests() of the whole
    arrays.  The three hashes run in their own threads (hashlib releases the
    GIL on large buffers), so a 100 GB stream hashes at ~3x one core."""

    def __init__(self):
        from concurrent.futures import ThreadPoolExecutor

        self.h = {k: hashlib.sha256() for k in ("S", "N", "AJI")}
        self.ex = ThreadPoolExecutor(max_workers=3)
        self.pairs = 0

    def update(self, S, N, AJI):
        parts = {"S": np.asarray(S, np.float64), "N": np.asarray(N, np.int32), "AJI": np.asarray(AJI, np.float64)}
        assert len(parts["S"]) == len(parts["N"]) == len(parts["AJI"])
        futs = [self.ex.submit(self.h[k].update, memoryview(np.ascontiguousarray(v)).cast("B"))
                for k, v in parts.items()]
        for f in futs:
            f.result()
        self.pairs += len(parts["S"])

    def hexdigests(self) -> dict:
        self.ex.shutdown()
        return {k: h.hexdigest() for k, h in self.h.items()}


def sha(*arrays) -> str:
    """SHA-256 over the arrays' little-endian bytes, in order."""
    h = hashlib.sha256()
    for a in arrays:
        a = np.ascontiguousarray(a)
        assert a.dtype.byteorder in "=<|"
        h.update(memoryview(a).cast("B"))
    return h.hexdigest()


def problem(name: str) -> dict:
    """The config's pfaai_problem fields (numpy arrays), generated as the GPU
    tests generate it."""
    from parfastaai_amd import _capi, syn

    c = CONFIGS[name]
    if c["kind"] == "all":
        g = syn.generate(c["n"], c["P"])
        return dict(mode=_capi.MODE_ALL, n_ids=c["n"], n_prot=c["P"], Lp=g["Lp"], F_prot=g["F_prot"],
                    F_genome=g["F_genome"], T=g["T"], G_off=g["G_off"], G_tet=g["G_tet"])
    nT, nQ, P, K = c["nT"], c["nQ"], c["P"], c["K"]
    gt = syn.generate(nT, P, clade_size=K)
    gq = syn.generate(nQ, P, clade_size=K, genome_seed=syn.DEFAULT_SEED + 1, n_clades=(nT + K - 1) // K,
                      clade_mod=True)
    m = syn.qt_merge(gt, gq)
    del gt, gq
    is_q = np.zeros(nT + nQ, np.uint8)
    is_q[nT:] = 1
    return dict(mode=_capi.MODE_QT, n_ids=nT + nQ, n_prot=P, n_qry=nQ, n_tgt=nT, is_q=is_q, Lp=m["Lp"],
                F_prot=m["F_prot"], F_genome=m["F_genome"], T=m["T"], G_off=m["G_off"], G_tet=m["G_tet"])


def input_digest(pb: dict) -> str:
    return sha(*(np.asarray(pb[k]) for k in ("Lp", "F_prot", "F_genome", "T", "G_off", "G_tet")))


def output_digests(S, N, AJI) -> dict:
    return {"S": sha(np.asarray(S, np.float64)), "N": sha(np.asarray(N, np.int32)),
            "AJI": sha(np.asarray(AJI, np.float64))}


def row_windows(n: int, max_pairs: int):
    """All-vs-all rows [lo, hi) cut so that no window holds more than
    max_pairs pairs (row r has n - 1 - r columns)."""
    lo = 0
    while lo < n:
        hi, pairs = lo, 0
        while hi < n and (hi == lo or pairs + (n - 1 - hi) <= max_pairs):
            pairs += n - 1 - hi
            hi += 1
        yield lo, hi
        lo = hi


def compute_streamed(name: str) -> dict:
    """An all-vs-all config whose outputs do not fit in memory: the oracle by
    row windows, each hashed in JAC order into RunningDigests."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    c = CONFIGS[name]
    t0 = time.time()
    pb = problem(name)
    t_gen = time.time() - t0
    din = input_digest(pb)
    nf, ng = len(pb["F_genome"]), len(pb["G_tet"])
    del pb["G_tet"], pb["G_off"]  # the oracle reads F and T only
    print(f"  {name}: generated in {t_gen:.0f}s, input digest {din[:12]}", flush=True)
    pr = O.Problem(pb)
    n = c["n"]
    rd = RunningDigests()
    ne = 0
    n_min, a_min, a_max = 1 << 30, 2.0, -1.0
    t1 = time.time()
    for lo, hi in row_windows(n, WINDOW_PAIRS):
        k = (hi - lo) * (n - 1) - (hi * (hi - 1) - lo * (lo - 1)) // 2  # sum of n - 1 - r over [lo, hi)
        S, N, A = np.empty(k), np.empty(k, np.int32), np.empty(k)
        ne += pr.full_rows(lo, hi, S, N, A)
        rd.update(S, N, A)
        if k:
            n_min, a_min, a_max = min(n_min, int(N.min())), min(a_min, float(A.min())), max(a_max, float(A.max()))
        del S, N, A
        print(f"  {name}: rows [{lo}, {hi}) of {n} at {time.time() - t1:.0f}s, |E| so far {ne}", flush=True)
    assert rd.pairs == n * (n - 1) // 2
    return {"config": c, "pairs": int(rd.pairs), "F": int(nf), "G": int(ng), "events": int(ne),
            "input_sha256": din, "sha256": rd.hexdigests(), "n_min": n_min, "aji_min": a_min, "aji_max": a_max,
            "oracle_s": round(time.time() - t1, 1), "generate_s": round(t_gen, 1), "window_pairs": WINDOW_PAIRS}


def compute(name: str, window: int = 1000) -> dict:
    if CONFIGS[name].get("streamed"):
        return compute_streamed(name)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    t0 = time.time()
    pb = problem(name)
    t_gen = time.time() - t0
    din = input_digest(pb)
    pr = O.Problem(pb)
    n = pr.n_pairs()
    S, N, A = np.empty(n), np.empty(n, np.int32), np.empty(n)
    rows = pr.mode.n_ids if pr.mode.mode == 0 else pr.mode.n_qry
    ni, nT = pr.mode.n_ids, pr.mode.n_tgt

    def first(r):
        return ni * r - (r + 1) * r // 2 if pr.mode.mode == 0 else r * nT

    ne = 0
    t1 = time.time()
    for lo in range(0, rows, window):
        hi = min(rows, lo + window)
        f, e = first(lo), first(hi)
        ne += pr.full_rows(lo, hi, S[f:e], N[f:e], A[f:e])
        print(f"  {name}: rows [{lo}, {hi}) of {rows} at {time.time() - t1:.0f}s", flush=True)
    out = {"config": CONFIGS[name], "pairs": int(n), "F": int(len(pb["F_genome"])), "G": int(len(pb["G_tet"])),
           "events": int(ne), "input_sha256": din, "sha256": output_digests(S, N, A),
           "n_min": int(N.min()), "aji_min": float(A.min()), "aji_max": float(A.max()),
           "oracle_s": round(time.time() - t1, 1), "generate_s": round(t_gen, 1)}
    return out


def main(argv):
    names = argv or list(CONFIGS)
    have = {}
    if os.path.exists(OUT):
        with open(OUT) as f:
            have = json.load(f)
    for name in names:
        print(f"{name} ...", flush=True)
        have[name] = compute(name)
        print(json.dumps({name: have[name]}), flush=True)
        with open(OUT, "w") as f:
            json.dump(have, f, indent=1, sort_keys=True)
            f.write("\n")


if __name__ == "__main__":
    sys.path.insert(0, ROOT)
    main(sys.argv[1:])
