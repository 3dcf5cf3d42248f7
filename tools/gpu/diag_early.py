#!/usr/bin/env python3
"""One-off diagnosis (round 6): the narrow rows' first member round issued
before S5 (a library built with it, EARLY_LIB) gave wrong N in the C3 digest
test's G-only phase after the diagnostics-variant tests had run in the same
process.  This runs those tests, then the C3 sequence (F+G load, full run,
8 row blocks, G-only reload + run) on the shipped library and on EARLY_LIB,
and reports where the two phase-3 outputs differ (cells, rows, values)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import pytest  # noqa: E402
import torch  # noqa: E402


def seq(lib, pb, n, npairs):
    from parfastaai_amd import _capi
    from parfastaai_amd.shard import split_rows
    eng = _capi.Engine(0, lib_path=lib)
    st = torch.cuda.current_stream().cuda_stream

    def run(rb, re, flags, bufs):
        eng.run(rb, re, flags | _capi.FLAG_EMIT_JAC, *(b.data_ptr() for b in bufs), stream=st)
        torch.cuda.synchronize()

    mk = lambda: [torch.full((npairs,), -1.0, dtype=torch.float64, device="cuda:0"),
                  torch.full((npairs,), -1.0, dtype=torch.float64, device="cuda:0"),
                  torch.full((npairs,), -1, dtype=torch.int32, device="cuda:0")]
    eng.load(**pb)
    b1 = mk()
    run(0, n, 0, b1)
    b2 = mk()
    for i, (rb, re) in enumerate(split_rows(n, 8)):
        run(rb, re, _capi.FLAG_KEEP_RUNS if i else 0, b2)
    del b1, b2
    eng.load(**{k: v for k, v in pb.items() if k not in ("Lp", "F_prot", "F_genome")})
    b3 = mk()
    run(0, n, 0, b3)
    out = [x.cpu().numpy() for x in b3]
    eng.close()
    return out


def main():
    rc = pytest.main(["-q", "-m", "gpu", "-p", "no:cacheprovider",
                      os.path.join(ROOT, "tests", "test_gpu_stream.py") + "::test_diagnostic_variants_equal_release_form"])
    print("variant tests rc", rc, flush=True)
    import make_full_digests as mkd
    pb = mkd.problem("C3")
    n = 10000
    npairs = n * (n - 1) // 2
    ref = seq(None, pb, n, npairs)
    early = seq(os.environ["EARLY_LIB"], pb, n, npairs)
    names = ("AJI", "S", "N")
    for nm, a, b in zip(names, ref, early):
        d = np.nonzero(a != b)[0]
        print(f"{nm}: {d.size} cells differ", flush=True)
        if d.size:
            # row of pair index k (all-vs-all: k = n a + b - (a + 2)(a + 1) / 2)
            rows = []
            for k in d[:2000:max(1, d.size // 2000)]:
                lo, hi = 0, n - 1
                while lo < hi:
                    m = (lo + hi + 1) // 2
                    if n * m - m * (m + 1) // 2 <= k:
                        lo = m
                    else:
                        hi = m - 1
                rows.append(lo)
            rows = np.array(rows)
            print(f"  rows min {rows.min()} max {rows.max()} distinct {np.unique(rows).size}", flush=True)
            for k in d[:8]:
                print(f"  k {k}: ref {a[k]!r} early {b[k]!r}; ref S {ref[1][k]!r} early S {early[1][k]!r}", flush=True)


if __name__ == "__main__":
    main()
