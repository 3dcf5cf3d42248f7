#!/usr/bin/env python3
"""Output-tile streaming at scale (BASELINE config C5
shape): SYN N genomes x P SCPs, all-vs-all, every AJI tile computed on the
GPU, copied to pinned host memory while the next tile computes
(pfaai_stream), and copied by the sink into one host array of the whole
JAC-ordered output (N = 100 000: 5e9 pairs, 40 GB).  Prints one JSON line:
pairs/s end to end (device compute + D2H + host copy, inputs resident),
|E|, tiles, and the device-side k_rows time.  The stream runs once per
--sinks entry on the same load, so the parts of the wall separate:
  noop   the sink returns at once: device compute + D2H into the pinned tile
         buffers (the library's side alone)
  copy   one numpy copy of each tile into the output array (round 4's sink)
  par    the same copy cut into --threads slices on a thread pool (numpy
         releases the GIL while it copies)
The wall of the last sink is the line's wall_s.

    python tools/gpu/stream_bench.py --genomes 100000 --tile-pairs 268435456 --sinks noop copy par
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one HIP runtime per process)


def log(m):
    print(f"[stream_bench] {m}", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genomes", type=int, default=100000)
    ap.add_argument("--prot", type=int, default=100)
    ap.add_argument("--tile-pairs", type=int, default=1 << 28)
    ap.add_argument("--check-rows", type=int, default=2, help="rows re-checked against a pfaai_run of them")
    ap.add_argument("--sinks", nargs="+", default=["par"], choices=["noop", "copy", "par"])
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--device-only", action="store_true",
                    help="the same row tiles by pfaai_run into two device buffers, no D2H: the row kernels "
                         "alone (the profile command of C5 -- the stream's tile copies are blit kernels that "
                         "share the CUs)")
    args = ap.parse_args()
    from concurrent.futures import ThreadPoolExecutor
    from parfastaai_amd import _capi, syn

    t0 = time.perf_counter()
    g = syn.generate(args.genomes, args.prot)
    n_f = len(g["F_genome"])
    log(f"SYN N={args.genomes} P={args.prot} |F|={n_f} generated in {time.perf_counter() - t0:.1f}s")
    eng = _capi.Engine(0)
    t0 = time.perf_counter()
    eng.load(mode=_capi.MODE_ALL, n_ids=args.genomes, n_prot=args.prot, Lp=g["Lp"], F_prot=g["F_prot"],
             F_genome=g["F_genome"], T=g["T"], G_off=g["G_off"], G_tet=g["G_tet"])
    del g
    log(f"pfaai_load {time.perf_counter() - t0:.1f}s")
    n_rows, n_pairs = eng.shape()
    out = np.empty(n_pairs, dtype=np.float64)
    out[:: 1 << 9] = 0.0  # touch every 4-KB page: the walls measure copies, not first-touch faults
    tiles = [0]
    last = [time.perf_counter()]
    pool = ThreadPoolExecutor(max_workers=args.threads)

    def sink(kind):
        def fn(rb, re, first, aji, S, N):
            if kind == "copy":
                out[first: first + len(aji)] = aji
            elif kind == "par":
                n, k = len(aji), args.threads
                cuts = [n * i // k for i in range(k + 1)]
                list(pool.map(lambda i: out.__setitem__(slice(first + cuts[i], first + cuts[i + 1]),
                                                        aji[cuts[i]: cuts[i + 1]]), range(k)))
            tiles[0] += 1
            now = time.perf_counter()
            if now - last[0] > 20:
                log(f"tile {tiles[0]}: rows [{rb}, {re})")
                last[0] = now
            return 0
        return fn

    if args.device_only:
        # row tiles of <= tile_pairs pairs, as pfaai_stream cuts them
        cuts = [0]
        while cuts[-1] < n_rows:
            lo, hi = cuts[-1] + 1, n_rows
            while lo < hi:  # the largest re whose span fits
                mid = (lo + hi + 1) // 2
                if eng.row_span(cuts[-1], mid)[1] <= args.tile_pairs:
                    lo = mid
                else:
                    hi = mid - 1
            cuts.append(lo)
        bufs = [torch.empty(args.tile_pairs, dtype=torch.float64, device="cuda:0") for _ in range(2)]
        st = torch.cuda.current_stream().cuda_stream
        for rep in range(3):  # pass 0 builds the window tables and warms the clocks; pass 1 counts |E|; pass 2 is timed back to back
            eng.timing(reset=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            n_events = 0
            for k in range(len(cuts) - 1):
                f, c = eng.row_span(cuts[k], cuts[k + 1])
                eng.run(cuts[k], cuts[k + 1], 0, bufs[k & 1].data_ptr() - f * 8, stream=st)
                if rep == 1:  # (the event count is read after the run: a synchronising read per tile)
                    torch.cuda.synchronize()
                    n_events += eng.stats()["n_events"]
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            n_runs, ms_build, ms_rows = eng.timing(reset=True)
            if rep == 1:
                events = n_events
        print(json.dumps({
            "what": "C5 row tiles by pfaai_run into device buffers (no D2H): the row kernels alone",
            "genomes": args.genomes, "proteins": args.prot, "F": n_f, "pairs": n_pairs, "events": events,
            "tiles": len(cuts) - 1, "tile_pairs": args.tile_pairs, "wall_s": round(wall, 3),
            "device_ms_rows": round(ms_rows, 2), "device_ms_build": round(ms_build, 2), "runs": n_runs,
            "device_pairs_per_s": round(n_pairs / (ms_rows + ms_build) * 1e3, 1)}), flush=True)
        eng.close()
        return

    walls = {}
    for kind in args.sinks:
        tiles[0] = 0
        eng.timing(reset=True)
        t0 = time.perf_counter()
        n_events = eng.stream(0, n_rows, args.tile_pairs, 0, sink(kind))
        walls[kind] = round(time.perf_counter() - t0, 3)
        n_runs, ms_build, ms_rows = eng.timing(reset=True)
        log(f"sink {kind}: streamed {tiles[0]} tiles in {walls[kind]:.2f}s")
    wall = walls[args.sinks[-1]]
    # spot check: a few rows recomputed with pfaai_run into device memory
    ok = True
    for r in np.linspace(0, n_rows - 2, args.check_rows).astype(int):
        f, c = eng.row_span(int(r), int(r) + 1)
        d = torch.empty(max(c, 1), dtype=torch.float64, device="cuda:0")
        eng.run(int(r), int(r) + 1, 0, d.data_ptr() - f * 8, stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        ok &= bool(np.array_equal(d[:c].cpu().numpy(), out[f: f + c]))
    vmin, vmax = float(out.min()), float(out.max())
    line = {
        "what": "pfaai_stream all-vs-all, AJI tiles to host (SURVEY 8f rank 4, config C5 shape on 1 GPU)",
        "genomes": args.genomes, "proteins": args.prot, "F": n_f, "pairs": n_pairs, "events": n_events,
        "tiles": tiles[0], "tile_pairs": args.tile_pairs,
        "wall_s": round(wall, 3), "pairs_per_s": round(n_pairs / wall, 1), "walls_by_sink_s": walls,
        "sink_threads": args.threads,
        "device_ms_rows": round(ms_rows, 2), "device_ms_build": round(ms_build, 2), "runs": n_runs,
        "device_pairs_per_s": round(n_pairs / (ms_rows + ms_build) * 1e3, 1),
        "d2h_GBps_effective": round(8 * n_pairs / wall / 1e9, 2),
        "rows_recheck_bit_exact": ok, "aji_range": [vmin, vmax],
    }
    print(json.dumps(line), flush=True)
    eng.close()
    if not ok or vmin < 0.0 or vmax > 1.0:
        sys.exit(1)


if __name__ == "__main__":
    main()
