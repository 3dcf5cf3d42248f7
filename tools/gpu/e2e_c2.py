#!/usr/bin/env python3
"""End-to-end drop-in check at BASELINE config C2 (SYN 2 000 genomes x 100
SCPs): the same SQLite DB through
  ours     par_fastaai_amd (this repo's CLI: parallel `<p>_genomes` ingest,
           F built on the GPU, k_blk_end + k_rows_pl, parallel CSV writer),
  dropin   oracle/_ref/par_fastaai_hip.x (the reference's main.cpp with
           INTEGRATION.md §1's five-line swap: its own loader and CSV writer,
           no E, ParFAAIHipImpl on the GPU) -- if built,
  ref      oracle/_ref/par_fastaai.x (the reference, built from its sources),
each run --repeats times (medians reported), the reference with
OMP_NUM_THREADS = this process's usable CPUs (affinity capped by the cgroup quota,
bench.usable_cpus; BASELINE.md plan) unless
--threads is given; all CSV outputs must be byte identical.  Prints one JSON
line with the walls, every run's phase lines and the host.

    python tools/gpu/e2e_c2.py [--genomes 2000] [--repeats 3]
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import bench  # host_info / usable_cpus

    ap = argparse.ArgumentParser()
    ap.add_argument("--genomes", type=int, default=2000)
    ap.add_argument("--prot", type=int, default=100)
    ap.add_argument("--workdir", default="/tmp/pfaai_e2e")
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--threads", type=int, default=None, help="reference OpenMP threads (default: usable CPUs)")
    ap.add_argument("--ref-timeout", type=int, default=600)
    ap.add_argument("--ours-args", default="", help="extra par_fastaai_amd options, e.g. --stream-csv")
    ap.add_argument("--skip-ref", action="store_true", help="ours and the drop-in only (no reference runs)")
    a = ap.parse_args()
    from parfastaai_amd import syn

    threads = a.threads or bench.usable_cpus()
    os.makedirs(a.workdir, exist_ok=True)
    db = os.path.join(a.workdir, f"syn{a.genomes}.db")
    t0 = time.perf_counter()
    if not os.path.exists(db):
        syn.write_db(db, a.genomes, a.prot)
    print(f"[e2e] DB {db} ({os.path.getsize(db) / 1e9:.2f} GB) in {time.perf_counter() - t0:.1f}s", file=sys.stderr,
          flush=True)

    def run(cmd, env=None, timeout=600):
        t = time.perf_counter()
        p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
        while True:  # a heartbeat line every 30 s (a long silent run looks hung)
            try:
                out, err = p.communicate(timeout=30)
                break
            except subprocess.TimeoutExpired:
                if time.perf_counter() - t > timeout:
                    p.kill()
                    raise SystemExit(f"{cmd[0]} timed out")
                print(f"[e2e] {os.path.basename(cmd[0])} running {time.perf_counter() - t:.0f}s", file=sys.stderr,
                      flush=True)
        w = time.perf_counter() - t
        if p.returncode:
            print(out[-3000:], err[-3000:], file=sys.stderr)
            raise SystemExit(f"{cmd[0]} exited {p.returncode}")
        for l in err.splitlines():  # PFAAI_TRACE_COMPUTE=1: the library's phase lines
            if l.startswith("[pfaai_"):
                print(f"[e2e] {os.path.basename(cmd[0])} {l}", file=sys.stderr, flush=True)
        return w, [l.strip() for l in out.splitlines() if ":" in l and ("ms" in l or "time" in l.lower())]

    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    clis = {"ours": [os.path.join(ROOT, "parfastaai_amd", "lib", "par_fastaai_amd")],
            "dropin": [os.path.join(ROOT, "oracle", "_ref", "par_fastaai_hip.x")],
            "ref": [os.path.join(ROOT, "oracle", "_ref", "par_fastaai.x")]}
    if not os.path.exists(clis["dropin"][0]):
        del clis["dropin"]
    if a.skip_ref:
        del clis["ref"]
    walls, phases, csvs = {}, {}, {}
    for k in range(a.repeats):
        for name, cmd in clis.items():
            out = os.path.join(a.workdir, f"{name}.csv")
            extra = a.ours_args.split() if name == "ours" else []
            w, ph = run(cmd + [db, out, *extra], env if name != "ours" else None, a.ref_timeout)
            walls.setdefault(name, []).append(round(w, 3))
            phases.setdefault(name, []).append(ph)
            data = open(out, "rb").read()
            if name in csvs:
                assert data == csvs[name], f"{name}: run {k} wrote different bytes"
            csvs[name] = data
            print(f"[e2e] {name} run {k}: {w:.2f}s", file=sys.stderr, flush=True)
    first = next(iter(csvs.values()))
    same = all(v == first for v in csvs.values())
    # the reference binary's CSV of this DB, pinned by its SHA-256
    # (tests/golden/full_digests.json C2_cli_csv) -- checked even when the
    # reference is not run here
    import hashlib
    ref_digest = None
    if a.genomes == 2000 and a.prot == 100:
        ref_digest = json.load(open(os.path.join(ROOT, "tests", "golden", "full_digests.json")))["C2_cli_csv"]["sha256"]
    digest_ok = None if ref_digest is None else all(hashlib.sha256(v).hexdigest() == ref_digest for v in csvs.values())
    med = {k: round(statistics.median(v), 3) for k, v in walls.items()}
    pairs = a.genomes * (a.genomes - 1) // 2
    res = {"what": "end-to-end CLI, SQLite DB -> CSV (BASELINE config C2 shape); medians of repeated runs",
           "genomes": a.genomes, "proteins": a.prot, "pairs": pairs, "repeats": a.repeats,
           "ours_wall_s": med.get("ours"), "ours_args": a.ours_args, "dropin_wall_s": med.get("dropin"),
           "reference_wall_s": med.get("ref"), "reference_threads": threads, "walls_s": walls,
           "phases_last_run": {k: v[-1] for k, v in phases.items()}, "host": bench.host_info(threads),
           "csv_byte_identical": same, "csv_bytes": len(first),
           "csv_equals_reference_binary_digest": digest_ok}
    if "ref" in med:
        res["speedup_wall"] = round(med["ref"] / med["ours"], 1)
        if "dropin" in med:
            res["speedup_wall_dropin"] = round(med["ref"] / med["dropin"], 1)
    print(json.dumps(res), flush=True)
    sys.exit(0 if same and digest_ok is not False else 1)


if __name__ == "__main__":
    main()
