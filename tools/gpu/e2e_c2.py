#!/usr/bin/env python3
"""End-to-end drop-in check at BASELINE config C2 (SYN 2 000 genomes x 100
SCPs): the same SQLite DB through our CLI (one MI355X) and through the
reference CLI (oracle/_ref/par_fastaai.x, built from its own sources; 16
OpenMP threads on the box's host cores); the two CSV outputs must be byte
identical.  Prints one JSON line with both walls and each CLI's phase lines.

    python tools/gpu/e2e_c2.py [--genomes 2000]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genomes", type=int, default=2000)
    ap.add_argument("--prot", type=int, default=100)
    ap.add_argument("--workdir", default="/tmp/pfaai_e2e")
    ap.add_argument("--ref-timeout", type=int, default=600)
    ap.add_argument("--ours-args", default="", help="extra par_fastaai_amd options, e.g. --stream-csv")
    ap.add_argument("--ref-csv", default=None, help="compare with this reference CSV instead of running the reference")
    a = ap.parse_args()
    from parfastaai_amd import syn

    os.makedirs(a.workdir, exist_ok=True)
    db = os.path.join(a.workdir, f"syn{a.genomes}.db")
    t0 = time.perf_counter()
    if not os.path.exists(db):
        syn.write_db(db, a.genomes, a.prot)
    t_db = time.perf_counter() - t0
    print(f"[e2e] DB {db} ({os.path.getsize(db) / 1e9:.2f} GB) in {t_db:.1f}s", file=sys.stderr, flush=True)

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
        return w, [l.strip() for l in out.splitlines() if ":" in l and ("ms" in l or "time" in l.lower())]

    ours_csv, ref_csv = os.path.join(a.workdir, "ours.csv"), os.path.join(a.workdir, "ref.csv")
    w_ours, l_ours = run([os.path.join(ROOT, "parfastaai_amd", "lib", "par_fastaai_amd"), db, ours_csv,
                          *a.ours_args.split()])
    print(f"[e2e] ours {w_ours:.2f}s", file=sys.stderr, flush=True)
    env = dict(os.environ, OMP_NUM_THREADS="16")
    if a.ref_csv:  # an earlier reference run of the same DB
        ref_csv, w_ref, l_ref = a.ref_csv, float("nan"), []
    else:
        w_ref, l_ref = run([os.path.join(ROOT, "oracle", "_ref", "par_fastaai.x"), db, ref_csv], env, a.ref_timeout)
        print(f"[e2e] reference {w_ref:.2f}s", file=sys.stderr, flush=True)
    same = open(ours_csv, "rb").read() == open(ref_csv, "rb").read()
    pairs = a.genomes * (a.genomes - 1) // 2
    print(json.dumps({
        "what": "end-to-end CLI, SQLite DB -> CSV (BASELINE config C2 shape)",
        "genomes": a.genomes, "proteins": a.prot, "pairs": pairs,
        "ours_wall_s": round(w_ours, 2), "ours_args": a.ours_args, "ours_phases": l_ours,
        "reference_wall_s": round(w_ref, 2), "reference_threads": 16, "reference_phases": l_ref,
        "speedup_wall": round(w_ref / w_ours, 1), "csv_byte_identical": same,
        "csv_bytes": os.path.getsize(ours_csv),
    }), flush=True)
    sys.exit(0 if same else 1)


if __name__ == "__main__":
    main()
