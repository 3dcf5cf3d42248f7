#!/usr/bin/env python3
"""Kernel statistics from a rocprofv3 --kernel-trace database (rocpd SQLite,
the tool's default output on this image) or its CSV kernel trace
(`--output-format csv`: <prefix>_kernel_trace.csv): per kernel the number of
dispatches and the mean / median / min / max duration, and optionally the
dispatch sequence of one load or step (--timeline).

    python tools/rocpd_stats.py gpurun_out/r04b/prof/load_results.db [--csv OUT] [--timeline N]
"""
import argparse
import csv
import re
import sqlite3
import statistics
import sys


def short(name):
    """Kernel name without the argument list (templates kept)."""
    depth = 0
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return name[:i]
    return name


def dispatches(db):
    if db.endswith(".csv"):  # rocprofv3 --output-format csv: <prefix>_kernel_trace.csv
        with open(db) as f:
            rows = list(csv.DictReader(f))
        out = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Stream_Id"]))
               for r in rows]
        return sorted(out, key=lambda d: d[1])
    con = sqlite3.connect(db)
    names = {r[0]: r[1] for r in con.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
    rows = con.execute("select kernel_id, start, end, stream_id from rocpd_kernel_dispatch order by start").fetchall()
    return [(short(names.get(k, str(k))), s, e, st) for k, s, e, st in rows]


def stats(ds):
    by = {}
    for name, s, e, _ in ds:
        by.setdefault(name, []).append((e - s) / 1e6)  # ns -> ms
    out = []
    for name, v in by.items():
        out.append({"kernel": name, "calls": len(v), "total_ms": round(sum(v), 4), "mean_ms": round(sum(v) / len(v), 4),
                    "median_ms": round(statistics.median(v), 4), "min_ms": round(min(v), 4),
                    "max_ms": round(max(v), 4)})
    return sorted(out, key=lambda r: -r["total_ms"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--timeline", type=int, default=0, help="print the first N dispatches (start offset, ms)")
    ap.add_argument("--match", default=None, help="regex: only kernels whose name matches")
    a = ap.parse_args()
    ds = dispatches(a.db)
    if a.match:
        ds = [d for d in ds if re.search(a.match, d[0])]
    rows = stats(ds)
    w = csv.DictWriter(open(a.csv, "w") if a.csv else sys.stdout, fieldnames=list(rows[0].keys()))
    w.writeheader()
    w.writerows(rows)
    if a.timeline:
        t0 = ds[0][1]
        for name, s, e, st in ds[:a.timeline]:
            print(f"{(s - t0) / 1e6:10.4f} {(e - s) / 1e6:8.4f} s{st} {name[:110]}")


if __name__ == "__main__":
    main()
