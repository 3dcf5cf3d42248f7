"""Summarise rocprofv3 --pmc passes (tools/gpu/pmc.sh) per kernel.

Reads <dir>/p*/run_counter_collection.csv (one counter group per pass, each
over the same 10k all-vs-all run), averages every counter over the dispatches
of each kernel, derives the ratios DESIGN.md quotes, and writes

  profiles/<tag>_pmc.json   -- every kernel, every counter, derived ratios
  profiles/pmc_k_rows.json  -- HBM bytes per k_rows launch (bench.py's
                               roofline.traffic)

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3):
FETCH_SIZE and WRITE_SIZE are in KiB; the x2 gfx950 FETCH correction is
calibrated only for 16-B-per-lane streaming reads.  k_rows' reads are 4-8 B
gathers (member ids, work records, T entries), so the raw figure is used and
the x2 figure is recorded next to it as an upper bound.

usage: python tools/pmc_summary.py gpurun_out/pmc r01 [--no-k-rows] [--what "..."]
  --no-k-rows   a profile of another workload (C4, C5): write only
                profiles/<tag>_pmc.json, not bench.py's pmc_k_rows.json
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    n = name.split("(")[0]
    for pre in ("void ",):
        if n.startswith(pre):
            n = n[len(pre):]
    return n


def collect(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} | {"_dispatches": max(len(v) for v in cs.values())}
            for k, cs in acc.items()}


def derive(c):
    out = {}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        out["hbm_read_bytes"] = c["FETCH_SIZE"] * 1024
        out["hbm_read_bytes_x2_bound"] = 2 * c["FETCH_SIZE"] * 1024
        out["hbm_write_bytes"] = c["WRITE_SIZE"] * 1024
        out["hbm_bytes"] = out["hbm_read_bytes"] + out["hbm_write_bytes"]
    if c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0) > 0:
        out["l2_hit_rate"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    if c.get("SQ_WAVE_CYCLES", 0) > 0:
        w = c["SQ_WAVE_CYCLES"]
        out["wave_frac_waiting"] = c.get("SQ_WAIT_ANY", 0) / w
        out["wave_frac_issue_stall"] = c.get("SQ_WAIT_INST_ANY", 0) / w
        out["wave_frac_active"] = c.get("SQ_ACTIVE_INST_ANY", 0) / w
    if c.get("SQ_ACTIVE_INST_VALU", 0) > 0 and c.get("GRBM_GUI_ACTIVE", 0) > 0:
        # SQ_ACTIVE_INST_* count quad-cycles summed over waves; GRBM_GUI_ACTIVE is
        # the kernel's cycles summed over the 8 XCDs (MI355X_MICROARCH.md): the
        # fraction of every SIMD's cycles issuing VALU (1024 SIMDs)
        out["valu_busy"] = c["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / (c["GRBM_GUI_ACTIVE"] / 8)
        out["kernel_cycles"] = c["GRBM_GUI_ACTIVE"] / 8
    if c.get("SQ_LDS_IDX_ACTIVE", 0) > 0:
        out["lds_conflict_frac"] = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"]
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    d = args[0] if args else "gpurun_out/pmc"
    tag = args[1] if len(args) > 1 else "r01"
    what = sys.argv[sys.argv.index("--what") + 1] if "--what" in sys.argv else "10k SYN all-vs-all"
    if "--what" in sys.argv:
        args.remove(what) if what in args else None
    ks = collect(d)
    if not ks:
        sys.exit(f"no counter CSVs under {d}")
    res = {k: {"counters": c, "derived": derive(c)} for k, c in ks.items() if k.startswith("pfaai::") or "pfaai::" in k}
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    with open(os.path.join(prof, f"{tag}_pmc.json"), "w") as f:
        json.dump({"source": f"rocprofv3 --pmc --kernel-trace, one counter group per pass, {what}",
                   "kernels": res}, f, indent=1, sort_keys=True)
    # One all-vs-all step may run two row kernels at once (pfaai_launch.hpp
    # launch_narrow: the wide rows as 1024-thread workgroups on the step's
    # stream, the narrow end as 512-thread ones on the side stream).  The step
    # figures add both: bytes and instructions summed; VALU busy over the sum
    # of their cycles, since counter collection serialises the dispatches.
    rows = sorted((k for k in res if "k_rows" in k),
                  key=lambda k: -res[k]["derived"].get("kernel_cycles", 0))
    if rows and "--no-k-rows" not in sys.argv:
        k = rows[0]
        dv = res[k]["derived"]

        def total(get):
            xs = [get(r) for r in rows]
            return sum(xs) if all(x is not None for x in xs) else None

        valu_q = total(lambda r: res[r]["counters"].get("SQ_ACTIVE_INST_VALU"))
        cyc = total(lambda r: res[r]["derived"].get("kernel_cycles"))
        with open(os.path.join(prof, "pmc_k_rows.json"), "w") as f:
            json.dump({"kernel": k, "kernels": rows,
                       "hbm_bytes_per_launch": total(lambda r: res[r]["derived"].get("hbm_bytes")),
                       "hbm_read_bytes_x2_bound": total(lambda r: res[r]["derived"].get("hbm_read_bytes_x2_bound")),
                       "valu_busy": valu_q * 4 / 1024 / cyc if valu_q and cyc else dv.get("valu_busy"),
                       "valu_busy_main": dv.get("valu_busy"),
                       "wave_frac_waiting": dv.get("wave_frac_waiting"),
                       "lds_conflict_frac": dv.get("lds_conflict_frac"),
                       "valu_insts": total(lambda r: res[r]["counters"].get("SQ_INSTS_VALU")),
                       "salu_insts": total(lambda r: res[r]["counters"].get("SQ_INSTS_SALU")),
                       "note": "FETCH_SIZE+WRITE_SIZE KiB x 1024 summed over the step's row kernels "
                               "(one step covers all 10k rows)",
                       "tag": tag}, f, indent=1)
    for k, v in res.items():
        dv = v["derived"]
        print(f"{k:40s} " + " ".join(f"{n}={x:.4g}" for n, x in dv.items()))


if __name__ == "__main__":
    main()
