"""Print per-kernel PMC counters from tools/gpu/pmc_pl.sh output dirs.

    python tools/gpu/pmc_cmp.py gpurun_out/pmc13 [gpurun_out/pmc12 ...]
"""
import collections
import csv
import glob
import os
import sys

for d in sys.argv[1:]:
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
            acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
    print(f"== {d}")
    for k, cs in acc.items():
        if "fill" in k or "copy" in k:
            continue
        print(f"  {k}")
        for c, v in sorted(cs.items()):
            print(f"      {c:42s} {v:16.4g}")
