#!/bin/bash
# Round 3: SQ / memory counters of the transposition sort kernels (both-given
# load at 10k), one counter group per rocprofv3 pass.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/sortpmc
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" \
           "SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM" "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$PWD/gpurun_out/sortpmc/p$i" -o run \
      -- python3 tools/gpu/load_bench.py --orient both --reps 1 > gpurun_out/sortpmc/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 gpurun_out/sortpmc/p$i.log; exit 1; }
  echo "pass $i done"
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(dict)
for f in sorted(glob.glob("gpurun_out/sortpmc/p*/**/run_counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].replace("void pfaai::", "")[:70]
        acc[n][r["Counter_Name"]] = acc[n].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for n, d in acc.items():
    if "sort" in n or "hash" in n:
        print(n)
        for k in sorted(d):
            print(f"    {k:32s} {d[k]:.4g}")
PY
