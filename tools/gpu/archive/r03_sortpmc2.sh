#!/bin/bash
# Round 3: counters of the transposition sort (both-given load at 10k, the
# release library), one counter group per rocprofv3 pass.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${TAG:-r03i}/pmc
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$PWD/$OUT/p$i" -o run \
      -- python3 tools/gpu/load_bench.py --orient ${ORIENT:-both} --reps 1 > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 $OUT/p$i.log; exit 1; }
  echo "pass $i done"
done
python3 - $OUT <<'PY'
import csv, glob, collections, sys
acc = collections.defaultdict(dict)
for f in sorted(glob.glob(sys.argv[1] + "/p*/**/run_counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].replace("void pfaai::", "")[:70]
        acc[n][r["Counter_Name"]] = acc[n].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for n, d in acc.items():
    if "sort" in n or "gend" in n or "hash" in n:
        print(n)
        for k in sorted(d):
            print(f"    {k:36s} {d[k]:.4g}")
PY
