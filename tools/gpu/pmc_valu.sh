#!/bin/bash
# SQ instruction counters of k_rows_pl for two row-kernel variants (diagnostics
# library), one rocprofv3 --pmc pass each: does a change cut VALU / SALU / LDS
# instructions, and by how much.   usage: pmc_valu.sh VARIANT_ENV...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc_valu
export TMPDIR=/tmp PFAAI_HIP_LIB=parfastaai_amd/lib/libpfaai_hip_diag.so
i=0
for v in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES \
      --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_valu/v$i" -o run -- \
      python3 tools/gpu/ab_rows.py --genomes 10000 --rounds 0 --variants "$v" > gpurun_out/pmc_valu/v$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/pmc_valu/v$i.log; exit 1; }
  python3 - "$v" "gpurun_out/pmc_valu/v$i/run_counter_collection.csv" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[2])):
    if "k_rows_pl" in r["Kernel_Name"]:
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
print(sys.argv[1], " ".join(f"{k}={v:.4g}" for k, v in sorted(acc.items())))
PY
done
