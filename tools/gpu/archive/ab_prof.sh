#!/bin/bash
# A/B of k_rows variants (no tests), then a kernel trace of one round.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-ab}
timeout -k 10 600 python tools/gpu/ab_rows.py --genomes 10000 --rounds 4 ${AB_ARGS:---variants PFAAI_ROWS_KERNEL=pl PFAAI_ROWS_KERNEL=pl512} 2>&1 | tail -6 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run -- python3 tools/gpu/ab_rows.py --genomes 10000 --rounds 1 --variants ${PROF_VARIANT:-PFAAI_ROWS_KERNEL=pl} > gpurun_out/prof_$TAG.log 2>&1
rc=$?
python3 - <<PY
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_$TAG/run_kernel_stats.csv")))
for r in rows[:12]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms {int(r['Calls']):4d} calls  avg {float(r['AverageNs'])/1e6:8.3f}  {r['Name'][:100]}")
PY
exit $rc
