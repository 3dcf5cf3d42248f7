#!/bin/bash
# One profiling session for the round's committed numbers (run under gpurun):
#   1. rocprofv3 PMC passes over one 10k row-kernel run -> profiles/<TAG>_pmc.json
#      and profiles/pmc_k_rows.json (HBM bytes per k_rows_pl launch)
#   2. bench.py at 10k (reads that traffic figure) -> gpurun_out/bench_<TAG>.json
#   3. rocprofv3 --kernel-trace --stats of the same bench command
# Results to copy into profiles/ land under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01v5}
PMC_TAG=pmc_$TAG PMC_SET=${PMC_SET:-full} bash tools/gpu/pmc_pl.sh > gpurun_out/pmc_$TAG.log 2>&1 || { tail -5 gpurun_out/pmc_$TAG.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc_$TAG $TAG > gpurun_out/pmc_summary_$TAG.txt || exit 1
cp profiles/${TAG}_pmc.json profiles/pmc_k_rows.json gpurun_out/
cat gpurun_out/pmc_summary_$TAG.txt
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log || { tail -5 gpurun_out/bench_$TAG.log; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/stats_$TAG" -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline none > gpurun_out/stats_$TAG.log 2>&1 || { tail -5 gpurun_out/stats_$TAG.log; exit 1; }
python3 - <<PY
import csv
for r in list(csv.DictReader(open("gpurun_out/stats_$TAG/run_kernel_stats.csv")))[:8]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms {int(r['Calls']):4d} calls  avg {float(r['AverageNs'])/1e6:8.3f}  {r['Name'][:90]}")
PY
