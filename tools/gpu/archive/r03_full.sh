#!/bin/bash
# Round 3: the whole -m gpu suite, then the bench line and its kernel trace.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp PFAAI_PROGRESS=gpurun_out/progress.log
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -rf --timeout 600 --timeout-method thread \
    > gpurun_out/pytest_full.log 2>&1 || { tail -40 gpurun_out/pytest_full.log; exit 1; }
tail -3 gpurun_out/pytest_full.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline none > gpurun_out/bench_full.json 2> gpurun_out/bench_full.log || { tail -5 gpurun_out/bench_full.log; exit 1; }
cat gpurun_out/bench_full.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/stats_full" -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline none > gpurun_out/stats_full.log 2>&1 || { tail -5 gpurun_out/stats_full.log; exit 1; }
python3 - <<PY
import csv, glob
f = glob.glob("gpurun_out/stats_full/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms {int(r['Calls']):4d} calls  avg {float(r['AverageNs'])/1e6:8.3f}  {r['Name'][:100]}")
PY
