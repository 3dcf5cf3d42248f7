#!/bin/bash
# Round 3: the load-time transposition sort -- its tests, the orientation
# and parity suites, the bench line (load object), and a rocprofv3 kernel
# trace of the bench (load kernels + step kernels).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_load_sort.py tests/test_gpu_orientations.py tests/test_gpu_build_f.py \
    tests/test_gpu_load_errors.py tests/test_gpu_parity.py tests/test_gpu_edges.py -x -v -rf --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_sort.log 2>&1 || { tail -40 gpurun_out/pytest_sort.log; exit 1; }
tail -3 gpurun_out/pytest_sort.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline none > gpurun_out/bench_sort.json 2> gpurun_out/bench_sort.log || { tail -5 gpurun_out/bench_sort.log; exit 1; }
cat gpurun_out/bench_sort.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/stats_sort" -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline none > gpurun_out/stats_sort.log 2>&1 || { tail -5 gpurun_out/stats_sort.log; exit 1; }
python3 - <<PY
import csv, glob
f = glob.glob("gpurun_out/stats_sort/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:16]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms {int(r['Calls']):4d} calls  avg {float(r['AverageNs'])/1e6:8.3f}  {r['Name'][:100]}")
PY
