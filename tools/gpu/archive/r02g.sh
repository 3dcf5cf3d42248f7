#!/bin/bash
# Round-2 (g): the u32 run-end table (k_blk_end) under k_rows_pl WK 3 -- one
# bench line first (k_build / k_rows times vs r02f), then the GPU suite.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline none > gpurun_out/bench_g.log 2>&1 || { tail -20 gpurun_out/bench_g.log; exit 1; }
tail -1 gpurun_out/bench_g.log
bash tools/gpu/r02_tests.sh
