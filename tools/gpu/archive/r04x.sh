#!/bin/bash
# counters per row-kernel dispatch of the first runs after a load (cold start)
set -o pipefail
mkdir -p gpurun_out/r04x
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/r04x/p1 -o run -- python3 tools/gpu/first_step.py > gpurun_out/r04x/p1.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/r04x/p2 -o run -- python3 tools/gpu/first_step.py > gpurun_out/r04x/p2.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d gpurun_out/r04x/p3 -o run -- python3 tools/gpu/first_step.py > gpurun_out/r04x/p3.log 2>&1
