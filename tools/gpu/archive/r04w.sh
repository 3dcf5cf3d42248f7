#!/bin/bash
# wide launch enqueued before the narrow one: first runs after a load, bench,
# the row-kernel tests
set -o pipefail
mkdir -p gpurun_out/r04w
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/gpu/first_step.py > gpurun_out/r04w/first.json 2>&1 &&
timeout -k 10 300 python -u bench.py --cpu-baseline none > gpurun_out/r04w/bench.json 2> gpurun_out/r04w/bench.err &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_load_rows.py tests/test_gpu_group.py > gpurun_out/r04w/tests.log 2>&1
