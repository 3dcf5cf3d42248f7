#!/bin/bash
# the group API (RCCL communicator, one rank on this box) + the ABI tests
set -o pipefail
O=gpurun_out/r04q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_group.py tests/test_gpu_load_rows.py > $O/tests.log 2>&1
