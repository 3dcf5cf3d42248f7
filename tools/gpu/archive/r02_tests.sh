#!/bin/bash
# Round-2 GPU check: the whole -m gpu suite (progress of the long config
# tests in gpurun_out/progress.log), then one short bench line.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export PFAAI_PROGRESS=gpurun_out/progress.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rf --timeout 600 --timeout-method thread \
    "$@" > gpurun_out/pytest.log 2>&1
rc=$?
tail -5 gpurun_out/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
exit $rc
