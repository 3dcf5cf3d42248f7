#!/bin/bash
# Multi-context paths (CLI --devices, pfaai_compute_rows) + the full GPU suite + smoke.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
echo "== cli + stream tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_cli.py tests/test_gpu_stream.py -x -q --timeout 300 --timeout-method thread > gpurun_out/multi_tests.log 2>&1; rc=$?; tail -15 gpurun_out/multi_tests.log; [ $rc -eq 0 ] || exit $rc
echo "== gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -4 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -1 gpurun_out/smoke.log; exit $rc
