#!/bin/bash
# GPU session: parity tests, then a rocprofv3 kernel trace of the 10k bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-r01}
echo "== gpu tests"
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -25 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
echo "== rocprof kernel trace (10k bench)"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline none > gpurun_out/prof_bench.log 2>&1
rc=$?; tail -3 gpurun_out/prof_bench.log; exit $rc
