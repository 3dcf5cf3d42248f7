#!/bin/bash
# GPU session: new parity tests (streaming, KEEP_RUNS, |F| > 2^30), the full
# GPU suite, the 10k bench, then output-tile streaming at 40k and 100k.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
echo "== stream tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -x -v --timeout 600 --timeout-method thread > gpurun_out/stream_tests.log 2>&1; rc=$?; tail -12 gpurun_out/stream_tests.log; [ $rc -eq 0 ] || exit $rc
echo "== gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -5 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
echo "== bench 10k"
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --cpu-baseline none > gpurun_out/bench_10k.json 2> gpurun_out/bench_10k.log; rc=$?; cat gpurun_out/bench_10k.json; [ $rc -eq 0 ] || exit $rc
echo "== bench 10k, BIGF row kernel forced (A/B)"
PFAAI_PL_BIGF=1 timeout -k 10 600 python bench.py --steps 10 --warmup 3 --cpu-baseline none > gpurun_out/bench_10k_bigf.json 2> gpurun_out/bench_10k_bigf.log; rc=$?; cut -c1-400 gpurun_out/bench_10k_bigf.json; [ $rc -eq 0 ] || exit $rc
echo "== stream 40k"
timeout -k 10 600 python tools/gpu/stream_bench.py --genomes 40000 > gpurun_out/stream_40k.json 2> gpurun_out/stream_40k.log; rc=$?; tail -3 gpurun_out/stream_40k.log; cat gpurun_out/stream_40k.json; [ $rc -eq 0 ] || exit $rc
echo "== stream 100k"
timeout -k 10 900 python tools/gpu/stream_bench.py --genomes 100000 > gpurun_out/stream_100k.json 2> gpurun_out/stream_100k.log; rc=$?; tail -3 gpurun_out/stream_100k.log; cat gpurun_out/stream_100k.json; exit $rc
