#!/bin/bash
# Column windows: parity (new + full suite), then 10k bench (unchanged path),
# 40k / 100k streaming and QT C4 with windows, and a windows-off A/B at 40k.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
echo "== stream/window tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -x -v --timeout 600 --timeout-method thread > gpurun_out/win_tests.log 2>&1; rc=$?; tail -14 gpurun_out/win_tests.log; [ $rc -eq 0 ] || exit $rc
echo "== gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -4 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
echo "== bench 10k"
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --cpu-baseline none > gpurun_out/bench_10k.json 2> gpurun_out/bench_10k.log; rc=$?; cut -c1-300 gpurun_out/bench_10k.json; [ $rc -eq 0 ] || exit $rc
echo "== ab windows 40k rows 0:4000"
timeout -k 10 300 python tools/gpu/ab_rows.py --genomes 40000 --rows 0:4000 --rounds 2 --variants PFAAI_PL_WINDOWS=1 PFAAI_PL_WINDOWS=0 > gpurun_out/ab_win40k.log 2>&1; rc=$?; tail -3 gpurun_out/ab_win40k.log; [ $rc -eq 0 ] || exit $rc
for n in 40000 100000; do
echo "== stream $n"
timeout -k 10 600 python tools/gpu/stream_bench.py --genomes $n > gpurun_out/stream_$n.json 2> gpurun_out/stream_$n.log; rc=$?; cat gpurun_out/stream_$n.json; [ $rc -eq 0 ] || exit $rc
done
echo "== qt 50000 x 1000"
timeout -k 10 600 python tools/gpu/qt_bench.py > gpurun_out/qt_c4.json 2> gpurun_out/qt_c4.log; rc=$?; cat gpurun_out/qt_c4.json; exit $rc
