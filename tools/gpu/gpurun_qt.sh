#!/bin/bash
# QT (config C4 shape) on one GPU, small then full; shard/chunk timing at 10k.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
echo "== qt small"
timeout -k 10 300 python tools/gpu/qt_bench.py --targets 600 --queries 40 --prot 30 > gpurun_out/qt_small.json 2> gpurun_out/qt_small.log; rc=$?; tail -3 gpurun_out/qt_small.log; cat gpurun_out/qt_small.json; [ $rc -eq 0 ] || exit $rc
echo "== qt 50000 x 1000"
timeout -k 10 600 python tools/gpu/qt_bench.py > gpurun_out/qt_c4.json 2> gpurun_out/qt_c4.log; rc=$?; tail -3 gpurun_out/qt_c4.log; cat gpurun_out/qt_c4.json; [ $rc -eq 0 ] || exit $rc
echo "== shard / chunk times 10k x 8"
timeout -k 10 300 python tools/gpu/shard_times.py 10000 8 > gpurun_out/shard_times.log 2>&1; rc=$?; tail -8 gpurun_out/shard_times.log; exit $rc
