#!/bin/bash
# k_blk thread-count A/B: window tables at QT C4 (1024 default vs 256),
# the 10k table (256 default vs 1024); parity of the window path re-run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
echo "== window tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 600 --timeout-method thread > gpurun_out/win_tests.log 2>&1; rc=$?; tail -2 gpurun_out/win_tests.log; [ $rc -eq 0 ] || exit $rc
echo "== qt C4, k_blk<true> 1024 threads"
timeout -k 10 600 python tools/gpu/qt_bench.py > gpurun_out/qt_c4.json 2> gpurun_out/qt_c4.log; rc=$?; cat gpurun_out/qt_c4.json; [ $rc -eq 0 ] || exit $rc
echo "== qt C4, k_blk<true> 256 threads"
PFAAI_BLK_THREADS=256 timeout -k 10 600 python tools/gpu/qt_bench.py > gpurun_out/qt_c4_256.json 2> gpurun_out/qt_c4_256.log; rc=$?; cat gpurun_out/qt_c4_256.json; [ $rc -eq 0 ] || exit $rc
echo "== 10k k_blk 256 vs 1024"
timeout -k 10 300 python tools/gpu/ab_rows.py --genomes 10000 --rounds 3 --variants PFAAI_BLK_THREADS=256 PFAAI_BLK_THREADS=1024 > gpurun_out/ab_blk10k.log 2>&1; rc=$?; tail -3 gpurun_out/ab_blk10k.log; exit $rc
