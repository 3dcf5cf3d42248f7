#!/bin/bash
# Round-2 (j): C4 (QT 50 000 x 1 000) and C5 (100k streamed) re-measured on
# the round-2 kernels, and a 1-GPU bench line of the new bench.py.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline none > gpurun_out/bench_j.json 2> gpurun_out/bench_j.log || { tail -5 gpurun_out/bench_j.log; exit 1; }
cat gpurun_out/bench_j.json
timeout -k 10 600 python tools/gpu/qt_bench.py > gpurun_out/qt_c4.json 2> gpurun_out/qt_c4.log || { tail -5 gpurun_out/qt_c4.log; exit 1; }
cat gpurun_out/qt_c4.json
timeout -k 10 600 python tools/gpu/stream_bench.py --genomes 40000 > gpurun_out/stream_40k.json 2> gpurun_out/stream_40k.log || { tail -5 gpurun_out/stream_40k.log; exit 1; }
cat gpurun_out/stream_40k.json
timeout -k 10 900 python tools/gpu/stream_bench.py --genomes 100000 > gpurun_out/stream_100k.json 2> gpurun_out/stream_100k.log || { tail -5 gpurun_out/stream_100k.log; exit 1; }
cat gpurun_out/stream_100k.json
