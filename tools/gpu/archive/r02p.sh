#!/bin/bash
# Round-2 (p): S5 skip in WK 3 only -- C4 / C5 re-measured, bench, suite.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python tools/gpu/qt_bench.py > gpurun_out/qt_c4.json 2> gpurun_out/qt_c4.log || { tail -5 gpurun_out/qt_c4.log; exit 1; }
timeout -k 10 600 python tools/gpu/stream_bench.py --genomes 40000 > gpurun_out/stream_40k.json 2> gpurun_out/stream_40k.log || { tail -5 gpurun_out/stream_40k.log; exit 1; }
timeout -k 10 900 python tools/gpu/stream_bench.py --genomes 100000 > gpurun_out/stream_100k.json 2> gpurun_out/stream_100k.log || { tail -5 gpurun_out/stream_100k.log; exit 1; }
python -c "
import json
d=json.load(open('gpurun_out/qt_c4.json')); print('qt', d['ms_per_step'], d['k_blk_ms'], d['k_rows_ms'], d['rows_check_vs_oracle_bit_exact'])
for f in ('gpurun_out/stream_40k.json','gpurun_out/stream_100k.json'):
    d=json.load(open(f)); print(f, d['wall_s'], d['device_ms_rows'], d['device_ms_build'], d['rows_recheck_bit_exact'])"
bash tools/gpu/r02_tests.sh
