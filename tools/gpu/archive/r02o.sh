#!/bin/bash
# Round-2 (o): per-launch width only with G_pos -- C5 streams re-measured,
# the stream / config tests, then the whole suite + bench.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python tools/gpu/stream_bench.py --genomes 40000 > gpurun_out/stream_40k.json 2> gpurun_out/stream_40k.log || { tail -5 gpurun_out/stream_40k.log; exit 1; }
timeout -k 10 900 python tools/gpu/stream_bench.py --genomes 100000 > gpurun_out/stream_100k.json 2> gpurun_out/stream_100k.log || { tail -5 gpurun_out/stream_100k.log; exit 1; }
python -c "
import json
for f in ('gpurun_out/stream_40k.json','gpurun_out/stream_100k.json'):
    d=json.load(open(f)); print(f, d['wall_s'], d['device_ms_rows'], d['device_ms_build'], d['rows_recheck_bit_exact'])"
bash tools/gpu/r02_tests.sh
