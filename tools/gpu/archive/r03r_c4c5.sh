#!/bin/bash
# Round 3: configs C4 (QT 50 000 x 1 000) and C5 (100k streamed), 40k streamed.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${TAG:-r03r}
mkdir -p $OUT
timeout -k 10 600 python tools/gpu/qt_bench.py > $OUT/qt_c4.json 2> $OUT/qt_c4.log || { tail -5 $OUT/qt_c4.log; exit 1; }
cat $OUT/qt_c4.json
timeout -k 10 600 python tools/gpu/stream_bench.py --genomes 40000 > $OUT/stream_40k.json 2> $OUT/stream_40k.log || { tail -5 $OUT/stream_40k.log; exit 1; }
cat $OUT/stream_40k.json
timeout -k 10 900 python tools/gpu/stream_bench.py --genomes 100000 > $OUT/stream_100k.json 2> $OUT/stream_100k.log || { tail -5 $OUT/stream_100k.log; exit 1; }
cat $OUT/stream_100k.json
