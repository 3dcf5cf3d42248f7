#!/bin/bash
# round-4 refresh of the secondary numbers: C2 end to end (ours / drop-in /
# reference, medians of 3, CSV byte-identical), 50 000 x 1 000 QT, 100k
# all-vs-all streamed to host memory
set -o pipefail
O=gpurun_out/r04p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/gpu/e2e_c2.py --repeats 3 > $O/e2e_c2.json 2> $O/e2e_c2.log &&
timeout -k 10 300 python -u tools/gpu/qt_bench.py --targets 50000 --queries 1000 > $O/qt_50k.json 2> $O/qt_50k.log &&
timeout -k 10 600 python -u tools/gpu/stream_bench.py --genomes 100000 --tile-pairs 268435456 > $O/stream_100k.json 2> $O/stream_100k.log
