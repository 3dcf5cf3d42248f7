#!/bin/bash
# the whole GPU suite, the default bench line, the shipped 8-way split timed
set -o pipefail
O=gpurun_out/r04i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 600 python -u tools/gpu/shard_calib.py 10000 8 0 --cuts "894,1841,2851,3875,5132,6460,7988;908,1866,2879,3901,5165,6421,7952" > $O/shard_cuts.txt 2>&1
