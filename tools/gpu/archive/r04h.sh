#!/bin/bash
# the workgroup-model split against the best descent split, timed twice each
set -o pipefail
O=gpurun_out/r04h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/gpu/shard_calib.py 10000 8 0 --cuts "768,1792,2816,3840,5120,6400,7936;908,1866,2879,3901,5165,6421,7952;927,1907,2951,4072,5292,6643,8177" > $O/shard_cuts.txt 2>&1
