#!/bin/bash
# candidate 8-way splits timed twice each (tools/gpu/shard_calib.py --cuts)
set -o pipefail
O=gpurun_out/r04f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/gpu/shard_calib.py 10000 8 0 --cuts "927,1907,2951,4072,5292,6643,8177;908,1866,2879,3901,5165,6421,7952;908,1866,2823,3901,5141,6485,7952;900,1800,2750,3850,5100,6450,7952" > $O/shard_cuts.txt 2>&1
