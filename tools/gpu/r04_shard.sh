#!/bin/bash
# the 8-way row-block balance measured on one GPU (tools/gpu/shard_calib.py)
set -o pipefail
mkdir -p gpurun_out/r04d
timeout -k 10 600 python -u tools/gpu/shard_calib.py 10000 8 3 > gpurun_out/r04d/shard_calib.txt 2>&1
