#!/bin/bash
# the 8-way row-block balance measured on one GPU (tools/gpu/shard_calib.py)
# and a kernel trace of the eight per-rank loads
set -o pipefail
O=gpurun_out/r04e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/gpu/shard_calib.py 10000 8 3 > $O/shard_calib.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o load -- python3 tools/gpu/load_bench.py --genomes 10000 --orient both --reps 1 --parts 8 > $O/prof.log 2>&1 &&
timeout -k 10 300 python -u tools/gpu/load_bench.py --genomes 10000 --orient both --reps 3 > $O/load_both.json 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/proff -o load -- python3 tools/gpu/load_bench.py --genomes 10000 --orient both --reps 3 > $O/proff.log 2>&1
