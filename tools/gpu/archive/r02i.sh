#!/bin/bash
# Round-2 (i): k_blk_end tile A/B, clean 8-way shard times, then the whole GPU suite.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gpu/ab_rows.py --genomes 10000 --rounds 5 --variants PFAAI_BLK_END_TILE=64 \
    PFAAI_BLK_END_TILE=32 PFAAI_BLK_END_TILE=16 PFAAI_BLK_END_TILE=16,PFAAI_BLK_END_U=2 2>&1 | grep -v amdgpu.ids > gpurun_out/ab_blk_end_tile.txt || exit 1
cat gpurun_out/ab_blk_end_tile.txt
SHARD_FRACS=1.0,1.5 timeout -k 10 400 python -u tools/gpu/shard_times.py 10000 8 2>&1 | grep -v amdgpu.ids > gpurun_out/shard_times.txt || exit 1
cat gpurun_out/shard_times.txt
bash tools/gpu/r02_tests.sh
