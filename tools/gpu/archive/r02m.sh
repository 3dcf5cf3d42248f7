#!/bin/bash
# Round-2 (m): KW per launch from the launch's widest all-vs-all row --
# 8-way shard times with and without it, then the whole GPU suite + bench.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
SHARD_FRACS=1.0,1.5 timeout -k 10 400 python -u tools/gpu/shard_times.py 10000 8 2>&1 | grep -v amdgpu.ids > gpurun_out/shard_times_m.txt || exit 1
PFAAI_PL_LAUNCH_COLS=0 timeout -k 10 400 python -u tools/gpu/shard_times.py 10000 8 2>&1 | grep -v amdgpu.ids > gpurun_out/shard_times_m0.txt || exit 1
echo "== KW per launch"; head -8 gpurun_out/shard_times_m.txt | cut -c1-200
echo "== problem KW"; head -6 gpurun_out/shard_times_m0.txt | cut -c1-200
bash tools/gpu/r02_tests.sh
