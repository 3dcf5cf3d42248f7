#!/bin/bash
# Round 3 profile set: k_rows_pl PMC passes (HBM traffic, SQ counters, VALU
# busy) -> profiles/<TAG>_pmc.json + pmc_k_rows.json, and the 8-way shard
# times of the row kernel on one GPU (cost-model split).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp GRAFT_REPO_ROOT=${GRAFT_REPO_ROOT:-$PWD}
TAG=${TAG:-r03c}
PMC_TAG=pmc_$TAG PMC_SET=full bash tools/gpu/pmc_pl.sh > gpurun_out/pmc_$TAG.log 2>&1 || { tail -5 gpurun_out/pmc_$TAG.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc_$TAG $TAG > gpurun_out/pmc_summary_$TAG.txt || exit 1
cp profiles/${TAG}_pmc.json profiles/pmc_k_rows.json gpurun_out/
cat gpurun_out/pmc_summary_$TAG.txt
SHARD_FRACS=${SHARD_FRACS:-0.75,1.25} timeout -k 10 600 python3 tools/gpu/shard_times.py 10000 8 > gpurun_out/shard_times_$TAG.txt 2>&1 || { tail -5 gpurun_out/shard_times_$TAG.txt; exit 1; }
cat gpurun_out/shard_times_$TAG.txt
