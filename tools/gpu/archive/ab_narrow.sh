#!/bin/bash
# A/B of the narrow-row launch (PFAAI_PL_NARROW=0|1|2) over all 10k rows and
# over the last 8-way shard's rows (results compared bit for bit by ab_rows.py).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gpu/ab_rows.py --genomes 10000 --rounds 5 \
    --variants PFAAI_PL_NARROW=0 PFAAI_PL_NARROW=1 PFAAI_PL_NARROW=2 2>&1 | grep -v amdgpu.ids > gpurun_out/ab_narrow_kw1.txt || exit 1
timeout -k 10 300 python -u tools/gpu/ab_rows.py --genomes 10000 --rounds 5 --rows 8358:10000 \
    --variants PFAAI_PL_NARROW=0 PFAAI_PL_NARROW=1 PFAAI_PL_NARROW=2 2>&1 | grep -v amdgpu.ids >> gpurun_out/ab_narrow_kw1.txt || exit 1
timeout -k 10 300 python -u tools/gpu/ab_rows.py --genomes 2000 --rounds 5 \
    --variants PFAAI_PL_NARROW=0 PFAAI_PL_NARROW=1 PFAAI_PL_NARROW=2 2>&1 | grep -v amdgpu.ids >> gpurun_out/ab_narrow_kw1.txt || exit 1
cat gpurun_out/ab_narrow_kw1.txt
