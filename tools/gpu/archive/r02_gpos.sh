#!/bin/bash
# A/B of the G_pos walk (WK 3) against the line-task form at 10k (diagnostics
# build, results compared bit for bit by ab_rows.py), then the GPU suite and
# one bench line with the release build.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
PFAAI_HIP_LIB=parfastaai_amd/lib/libpfaai_hip_diag.so timeout -k 10 300 python tools/gpu/ab_rows.py --genomes 10000 \
    --rounds 5 --variants PFAAI_ROWS_KERNEL=pl PFAAI_PL_NOGPOS=1 > gpurun_out/ab_gpos.txt 2>&1 || { cat gpurun_out/ab_gpos.txt; exit 1; }
cat gpurun_out/ab_gpos.txt
bash tools/gpu/r02_tests.sh
