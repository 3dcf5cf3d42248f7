#!/bin/bash
# Round 5: k_rows_pl variants on the narrow launch alone (512 threads) and on the whole matrix.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-r05j}
mkdir -p $OUT
export PFAAI_HIP_LIB=parfastaai_amd/lib/libpfaai_hip_diag.so
timeout -k 10 300 python3 -u tools/gpu/ab_rows.py --genomes 10000 --rounds 7 --rows 7952:10000 \
    --variants PFAAI_PL_V=0 PFAAI_PL_V=25 PFAAI_PL_V=27 > $OUT/ab_v_narrow.txt 2>&1 || exit 1
