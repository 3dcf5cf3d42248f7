#!/bin/bash
# Round 5: k_rows_pl variant A/B (PFAAI_PL_V, diagnostics library), 10k all-vs-all.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-r05c}
mkdir -p $OUT
export PFAAI_HIP_LIB=parfastaai_amd/lib/libpfaai_hip_diag.so
timeout -k 10 300 python3 -u tools/gpu/ab_rows.py --genomes 10000 --rounds 7 \
    --variants PFAAI_PL_V=3 PFAAI_PL_V=19 PFAAI_PL_V=27 > $OUT/ab_v.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/gpu/ab_rows.py --genomes 10000 --rounds 7 --rows 0:894 \
    --variants PFAAI_PL_V=3 PFAAI_PL_V=19 PFAAI_PL_V=27 > $OUT/ab_v_narrow.txt 2>&1 || exit 1
