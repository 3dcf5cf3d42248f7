#!/bin/bash
# Round 5: S5 bits on the column-window form (40k all-vs-all, BIGF), then the suite + bench + smoke.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-r05k}
mkdir -p $OUT
PFAAI_HIP_LIB=parfastaai_amd/lib/libpfaai_hip_diag.so timeout -k 10 300 python3 -u tools/gpu/ab_rows.py --genomes 40000 --rounds 3 \
    --variants PFAAI_PL_VG=0 PFAAI_PL_VG=9 > $OUT/ab_vg_40k.txt 2>&1 || exit 1
TAG=${TAG:-r05k} bash tools/gpu/r05_suite.sh
