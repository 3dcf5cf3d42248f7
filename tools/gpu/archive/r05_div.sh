#!/bin/bash
# Round 5: S5 reciprocal-table A/B (diagnostics library) + kernel parity tests.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-r05b}
mkdir -p $OUT
export PFAAI_HIP_LIB=parfastaai_amd/lib/libpfaai_hip_diag.so
timeout -k 10 240 python3 -u tools/gpu/ab_rows.py --genomes 10000 --rounds 5 --rows 1808:7952 \
    --variants PFAAI_PL_DIV=0 PFAAI_PL_DIV=1 PFAAI_PL_DIV=2 > $OUT/ab_div_kw4.txt 2>&1 || exit 1
timeout -k 10 240 python3 -u tools/gpu/ab_rows.py --genomes 10000 --rounds 5 \
    --variants PFAAI_PL_DIV=0 PFAAI_PL_DIV=1,PFAAI_PL_NK2=1 PFAAI_PL_DIV=1 > $OUT/ab_div_all.txt 2>&1 || exit 1
unset PFAAI_HIP_LIB
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity.py \
    tests/test_gpu_edges.py > $OUT/tests.txt 2>&1 || exit 1
