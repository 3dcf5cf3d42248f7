#!/bin/bash
# GPU session: parity tests, then interleaved A/B of row-kernel variants at 10k.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -15 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/gpu/ab_rows.py --genomes ${AB_GENOMES:-10000} --rounds 3 --variants ${AB_VARIANTS:-PFAAI_ROWS_KERNEL=pl PFAAI_ROWS_KERNEL=pl512} 2>&1 | tail -8
