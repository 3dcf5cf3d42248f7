#!/bin/bash
# GPU session: parity tests, then interleaved A/B timing of k_rows variants at 10k.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -15 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/gpu/ab_rows.py --genomes 10000 --rounds 5 ${AB_ARGS:---variants PFAAI_ROWS_OCC=2 PFAAI_ROWS_OCC=3} 2>&1 | tail -6
