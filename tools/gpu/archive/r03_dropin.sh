#!/bin/bash
# Round 3: the reference-side drop-in binary's GPU tests, the CLI tests, the
# release-library switch test, then the C2 end-to-end comparison (medians of
# 3 runs of ours, the drop-in and the reference at usable-CPU threads).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_cli.py tests/test_gpu_kernels.py -x -v -rf \
    --timeout 300 --timeout-method thread > gpurun_out/pytest_dropin.log 2>&1 || { tail -30 gpurun_out/pytest_dropin.log; exit 1; }
tail -3 gpurun_out/pytest_dropin.log
timeout -k 10 900 python -u tools/gpu/e2e_c2.py --repeats ${REPEATS:-3} > gpurun_out/e2e_c2.json 2> gpurun_out/e2e_c2.log || { tail -20 gpurun_out/e2e_c2.log; exit 1; }
cat gpurun_out/e2e_c2.json
