#!/bin/bash
# Round 4: whole-output digests (C2/C3/C4), the CLI (G_pos on the G-only load,
# exact orientation check, C2 CSV vs the reference's digest), one bench line.
set -o pipefail
mkdir -p gpurun_out/r04
export PFAAI_PROGRESS=gpurun_out/r04/progress.txt
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
    tests/test_gpu_configs.py tests/test_gpu_cli.py > gpurun_out/r04/tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline none > gpurun_out/r04/bench.json 2> gpurun_out/r04/bench.err
