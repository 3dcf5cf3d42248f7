#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r04y
timeout -k 10 300 python -u tools/gpu/first_step.py > gpurun_out/r04y/first.json 2>&1 &&
timeout -k 10 300 python -u tools/gpu/first_step.py --busy > gpurun_out/r04y/first_busy.json 2>&1
