#!/bin/bash
set -o pipefail
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 300 python -u tools/gpu/first_step.py > $O/first.json 2>&1 &&
HIP_ENABLE_DEFERRED_LOADING=0 timeout -k 10 300 python -u tools/gpu/first_step.py > $O/first_nodefer.json 2>&1
