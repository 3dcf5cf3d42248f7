#!/bin/bash
# first run after a load vs the next ones, then the round's profile set
set -o pipefail
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 300 python -u tools/gpu/first_step.py > $O/first.json 2>&1 &&
PROF_TAG=r04k bash tools/gpu/profile_bench.sh
