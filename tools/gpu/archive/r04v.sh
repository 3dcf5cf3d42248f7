#!/bin/bash
# the final tree: GPU suite and smoke
set -o pipefail
mkdir -p gpurun_out/r04v
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r04v/tests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04v/smoke.log 2>&1
