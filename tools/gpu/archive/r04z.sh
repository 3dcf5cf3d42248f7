#!/bin/bash
# round-4 close: smoke, the profile set of the bench command (one build:
# bench line, kernel stats with median / min, PMC passes), C2 end to end
set -o pipefail
mkdir -p gpurun_out/r04z
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04z/smoke.log 2>&1 &&
PROF_TAG=r04z bash tools/gpu/profile_bench.sh > gpurun_out/r04z/profile.log 2>&1 &&
timeout -k 10 900 python -u tools/gpu/e2e_c2.py --repeats 3 > gpurun_out/r04z/e2e_c2.json 2> gpurun_out/r04z/e2e_c2.log
