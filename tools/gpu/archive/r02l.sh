#!/bin/bash
# Round-2 (l): smoke, the whole GPU suite + a bench line, then the C2
# end-to-end drop-in check against the reference CLI.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
bash tools/gpu/r02_tests.sh || exit $?
timeout -k 10 700 python -u tools/gpu/e2e_c2.py > gpurun_out/e2e_c2.json 2> gpurun_out/e2e_c2.log || { tail -5 gpurun_out/e2e_c2.log; exit 1; }
cat gpurun_out/e2e_c2.json
