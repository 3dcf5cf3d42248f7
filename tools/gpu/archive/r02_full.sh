#!/bin/bash
# Round-2 GPU pass: the whole -m gpu suite, the C2 end-to-end CLI run vs the
# reference binary, one bench line.  Logs under gpurun_out/.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export PFAAI_PROGRESS=gpurun_out/progress.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rf --timeout 600 --timeout-method thread \
    > gpurun_out/pytest.log 2>&1
rc=$?
tail -4 gpurun_out/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
if [ "${SKIP_E2E:-0}" != 1 ]; then
    timeout -k 10 400 python -u tools/gpu/e2e_c2.py > gpurun_out/e2e_c2.json 2> gpurun_out/e2e_c2.log || exit $?
    cat gpurun_out/e2e_c2.json
fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
exit $rc
