#!/bin/bash
# Round-3 GPU check: the -m gpu suite, then bench.py's self-spawned N > 1
# flow rehearsed on the one GPU (gloo), then one short bench line.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export PFAAI_PROGRESS=gpurun_out/progress.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -rf --timeout 600 --timeout-method thread \
    "$@" > gpurun_out/pytest.log 2>&1
rc=$?
tail -5 gpurun_out/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --gpus 2 --steps 3 --warmup 1 --rehearse-gloo --cpu-baseline none \
    > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.log || { tail -30 gpurun_out/rehearse2.log; exit 1; }
cat gpurun_out/rehearse2.json; grep -E "bit-exact|communicator" gpurun_out/rehearse2.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline none > gpurun_out/bench.json 2> gpurun_out/bench.log || { tail -5 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.json
