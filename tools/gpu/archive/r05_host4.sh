#!/bin/bash
# Round 5: the GPU suite, then the traced CLI at C2 (PFAAI_TRACE_COMPUTE=1) and a short bench.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-r05x}
mkdir -p $OUT
timeout -k 10 420 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $OUT/tests.txt 2>&1 || exit 1
PFAAI_TRACE_COMPUTE=1 timeout -k 10 400 python3 -u tools/gpu/e2e_c2.py --repeats 3 --skip-ref > $OUT/e2e_c2_noref.json 2> $OUT/e2e.err || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-baseline none > $OUT/bench.json 2> $OUT/bench.err || exit 1
