#!/bin/bash
# Round 5: traced host copies -- the CLI at C2 and the bench's load (PFAAI_TRACE_COMPUTE=1: per-copy lines).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-r05u}
mkdir -p $OUT
export PFAAI_TRACE_COMPUTE=1
timeout -k 10 400 python3 -u tools/gpu/e2e_c2.py --repeats 3 --skip-ref > $OUT/e2e_c2_noref.json 2> $OUT/e2e.err || exit 1
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --cpu-baseline none > $OUT/bench.json 2> $OUT/bench.err || exit 1
