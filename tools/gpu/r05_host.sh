#!/bin/bash
# Round 5: host paths -- the CLI at C2 (ours + drop-in, no reference runs), C5 streaming sinks, div check.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-r05l}
mkdir -p $OUT
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_kernels.py > $OUT/tests_kernels.txt 2>&1 || exit 1
timeout -k 10 400 python3 -u tools/gpu/e2e_c2.py --repeats 3 --skip-ref > $OUT/e2e_c2_noref.json 2> $OUT/e2e.err || exit 1
timeout -k 10 500 python3 -u tools/gpu/stream_bench.py --genomes 100000 --sinks noop copy par > $OUT/stream_100k.json 2> $OUT/stream.err || exit 1
