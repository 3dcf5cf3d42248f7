#!/bin/bash
# Round 5: host paths -- the GPU suite (SUITE=1) or the kernel tests, the CLI at C2 (ours + drop-in, no
# reference runs), C5 streaming sinks.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-r05l}
mkdir -p $OUT
if [ -n "$SUITE" ]; then
  timeout -k 10 420 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $OUT/tests.txt 2>&1 || exit 1
else
  timeout -k 10 200 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_kernels.py > $OUT/tests_kernels.txt 2>&1 || exit 1
fi
timeout -k 10 400 python3 -u tools/gpu/e2e_c2.py --repeats 3 --skip-ref > $OUT/e2e_c2_noref.json 2> $OUT/e2e.err || exit 1
[ -n "$NOSTREAM" ] && exit 0
timeout -k 10 500 python3 -u tools/gpu/stream_bench.py --genomes 100000 --sinks noop copy par > $OUT/stream_100k.json 2> $OUT/stream.err || exit 1
