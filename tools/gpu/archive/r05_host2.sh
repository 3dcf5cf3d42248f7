#!/bin/bash
# Round 5: the load-check tests and the CLI at C2 with the library's compute phase trace.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-r05s}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_load_sort.py tests/test_gpu_load_rows.py tests/test_gpu_kernels.py > $OUT/tests.txt 2>&1 || exit 1
PFAAI_TRACE_COMPUTE=1 timeout -k 10 400 python3 -u tools/gpu/e2e_c2.py --repeats 3 --skip-ref > $OUT/e2e_c2_noref.json 2> $OUT/e2e.err || exit 1
