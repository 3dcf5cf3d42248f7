#!/bin/bash
set -o pipefail
O=gpurun_out/r04u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_load_rows.py tests/test_gpu_load_sort.py "tests/test_gpu_configs.py::test_c2_whole_output" > $O/tests.log 2>&1 &&
timeout -k 10 300 python -u tools/gpu/load_bench.py --genomes 10000 --orient both --reps 5 > $O/load_both.json 2>&1 &&
timeout -k 10 300 python -u tools/gpu/load_bench.py --genomes 10000 --orient both --reps 2 --parts 8 > $O/load_parts8.json 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o load -- python3 tools/gpu/load_bench.py --genomes 10000 --orient both --reps 3 > $O/prof.log 2>&1
