#!/bin/bash
# the load paths' tests (sort, per-rank, whole-output digests at C2 / C3),
# load timings (full both-given, G only, 8-way per rank) and kernel traces
set -o pipefail
mkdir -p gpurun_out/r04c
export TMPDIR=/tmp
export PFAAI_PROGRESS=gpurun_out/r04c/progress.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_load_rows.py tests/test_gpu_load_sort.py "tests/test_gpu_configs.py::test_c2_whole_output" \
    "tests/test_gpu_configs.py::test_c3_10k_all_vs_all_and_8way_rowblocks" > gpurun_out/r04c/tests.log 2>&1 &&
timeout -k 10 300 python -u tools/gpu/load_bench.py --genomes 10000 --orient both --reps 3 > gpurun_out/r04c/load_both.json 2>&1 &&
timeout -k 10 300 python -u tools/gpu/load_bench.py --genomes 10000 --orient both --reps 2 --parts 8 > gpurun_out/r04c/load_parts8.json 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04c/prof -o load -- python3 tools/gpu/load_bench.py --genomes 10000 --orient both --reps 3 > gpurun_out/r04c/prof.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04c/profg -o load -- python3 tools/gpu/load_bench.py --genomes 10000 --orient g --reps 3 > gpurun_out/r04c/profg.log 2>&1
