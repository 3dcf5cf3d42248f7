#!/bin/bash
# Round 4: the run-end sort (G_pos + G_end in one F -> G sort) and per-rank
# loads: GPU tests of the load paths and whole-output digests, load timings
# (full and 8-way per rank), the bench line, a kernel-stats profile of the load.
set -o pipefail
mkdir -p gpurun_out/r04b
export PFAAI_PROGRESS=gpurun_out/r04b/progress.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
    tests/test_gpu_load_rows.py tests/test_gpu_load_sort.py tests/test_gpu_configs.py > gpurun_out/r04b/tests.log 2>&1 &&
timeout -k 10 300 python -u tools/gpu/load_bench.py --genomes 10000 --orient both --reps 3 > gpurun_out/r04b/load_both.json 2>&1 &&
timeout -k 10 300 python -u tools/gpu/load_bench.py --genomes 10000 --orient g --reps 3 > gpurun_out/r04b/load_g.json 2>&1 &&
timeout -k 10 300 python -u tools/gpu/load_bench.py --genomes 10000 --orient both --reps 2 --parts 8 > gpurun_out/r04b/load_parts8.json 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline none > gpurun_out/r04b/bench.json 2> gpurun_out/r04b/bench.err &&
export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04b/prof -o load -- python3 tools/gpu/load_bench.py --genomes 10000 --orient both --reps 3 > gpurun_out/r04b/prof.log 2>&1
