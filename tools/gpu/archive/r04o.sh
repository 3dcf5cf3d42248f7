#!/bin/bash
# the whole GPU suite, load timings + trace, the default bench line
set -o pipefail
O=gpurun_out/r04o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/gpu/load_bench.py --genomes 10000 --orient both --reps 3 > $O/load_both.json 2>&1 &&
timeout -k 10 300 python -u tools/gpu/load_bench.py --genomes 10000 --orient both --reps 2 --parts 8 > $O/load_parts8.json 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o load -- python3 tools/gpu/load_bench.py --genomes 10000 --orient both --reps 3 > $O/prof.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof8 -o load -- python3 tools/gpu/load_bench.py --genomes 10000 --orient both --reps 1 --parts 8 > $O/prof8.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
