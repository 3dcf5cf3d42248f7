#!/bin/bash
# load tests, full and per-rank load timings, candidate 8-way splits
set -o pipefail
O=gpurun_out/r04g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_load_rows.py tests/test_gpu_load_sort.py "tests/test_gpu_configs.py::test_c2_whole_output" \
    "tests/test_gpu_configs.py::test_c3_10k_all_vs_all_and_8way_rowblocks" > $O/tests.log 2>&1 &&
timeout -k 10 300 python -u tools/gpu/load_bench.py --genomes 10000 --orient both --reps 3 > $O/load_both.json 2>&1 &&
timeout -k 10 300 python -u tools/gpu/load_bench.py --genomes 10000 --orient both --reps 2 --parts 8 > $O/load_parts8.json 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o load -- python3 tools/gpu/load_bench.py --genomes 10000 --orient both --reps 1 --parts 8 > $O/prof.log 2>&1 &&
timeout -k 10 600 python -u tools/gpu/shard_calib.py 10000 8 0 --cuts "927,1907,2951,4072,5292,6643,8177;908,1866,2879,3901,5165,6421,7952;908,1866,2823,3901,5141,6485,7952;900,1800,2750,3850,5100,6450,7952" > $O/shard_cuts.txt 2>&1
