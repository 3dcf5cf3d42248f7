#!/bin/bash
# Round 5: load with the fused member codes, the folded 8-way split emulation, load/config parity.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-r05g}
mkdir -p $OUT
export PFAAI_PROGRESS=$OUT/progress.txt
timeout -k 10 200 python3 -u tools/gpu/load_bench.py --genomes 10000 --orient both --reps 3 > $OUT/load_both.json 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/gpu/load_bench.py --genomes 10000 --orient g --reps 3 > $OUT/load_g.json 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/gpu/shard_fold.py 10000 8 --reps 5 > $OUT/shard_fold.txt 2>&1 || exit 1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_load_rows.py \
   tests/test_gpu_load_sort.py tests/test_gpu_configs.py -k "not c5" > $OUT/tests.txt 2>&1 || exit 1
