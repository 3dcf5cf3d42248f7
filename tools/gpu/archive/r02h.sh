#!/bin/bash
# Round-2 (h): narrow all-vs-all rows as 512-thread workgroups -- interleaved
# A/B (bit-equal asserted) over all rows and over the last 8-way shard, the
# shard times, then the all-vs-all parity tests.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gpu/ab_rows.py --genomes 10000 --rounds 5 \
    --variants PFAAI_PL_NARROW=0 PFAAI_PL_NARROW=1 > gpurun_out/ab_narrow.txt 2>&1 || { cat gpurun_out/ab_narrow.txt; exit 1; }
cat gpurun_out/ab_narrow.txt
timeout -k 10 300 python -u tools/gpu/ab_rows.py --genomes 10000 --rounds 5 --rows 8358:10000 \
    --variants PFAAI_PL_NARROW=0 PFAAI_PL_NARROW=1 > gpurun_out/ab_narrow_shard7.txt 2>&1 || { cat gpurun_out/ab_narrow_shard7.txt; exit 1; }
cat gpurun_out/ab_narrow_shard7.txt
SHARD_FRACS=1.0,1.5,2.0 timeout -k 10 400 python -u tools/gpu/shard_times.py 10000 8 > gpurun_out/shard_times.txt 2>&1 || { cat gpurun_out/shard_times.txt; exit 1; }
cat gpurun_out/shard_times.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_cli.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/pytest_h.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_h.log
exit $rc
