#!/bin/bash
# QT 50 000 x 1 000 (C4 shape): base vs new library, alternating processes,
# then the QT-touching GPU tests on the new one.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
: > gpurun_out/ab_qt.txt
for r in 1 2; do
  for lib in parfastaai_amd/lib/ab/libpfaai_hip_base.so parfastaai_amd/lib/libpfaai_hip.so; do
    PFAAI_HIP_LIB=$lib timeout -k 10 300 python tools/gpu/qt_bench.py > gpurun_out/qt.json 2> gpurun_out/qt.log || { tail -5 gpurun_out/qt.log; exit 1; }
    echo "$lib $(python -c "import json; d=json.load(open('gpurun_out/qt.json')); print(d['ms_per_step'], d['k_blk_ms'], d['k_rows_ms'], d['rows_check_vs_oracle_bit_exact'])")" >> gpurun_out/ab_qt.txt
  done
done
cat gpurun_out/ab_qt.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_stream.py tests/test_gpu_parity.py tests/test_gpu_stream_matrix.py -m gpu -x -q --timeout 400 --timeout-method thread 2>&1 | tail -3
