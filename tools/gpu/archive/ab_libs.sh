#!/bin/bash
# Interleaved A/B of two builds of libpfaai_hip.so (processes alternate,
# 3 x 3 row-kernel runs each at 10k): base = parfastaai_amd/lib/ab/libpfaai_hip_base.so,
# new = parfastaai_amd/lib/libpfaai_hip.so.  Then env A/Bs on the new build.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
out=gpurun_out/ab_libs.txt
: > $out
for r in 1 2 3; do
  for lib in parfastaai_amd/lib/ab/libpfaai_hip_base.so parfastaai_amd/lib/libpfaai_hip.so; do
    echo "== $lib" >> $out
    PFAAI_HIP_LIB=$lib timeout -k 10 120 python -u tools/gpu/ab_rows.py --genomes 10000 --rounds 3 \
      --variants PFAAI_ROWS_KERNEL=pl 2>&1 | grep -v amdgpu.ids >> $out || exit 1
  done
done
cat $out
for v in "${@}"; do
  timeout -k 10 300 python -u tools/gpu/ab_rows.py --genomes 10000 --rounds 5 --variants $v 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ab_env.txt || exit 1
done
