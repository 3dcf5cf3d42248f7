#!/bin/bash
# A/B of two builds of the library by whole bench runs, interleaved:
#   BASE=parfastaai_amd/lib/libpfaai_hip_abbase.so TAG=x bash tools/gpu/ab_lib.sh
# (the candidate is CAND, by default the in-tree libpfaai_hip.so).  Prints ms_per_step and the
# row-kernel time of every run.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${TAG:-ab_lib}
mkdir -p $OUT
BASE=${BASE:-parfastaai_amd/lib/libpfaai_hip_abbase.so}
for r in ${ROUNDS:-1 2 3}; do
  for v in base cand; do
    lib=${CAND:-parfastaai_amd/lib/libpfaai_hip.so}
    [ $v = base ] && lib=$BASE
    PFAAI_HIP_LIB=$PWD/$lib timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --cpu-baseline none \
        > $OUT/bench_${v}_$r.json 2> $OUT/bench_${v}_$r.log || { tail -5 $OUT/bench_${v}_$r.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['roofline']['kernel_ms'])" \
        $OUT/bench_${v}_$r.json $v
  done
done
