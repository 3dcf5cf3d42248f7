#!/bin/bash
# Round 5 A/B (diagnostics library): the upload's slot -> device step by DMA or by the copy kernel, and
# staged uploads above 512 MB or not; the bench's load times and first step (does a busy GPU during the
# upload keep the shader clock up for the load and the first step?).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-r05h}
mkdir -p $OUT
export PFAAI_HIP_LIB=$PWD/parfastaai_amd/lib/libpfaai_hip_diag.so
for rep in 1 2; do
for v in "" "PFAAI_H2D_KERNEL=1" "PFAAI_H2D_ALL=1" "PFAAI_H2D_KERNEL=1 PFAAI_H2D_ALL=1"; do
  echo "== $v rep $rep" >> $OUT/ab.txt
  env $v timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --cpu-baseline none > $OUT/b.json 2> $OUT/b.err || exit 1
  python3 -c "import json; d=json.load(open('$OUT/b.json')); l=d['load']; print('h2d', l['h2d_ms'], 'dev', l['device_ms'], 'first', l['first_step_ms'], 'one_shot', l['one_shot_ms'], 'step', d['ms_per_step'])" >> $OUT/ab.txt
done
done
