#!/bin/bash
# rocprofv3 kernel stats + PMC passes (one counter group per pass) for the
# C4 (query vs target, tools/gpu/qt_bench.py) or C5 (100k streamed,
# tools/gpu/stream_bench.py) workload -- VERDICT r05 #1's evidence set.
#   WHICH=c4 TAG=r06g bash tools/gpu/profile_c4c5.sh   (then tools/pmc_summary.py <out>/pmc <tag>_c4 --no-k-rows)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-prof}_${WHICH:-c4}
mkdir -p "$OUT"
if [ "${WHICH:-c4}" = c4 ]; then
  CMD="python3 tools/gpu/qt_bench.py --steps 3 --check-rows 1"
else
  CMD="python3 tools/gpu/stream_bench.py --genomes 100000 --device-only"
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ks" -o run -- $CMD > "$OUT/ks.log" 2>&1 || { tail -20 "$OUT/ks.log"; exit 1; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS" \
           "SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 400 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/pmc/p$i" -o run -- $CMD \
      > "$OUT/pmc_p$i.log" 2>&1 || { echo "pass $i ($grp) failed"; tail -20 "$OUT/pmc_p$i.log"; exit 1; }
done
ls "$OUT/ks" "$OUT"/pmc/*
