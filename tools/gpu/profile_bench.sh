#!/bin/bash
# The committed profile set of a round, all from ONE build and the bench's own
# command: the bench line; rocprofv3 kernel stats of the
# same command (tools/rocpd_stats.py: calls, mean, median, min, max per
# kernel); PMC passes over it, one counter group per run (HBM bytes, SQ
# instruction / busy counters) -> tools/pmc_summary.py.
#   PROF_TAG=r04z bash tools/gpu/profile_bench.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${PROF_TAG:-prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="python3 bench.py --steps 20 --warmup 5 --cpu-baseline none"
timeout -k 10 300 $BENCH > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks -o bench -- $BENCH > $OUT/ks.log 2>&1 || exit 1
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_WAVES" \
           "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/pmc/p$i -o run -- \
      python3 bench.py --steps 3 --warmup 1 --cpu-baseline none > $OUT/pmc_p$i.log 2>&1 || { echo "pass $i ($grp) failed"; exit 1; }
done
ls $OUT/ks $OUT/pmc/*
