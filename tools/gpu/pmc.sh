#!/bin/bash
# rocprofv3 PMC passes (one counter group per pass, kernel-trace only; never
# combined with sys/runtime traces) on one 10k all-vs-all run.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
CMD="python3 tools/gpu/ab_rows.py --genomes 10000 --rounds 0 --variants PFAAI_ROWS_OCC=3"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" "TA_BUSY_avr TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc/p$i" -o run -- $CMD > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i ($grp) failed"; tail -3 gpurun_out/pmc/p$i.log; }
done
ls gpurun_out/pmc/*/
