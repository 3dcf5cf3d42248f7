#!/bin/bash
# rocprofv3 PMC passes over one 10k all-vs-all row-kernel run (one counter
# group per pass, kernel trace only).  PMC_VARIANT selects the row kernel.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${PMC_TAG:-pmc}
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 tools/gpu/ab_rows.py --genomes ${PMC_GENOMES:-10000} --rounds 0 --variants ${PMC_VARIANT:-PFAAI_ROWS_KERNEL=pl}"
i=0
case "${PMC_SET:-hbm}" in
  hbm) G="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum" ;;
  sq) G="SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_WAVES;SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" ;;
  mem) G="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum;TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum;TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_LEVEL_sum" ;;
  full) G="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_WAVES;SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" ;;
  *) G="$PMC_SET" ;;
esac
IFS=';' read -ra PGRPS <<< "$G"
for grp in "${PGRPS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/p$i" -o run -- $CMD > $OUT/p$i.log 2>&1 || { echo "pass $i ($grp) failed"; tail -3 $OUT/p$i.log; exit 1; }
done
ls $OUT/*/
