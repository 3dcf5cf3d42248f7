#!/bin/bash
# Why does the per-event rate fall with N?  (1) column chunks alone: 10k
# with 2048-column chunks; (2) stream rate at 20k (|F| < 2^30) and 40k;
# (3) HBM traffic + L2 hits of one all-rows launch at 40k.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== 10k: KW 5 (1 chunk) vs KW 1 (5 chunks)"
timeout -k 10 300 python tools/gpu/ab_rows.py --genomes 10000 --rounds 3 --variants PFAAI_PL_KWMAX=5 PFAAI_PL_KWMAX=1 > gpurun_out/diag_kw.log 2>&1; rc=$?; tail -6 gpurun_out/diag_kw.log; [ $rc -eq 0 ] || exit $rc
for n in 20000 40000; do
echo "== stream $n"
timeout -k 10 300 python tools/gpu/stream_bench.py --genomes $n > gpurun_out/diag_stream_$n.json 2> gpurun_out/diag_stream_$n.log; rc=$?; cat gpurun_out/diag_stream_$n.json; [ $rc -eq 0 ] || exit $rc
done
echo "== PMC 40k"
PMC_TAG=pmc40k PMC_GENOMES=40000 PMC_SET="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum" timeout -k 10 600 bash tools/gpu/pmc_pl.sh > gpurun_out/diag_pmc40k.log 2>&1; rc=$?; tail -5 gpurun_out/diag_pmc40k.log; exit $rc
