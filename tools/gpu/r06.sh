#!/bin/bash
# Round 6 GPU steps, one box, in the order given by STEPS (space separated):
#   suite      the whole -m gpu suite
#   tests      the tests named in TESTS (pytest node ids / files)
#   qt         C4 shape: tools/gpu/qt_bench.py (50 000 targets x 1 000 queries)
#   qt_r05     the same against round 5's library (tools/_build/ab, A/B)
#   qt_t24 / qt_diag  the C4 run in the diagnostics build with / without PFAAI_PL_T24 (A/B of 24-member tasks)
#   stream     C5 shape: tools/gpu/stream_bench.py, 100 000 genomes, no-op sink
#   stream_t24 / stream_diag  the C5 run in the diagnostics build with / without PFAAI_PL_T24 (no re-check)
#   qt_rev / stream_rev / rev  the C4 / C5 / C3 (ab_rows) runs with PFAAI_PL_REV=1 (A/B of the round order)
#   sortab     A/B of the load sort's variants (tools/gpu/ab_sort.py, diagnostics build)
#   abprev     bench + C4 twice each, alternating this library and PREV (a saved earlier build)
#   stream_dev the C5 row tiles by pfaai_run into device buffers, no D2H (the row kernels alone)
#   stream_r05 the same against round 5's library
#   bench      the bench line (bench.py --steps 20 --warmup 5, no CPU baseline)
#   cyclic     one-GPU emulation of the 8-way split: contiguous vs block-cyclic (tools/gpu/shard_cyclic.py)
#   stag       A/B of k_rows_pl's S5-entry variants (PFAAI_PL_STAG, diagnostics build)
#   e2e        C2 end to end: ours and the drop-in (E2E_ARGS="" adds the reference, ~5 min)
#   rehearse   bench.py's N > 1 flow with gloo on the one GPU (tools/gpu/rehearse_multi.sh)
#   smoke      __graft_entry__.smoke()
# Every step has its own time limit and the first failure ends the call.
#   TAG=r06a STEPS="tests qt qt_r05" TESTS=tests/test_gpu_stream.py bash tools/gpu/r06.sh
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-r06}
mkdir -p "$OUT"
export TMPDIR=/tmp
R05=tools/_build/ab/libpfaai_hip_r05.so
PYT="python3 -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu"
for step in ${STEPS:-suite}; do
  echo "== $step $(date +%T)"
  case $step in
    suite) timeout -k 10 1000 $PYT tests > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; } ;;
    tests) timeout -k 10 900 $PYT $TESTS > "$OUT/tests_sel.txt" 2>&1 || { tail -30 "$OUT/tests_sel.txt"; exit 1; } ;;
    qt) timeout -k 10 500 python3 -u tools/gpu/qt_bench.py > "$OUT/qt_c4.json" 2> "$OUT/qt.err" || exit 1 ;;
    qt_r05) PFAAI_HIP_LIB=$R05 timeout -k 10 500 python3 -u tools/gpu/qt_bench.py > "$OUT/qt_c4_r05.json" 2> "$OUT/qt_r05.err" || exit 1 ;;
    qt_t24) PFAAI_HIP_LIB=parfastaai_amd/lib/libpfaai_hip_diag.so PFAAI_PL_T24=1 timeout -k 10 500 python3 -u tools/gpu/qt_bench.py > "$OUT/qt_c4_t24_diag.json" 2> "$OUT/qt_t24.err" || exit 1 ;;
    qt_diag) PFAAI_HIP_LIB=parfastaai_amd/lib/libpfaai_hip_diag.so timeout -k 10 500 python3 -u tools/gpu/qt_bench.py > "$OUT/qt_c4_diag.json" 2> "$OUT/qt_diag.err" || exit 1 ;;
    stream) timeout -k 10 600 python3 -u tools/gpu/stream_bench.py --genomes 100000 --sinks noop par > "$OUT/stream_100k.json" 2> "$OUT/stream.err" || exit 1 ;;
    stream_t24) PFAAI_HIP_LIB=parfastaai_amd/lib/libpfaai_hip_diag.so PFAAI_PL_T24=1 timeout -k 10 600 python3 -u tools/gpu/stream_bench.py --genomes 100000 --sinks noop --check-rows 0 > "$OUT/stream_100k_t24_diag.json" 2> "$OUT/stream_t24.err" || exit 1 ;;
    stream_diag) PFAAI_HIP_LIB=parfastaai_amd/lib/libpfaai_hip_diag.so timeout -k 10 600 python3 -u tools/gpu/stream_bench.py --genomes 100000 --sinks noop --check-rows 0 > "$OUT/stream_100k_diag.json" 2> "$OUT/stream_diag.err" || exit 1 ;;
    stream_rev) PFAAI_HIP_LIB=parfastaai_amd/lib/libpfaai_hip_diag.so PFAAI_PL_REV=1 timeout -k 10 600 python3 -u tools/gpu/stream_bench.py --genomes 100000 --sinks noop --check-rows 0 > "$OUT/stream_100k_rev_diag.json" 2> "$OUT/stream_rev.err" || exit 1 ;;
    qt_rev) PFAAI_HIP_LIB=parfastaai_amd/lib/libpfaai_hip_diag.so PFAAI_PL_REV=1 timeout -k 10 500 python3 -u tools/gpu/qt_bench.py > "$OUT/qt_c4_rev_diag.json" 2> "$OUT/qt_rev.err" || exit 1 ;;
    rev) PFAAI_HIP_LIB=parfastaai_amd/lib/libpfaai_hip_diag.so timeout -k 10 400 python3 -u tools/gpu/ab_rows.py --genomes 10000 --rounds 7 \
            --variants PFAAI_PL_REV=0 PFAAI_PL_REV=1 > "$OUT/ab_rev.txt" 2> "$OUT/ab_rev.err" || exit 1 ;;
    sortab) PFAAI_HIP_LIB=parfastaai_amd/lib/libpfaai_hip_diag.so timeout -k 10 400 python3 -u tools/gpu/ab_sort.py --genomes 10000 --rounds 5 \
            --variants - PFAAI_SORT_DIRECT=1 > "$OUT/ab_sort.txt" 2> "$OUT/ab_sort.err" || exit 1 ;;
    abprev) for L in parfastaai_amd/lib/libpfaai_hip.so $PREV parfastaai_amd/lib/libpfaai_hip.so $PREV; do
              n=$(basename $L .so)
              PFAAI_HIP_LIB=$L timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-baseline none >> "$OUT/abprev_bench_$n.json" 2>> "$OUT/abprev.err" || exit 1
              PFAAI_HIP_LIB=$L timeout -k 10 300 python3 -u tools/gpu/qt_bench.py --steps 5 >> "$OUT/abprev_qt_$n.json" 2>> "$OUT/abprev.err" || exit 1
            done ;;
    stream_dev) timeout -k 10 600 python3 -u tools/gpu/stream_bench.py --genomes 100000 --device-only > "$OUT/stream_100k_device.json" 2> "$OUT/stream_dev.err" || exit 1 ;;
    stream_r05) PFAAI_HIP_LIB=$R05 timeout -k 10 600 python3 -u tools/gpu/stream_bench.py --genomes 100000 --sinks noop par > "$OUT/stream_100k_r05.json" 2> "$OUT/stream_r05.err" || exit 1 ;;
    bench) timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-baseline none > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1 ;;
    cyclic) timeout -k 10 400 python3 -u tools/gpu/shard_cyclic.py 10000 8 --reps 5 > "$OUT/shard_cyclic.txt" 2> "$OUT/shard_cyclic.err" || exit 1 ;;
    stag) PFAAI_HIP_LIB=parfastaai_amd/lib/libpfaai_hip_diag.so timeout -k 10 400 python3 -u tools/gpu/ab_rows.py --genomes 10000 --rounds 7 \
            --variants ${STAG_VARIANTS:-PFAAI_PL_STAG=0 PFAAI_PL_STAG=1 PFAAI_PL_STAG=2 PFAAI_PL_STAG=3 PFAAI_PL_STAG=4 PFAAI_PL_STAG=5} \
            > "$OUT/ab_stag.txt" 2> "$OUT/ab_stag.err" || exit 1 ;;
    e2e) timeout -k 10 900 python3 -u tools/gpu/e2e_c2.py --repeats 3 ${E2E_ARGS:---skip-ref} > "$OUT/e2e_c2.json" 2> "$OUT/e2e.err" || exit 1 ;;
    rehearse) OUT="$OUT" bash tools/gpu/rehearse_multi.sh || exit 1 ;;
    smoke) timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  tail -c 600 "$OUT"/*.json 2>/dev/null | tail -3
done
echo "== done $(date +%T)"
