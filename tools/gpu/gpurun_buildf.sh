#!/bin/bash
# New device F build tests, the full GPU suite, smoke, and a KW A/B at 10k / 40k.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
echo "== build_f tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_build_f.py -x -v --timeout 240 --timeout-method thread > gpurun_out/buildf_tests.log 2>&1; rc=$?; tail -10 gpurun_out/buildf_tests.log; [ $rc -eq 0 ] || exit $rc
echo "== gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -4 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== KW A/B 10k"
timeout -k 10 300 python tools/gpu/ab_rows.py --genomes 10000 --rounds 3 --variants PFAAI_PL_KWMAX=5 PFAAI_PL_KWMAX=4 > gpurun_out/ab_kw10k.log 2>&1; rc=$?; tail -3 gpurun_out/ab_kw10k.log; [ $rc -eq 0 ] || exit $rc
echo "== KW A/B 40k rows 0:4000"
timeout -k 10 300 python tools/gpu/ab_rows.py --genomes 40000 --rows 0:4000 --rounds 2 --variants PFAAI_PL_KWMAX=5 PFAAI_PL_KWMAX=4 > gpurun_out/ab_kw40k.log 2>&1; rc=$?; tail -3 gpurun_out/ab_kw40k.log; exit $rc
