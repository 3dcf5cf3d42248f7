set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -2 gpurun_out/smoke.log &&
echo "== gpu tests"; timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -30 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] &&
echo "== bench 2k"; timeout -k 10 400 python bench.py --steps 5 --warmup 2 --genomes 2000 --cpu-baseline none > gpurun_out/bench_2k.log 2>&1; rc=$?; tail -5 gpurun_out/bench_2k.log; [ $rc -eq 0 ] &&
echo "== bench 10k"; timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_10k.log 2>&1; rc=$?; tail -5 gpurun_out/bench_10k.log; exit $rc
