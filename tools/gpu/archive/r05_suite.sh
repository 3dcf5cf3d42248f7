#!/bin/bash
# Round 5: the GPU suite, then the bench line and smoke, one box.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-r05e}
mkdir -p $OUT
export PFAAI_PROGRESS=$OUT/progress.txt
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $OUT/tests.log 2>&1
rc=$?; tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-baseline none > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
