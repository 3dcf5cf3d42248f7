#!/bin/bash
# Round 3: k_rows_pl lookahead form (LA) -- the whole GPU suite on the release
# library, then the 8-way shard times with LA off / KW <= 2 (default) / 3 / 5
# (diagnostics library, PFAAI_PL_LAKW), then the bench line.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${TAG:-r03l}
mkdir -p $OUT
export TMPDIR=/tmp PFAAI_PROGRESS=$OUT/progress.log
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q -rf --timeout 600 --timeout-method thread \
    > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
fi
for lakw in ${LAKWS:-0 2 3 5}; do
  PFAAI_HIP_LIB=parfastaai_amd/lib/libpfaai_hip_diag.so PFAAI_PL_LAKW=$lakw SHARD_FRACS=${SHARD_FRACS:-} \
      timeout -k 10 300 python3 -u tools/gpu/shard_times.py 10000 8 > $OUT/shard_la$lakw.txt 2>&1 || { tail -5 $OUT/shard_la$lakw.txt; exit 1; }
  echo "== LAKW=$lakw"; grep -E "k_rows ms|fit:" $OUT/shard_la$lakw.txt | cut -c1-200
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline none > $OUT/bench.json 2> $OUT/bench.log || { tail -5 $OUT/bench.log; exit 1; }
cat $OUT/bench.json
