#!/bin/bash
# Round 3: full GPU suite, the both-given load's kernel trace, the 8-way
# shard times for candidate cost-model fractions, and the bench line.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${TAG:-r03o}
mkdir -p $OUT
export TMPDIR=/tmp PFAAI_PROGRESS=$OUT/progress.log
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 600 --timeout-method thread \
    > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
fi
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/load_both" -o run \
    -- python3 tools/gpu/load_bench.py --orient both --reps 3 > $OUT/load_both.json 2> $OUT/load_both.log || { tail -5 $OUT/load_both.log; exit 1; }
cat $OUT/load_both.json
SHARD_FRACS=${SHARD_FRACS:-0.7,0.8,0.9} timeout -k 10 300 python3 -u tools/gpu/shard_times.py 10000 8 > $OUT/shard_times.txt 2>&1 || { tail -5 $OUT/shard_times.txt; exit 1; }
grep -E "k_rows ms|fit:" $OUT/shard_times.txt | cut -c1-160
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline none > $OUT/bench.json 2> $OUT/bench.log || { tail -5 $OUT/bench.log; exit 1; }
cat $OUT/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/stats" -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline none > $OUT/stats.log 2>&1 || { tail -5 $OUT/stats.log; exit 1; }
python3 - $OUT <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/stats/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:8]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms {int(r['Calls']):4d} calls  avg {float(r['AverageNs'])/1e6:8.3f}  {r['Name'][:90]}")
PY
