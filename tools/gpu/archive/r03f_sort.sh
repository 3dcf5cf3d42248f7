#!/bin/bash
# Round 3: transposition-sort workgroup shape (512-thread tiles, two per CU,
# with / without the next-tile prefetch, vs the 1024-thread form) and the
# batched k_gend: parity tests of the load paths on the release library, then
# load_bench kernel traces per variant (diagnostics library).
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${TAG:-r03f}
mkdir -p $OUT
export TMPDIR=/tmp
LIB=parfastaai_amd/lib/libpfaai_hip_diag.so
summ() {
python3 - "$1" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:12]:
    print(f"   {float(r['TotalDurationNs'])/1e6:8.3f} ms {int(r['Calls']):3d}x avg {float(r['AverageNs'])/1e6:7.3f}  {r['Name'][:95]}")
PY
}
timeout -k 10 600 python -u -m pytest tests/test_gpu_load_sort.py tests/test_gpu_orientations.py tests/test_gpu_load_errors.py tests/test_gpu_build_f.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
IFS="|" read -ra VLIST <<< "${VARIANTS:-nt1024 PFAAI_TSORT_NT=1024|pf1 PFAAI_TSORT_PF=1|pf0 PFAAI_TSORT_PF=0}"
for v in "${VLIST[@]}"; do
  set -- $v
  tag=$1; shift; envv="$*"
  for orient in ${ORIENTS:-both g f}; do
    env PFAAI_HIP_LIB=$LIB $envv timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$PWD/$OUT/${tag}_$orient" -o run -- python3 tools/gpu/load_bench.py --orient $orient --reps 2 \
        > $OUT/${tag}_$orient.json 2> $OUT/${tag}_$orient.log || { tail -5 $OUT/${tag}_$orient.log; exit 1; }
    echo "== $tag $orient: $(tail -1 $OUT/${tag}_$orient.json)"
    summ $OUT/${tag}_$orient
  done
done
