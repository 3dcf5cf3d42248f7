#!/bin/bash
# Round 3: the transposition sort's digit width (diagnostics build,
# PFAAI_TSORT_DB) at 10k for the both-given and G-only loads, kernel traces,
# and FETCH/WRITE counters of the default sort.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/sortab
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
timeout -k 10 600 python -u -m pytest tests/test_gpu_load_sort.py tests/test_gpu_orientations.py tests/test_gpu_load_errors.py -x -q --timeout 300 --timeout-method thread > gpurun_out/sortab/pytest.log 2>&1 || { tail -30 gpurun_out/sortab/pytest.log; exit 1; }
tail -2 gpurun_out/sortab/pytest.log
for orient in both g; do
  for db in 8 9 10 11; do
    tag=${orient}_db$db
    PFAAI_HIP_LIB=$LIB PFAAI_TSORT_DB=$db timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$PWD/gpurun_out/sortab/$tag" -o run -- python3 tools/gpu/load_bench.py --orient $orient --reps 2 \
        > gpurun_out/sortab/$tag.json 2> gpurun_out/sortab/$tag.log || { tail -5 gpurun_out/sortab/$tag.log; exit 1; }
    echo "== $tag: $(tail -1 gpurun_out/sortab/$tag.json)"
    summ gpurun_out/sortab/$tag
  done
done
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$PWD/gpurun_out/sortab/pmc$i" -o run \
      -- python3 tools/gpu/load_bench.py --orient both --reps 1 > gpurun_out/sortab/pmc$i.log 2>&1 || { echo "pmc $grp failed"; tail -3 gpurun_out/sortab/pmc$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(dict)
for f in sorted(glob.glob("gpurun_out/sortab/pmc*/**/run_counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0][-60:]
        acc[n][r["Counter_Name"]] = acc[n].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for n, d in acc.items():
    if "sort" in n or "fkeys" in n:
        print(n, {k: round(v / 1e6, 1) for k, v in d.items()}, "(FETCH/WRITE MB = KiB/1e6*1.024)")
PY
