set -o pipefail
cd /root/repo
mkdir -p gpurun_out /tmp/w
python -c "
import sys; sys.path.insert(0,'.')
from parfastaai_amd import syn
syn.write_db('/tmp/w/c2.db', 2000, 100)
" || exit 1
for r in 1 2; do
for e in "PFAAI_CLI_FAST_EXIT=1" "PFAAI_CLI_FAST_EXIT=0"; do
  s=$(date +%s%N)
  env $e timeout -k 10 120 ./parfastaai_amd/lib/par_fastaai_amd /tmp/w/c2.db /tmp/w/out_$r.csv > /tmp/w/log 2>&1 || { cat /tmp/w/log; exit 1; }
  t=$(date +%s%N)
  echo "$e wall $(( (t - s) / 1000000 )) ms; $(grep Total /tmp/w/log)"
done
done
cmp /tmp/w/out_1.csv /tmp/w/out_2.csv && echo "csv identical"
