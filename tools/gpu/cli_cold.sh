set -o pipefail
cd /root/repo
mkdir -p gpurun_out /tmp/w
python -c "
import sys; sys.path.insert(0,'.')
from parfastaai_amd import syn
syn.write_db('/tmp/w/c2.db', 2000, 100)
" || exit 1
for e in "" "HIP_ENABLE_DEFERRED_LOADING=0"; do
  echo "== env: $e"
  env $e timeout -k 10 120 ./parfastaai_amd/lib/par_fastaai_amd /tmp/w/c2.db /tmp/w/out.csv 2>&1 | grep -E "AJI|breakdown|Total|Load" || exit 1
done
