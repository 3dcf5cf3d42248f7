#!/bin/bash
# Rehearsal of bench.py's N > 1 flow on a one-GPU box (gloo, all ranks on
# device 0, transfers through host memory; RCCL refuses two ranks per device):
# the block-cyclic split (--split cyclic: row lists, grouped send / recv of the
# rows' segments into rank 0's array, double-buffered) with 2 and 3 ranks,
# the contiguous split with chunked gathers with 3, each ending in rank 0's
# bit-exact check of the assembled AJI against a single-device run.
#   OUT=gpurun_out/x bash tools/gpu/rehearse_multi.sh
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
export MASTER_ADDR=127.0.0.1
run() {  # name port nproc args...
  local name=$1 port=$2 np=$3; shift 3
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$np" --master-addr 127.0.0.1 \
      --master-port "$port" bench.py --gpus "$np" --steps 3 --warmup 1 --rehearse-gloo --cpu-baseline none "$@" \
      > "$OUT/$name.json" 2> "$OUT/$name.log" || { tail -30 "$OUT/$name.log"; return 1; }
  grep "bit-exact" "$OUT/$name.log"
}
run rehearse2_cyclic 29511 2 --split cyclic && run rehearse3_cyclic 29512 3 --split cyclic && \
    run rehearse3_contig 29513 3 --split contiguous --chunks 2 && run rehearse2_contig 29514 2 || exit 1
[ -n "$NO_RCCL" ] && exit 0
# the same flows through RCCL itself (--rccl-one-gpu: each rank its own NCCL
# host, RCCL's socket transport on loopback): gather and grouped send / recv
rccl() {  # name port nproc args...
  local name=$1 port=$2 np=$3; shift 3
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$np" --master-addr 127.0.0.1 \
      --master-port "$port" bench.py --gpus "$np" --steps 3 --warmup 1 --rccl-one-gpu --cpu-baseline none "$@" \
      > "$OUT/$name.json" 2> "$OUT/$name.log" || { tail -30 "$OUT/$name.log"; return 1; }
  grep -h "communicator\|bit-exact" "$OUT/$name.log"
}
rccl rccl2_contig 29521 2 --split contiguous && rccl rccl2_cyclic 29522 2 --split cyclic && \
    rccl rccl3_cyclic 29523 3 --split cyclic
