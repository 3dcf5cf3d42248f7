#!/bin/bash
# Rehearsal of bench.py's N > 1 path (RCCL pipelined gather) with 2 ranks on
# the box's one GPU (RCCL may refuse two ranks on one device; then gloo-free
# evidence is the CPU test).  Small DB so it is quick.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --genomes 2000 > gpurun_out/rehearse_n2.log 2>&1; rc=$?; tail -15 gpurun_out/rehearse_n2.log; exit $rc
