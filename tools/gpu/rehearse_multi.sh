#!/bin/bash
# Rehearsal of bench.py's N > 1 flow on a one-GPU box (gloo, all ranks on
# device 0, gather through host memory; RCCL refuses two ranks per device):
# split, spans, double-buffered / chunked gather, reassembly, and rank 0's
# bit-exact check of the gathered AJI against a single-device run.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --rehearse-gloo > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.log \
    || { tail -30 gpurun_out/rehearse2.log; exit 1; }
cat gpurun_out/rehearse2.json; grep "bit-exact" gpurun_out/rehearse2.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 \
    --master-port 29512 bench.py --gpus 3 --steps 3 --warmup 1 --chunks 2 --rehearse-gloo > gpurun_out/rehearse3.json 2> gpurun_out/rehearse3.log \
    || { tail -30 gpurun_out/rehearse3.log; exit 1; }
cat gpurun_out/rehearse3.json; grep "bit-exact" gpurun_out/rehearse3.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline none > gpurun_out/bench_k.json 2> gpurun_out/bench_k.log || { tail -5 gpurun_out/bench_k.log; exit 1; }
cat gpurun_out/bench_k.json
