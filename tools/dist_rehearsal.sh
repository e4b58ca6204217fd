#!/bin/bash
# multi-rank bench path rehearsed on one GPU: 2 ranks, gloo collectives through host copies
set -o pipefail
export PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --dist-backend gloo > gpurun_out/dist2.jsonl 2> gpurun_out/dist2.err && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --config 3 --steps 1 --warmup 1 --no-cpu-baseline --no-probe --dist-backend gloo > gpurun_out/dist2_c3.jsonl 2> gpurun_out/dist2_c3.err
rc=$?; cat gpurun_out/dist2.jsonl gpurun_out/dist2_c3.jsonl | cut -c1-300; tail -3 gpurun_out/dist2.err; exit $rc
