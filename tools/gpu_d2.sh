#!/bin/bash
# 2 ranks sharing one card (gloo), configs[3]: the overlapped scheduler's A/B knobs
set -o pipefail
export PYTHONPATH=.
O=gpurun_out/d2; mkdir -p $O
i=0
for m in "${@:---serial-codec}"; do
i=$((i+1))
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29540+i)) bench.py --gpus 2 --config 3 --steps 1 --warmup 1 --no-cpu-baseline --no-probe --dist-backend gloo $m > $O/c3_$i.jsonl 2> $O/c3_$i.err || { tail -5 $O/c3_$i.err; exit 1; }
echo "$m"; python3 tools/summ.py $O/c3_$i.jsonl
done
