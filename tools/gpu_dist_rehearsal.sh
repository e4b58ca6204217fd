#!/bin/bash
# the 2-rank gloo rehearsals (one card) of configs[2] / configs[3]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
O=gpurun_out/lines; mkdir -p $O
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --no-probe --dist-backend gloo > $O/dist2.jsonl 2> $O/dist2.err || { tail -5 $O/dist2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/dist2.jsonl').read().strip().splitlines()[-1]); print('dist2', d['value'], d['ms_per_step'], d['config'].get('codec_schedule'))"
