#!/bin/bash
# attention probe time vs B at t = 512 (one block per (stream, head): 12 B blocks over 256 CUs)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
O=gpurun_out/attnB; mkdir -p $O
for S in 16 21 24 32 40 42 48 64; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity-line --no-loaded-latency --streams $S --steps 4 --warmup 1 > $O/s$S.jsonl 2> $O/s$S.err || { echo "S=$S failed"; tail -5 $O/s$S.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels']; print('B', sys.argv[2], 'tok/s', d['value'], 'step_us', d['step_roofline']['us_per_step'], ' '.join(f\"{n.split()[1] if ' ' in n else n}={v['avg_us']}\" for n,v in k.items()))" $O/s$S.jsonl $S
done
