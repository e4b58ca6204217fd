#!/bin/bash
# A/B: decode steps replayed as HIP graphs (side stream) vs launched one by one (--no-graphs)
set -o pipefail
export PYTHONPATH=.
mkdir -p gpurun_out
for i in 1 2; do for g in "--graph-stream" ""; do for c in 1 2; do
  ex=""; [ "$c" == "2" ] && ex="--steps 2"
  timeout -k 10 200 python bench.py --config $c $ex --no-cpu-baseline --no-probe $g > gpurun_out/ab.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('c$c', '$g' or 'null stream', d['value'], d['ms_per_step'])"
done; done; done
