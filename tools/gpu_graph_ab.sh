#!/bin/bash
# bench A/B: launched kernels on the null stream vs HIP-graph replay on a side stream (--graph-stream),
# alternating, per config. Lines under gpurun_out/gab/.
set -o pipefail
export PYTHONPATH=.
O=gpurun_out/gab; mkdir -p $O
for cfg in ${CFGS:-2 4 1}; do
  for rep in 1 2; do
    for mode in "" "--graph-stream"; do
      timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-parity-line --no-probe $mode > $O/l.json 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
      python3 -c "
import json,sys
d=json.loads(open('$O/l.json').read().strip().splitlines()[-1])
print('cfg $cfg', '${mode:-null}', d['value'], d['ms_per_step'], (d.get('step_roofline') or {}).get('us_per_step'))" | tee -a $O/ab.txt
    done
  done
done
