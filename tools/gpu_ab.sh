#!/bin/bash
# Alternating A/B of bench.py lines on one box: A_ARGS vs B_ARGS (plus COMMON), PAIRS times.
# Outputs under gpurun_out/${OUT:-ab}; one summary line per run.
set -o pipefail
export PYTHONPATH=.
O=gpurun_out/${OUT:-ab}; mkdir -p $O
COMMON=${COMMON:-"--steps 8 --no-cpu-baseline --no-parity-line --no-probe --no-loaded-latency"}
for p in $(seq 1 ${PAIRS:-3}); do
  for v in A B; do
    eval args=\$${v}_ARGS
    timeout -k 10 300 python bench.py $COMMON $args > $O/$v$p.jsonl 2> $O/$v$p.err || { tail -5 $O/$v$p.err; exit 1; }
    python3 tools/summ.py $O/$v$p.jsonl
  done
done
