#!/bin/bash
# Per-kernel times of the decode step (default: the fp32 parity mode and the bf16 step at B = 32,
# positions 384..639; B / P0 / SPEC / WS / LVX_SWEEP_KV select others): rocprofv3 kernel-trace stats of tools/step_sweep.py (null stream: each
# kernel a dispatch of its own). Outputs under gpurun_out/fp32t.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
O=gpurun_out/fp32t; mkdir -p $O
SPEC=${SPEC:-}  # an option set for step_sweep (e.g. exp=8)
for w in ${WS:-fp32 bf16}; do
  LVX_SWEEP_W=$w timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $O/$w -o run --output-format csv -- python3 tools/step_sweep.py ${B:-32} ${P0:-384} $SPEC > $O/$w.log 2>&1 || { echo FAIL $w; tail -20 $O/$w.log; exit 1; }
  find $O/$w -name "*kernel_stats.csv" -exec cp {} $O/${w}_stats.csv \;
  rm -rf $O/$w
  grep us/step $O/$w.log
done
