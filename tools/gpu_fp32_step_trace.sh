#!/bin/bash
# kernel trace of the fp32 parity step (B = 32, t = 384-639, graph replay)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
O=gpurun_out/f32tr; mkdir -p $O
LVX_SWEEP_STREAM=1 LVX_SWEEP_W=fp32 timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 tools/step_sweep.py 32 384 '' > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
find $O/kt -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
rm -rf $O/kt
grep "us/step" $O/kt.log
python3 tools/kstats.py $O/kernel_stats.csv 2>/dev/null | head -20 || head -14 $O/kernel_stats.csv | cut -c1-150
