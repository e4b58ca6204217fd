#!/bin/bash
# in-step kernel durations and gaps at B = 1 / 2 (kernel trace of tools/prof_ar.py), per kernel
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
mkdir -p gpurun_out
rm -rf gpurun_out/t_*
for B in ${BS:-1 32}; do
  timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/t_$B -o run --output-format csv -- python3 tools/prof_ar.py bf16 $B > gpurun_out/t_$B.log 2>&1 || { echo "FAIL $B"; exit 1; }
  f=$(find gpurun_out/t_$B -name "*kernel_trace.csv" | head -1)
  python3 tools/trace_gaps.py $f 340 "ar_" > gpurun_out/t_${B}_gaps.txt
  cat gpurun_out/t_${B}_gaps.txt
done
