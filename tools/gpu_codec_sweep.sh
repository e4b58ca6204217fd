#!/bin/bash
# codec option sweep on one GPU: for each option string, the 32 x 256-frame decode timed with HIP events
# and a kernel trace of it (per-kernel averages of the named kernels). Outputs under gpurun_out/.
# usage: bash tools/gpu_codec_sweep.sh "kernel-substring ..." "opt=v,..." ["opt=v,..." ...]
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
keys=$1; shift
i=0
for o in "$@"; do
  i=$((i+1))
  timeout -k 10 120 python tools/codec_probe.py 20 bf16 "$o" 32x256 || exit 1
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/sw$i -o run --output-format csv -- python3 tools/codec_probe.py 10 bf16 "$o" 32x256 > gpurun_out/sw$i.log 2>&1 || { tail -5 gpurun_out/sw$i.log; exit 1; }
  f=$(find gpurun_out/sw$i -name '*kernel_stats.csv' | head -1)
  python3 tools/kstats.py "$f" $keys
done
