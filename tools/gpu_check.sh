#!/bin/bash
# one GPU round: parity tests, timing probe, kernel-trace profile
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 600 python -m pytest tests/ -m gpu -q -x > gpurun_out/tests.log 2>&1
echo "TESTS EXIT $?" >> gpurun_out/tests.log
tail -3 gpurun_out/tests.log
timeout -k 10 300 python tools/probe_ar.py bf16 > gpurun_out/probe.log 2>&1 || exit 1
timeout -k 10 300 python tools/probe_ar.py fp32 >> gpurun_out/probe.log 2>&1 || exit 1
cat gpurun_out/probe.log
if [ "$1" == "prof" ]; then
  cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
  rm -rf gpurun_out/prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 tools/prof_ar.py ${2:-bf16} ${3:-1} > gpurun_out/prof_log.txt 2>&1
fi
