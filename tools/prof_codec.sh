#!/bin/bash
# kernel-trace profile of the codec at S x L frames
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
rm -rf gpurun_out/p_c
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/p_c -o run --output-format csv -- python3 tools/prof_codec.py bf16 ${2:-256} ${1:-32} > gpurun_out/p_c.log 2>&1
