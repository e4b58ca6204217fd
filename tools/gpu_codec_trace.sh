#!/bin/bash
# codec per-kernel breakdown at 1 x 256 and 32 x 256 frames (bf16)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
mkdir -p gpurun_out
for S in 1 32; do
  rm -rf gpurun_out/p_c
  timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/p_c -o run --output-format csv -- python3 tools/prof_codec.py bf16 256 $S > gpurun_out/p_c.log 2>&1 || { echo FAIL; exit 1; }
  echo "== S=$S"
  python3 tools/codec_trace.py $(find gpurun_out/p_c -name "*kernel_trace.csv" | head -1) | tee gpurun_out/codec_trace_$S.txt
done
