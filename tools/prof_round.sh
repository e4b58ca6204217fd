#!/bin/bash
# kernel-trace profiles: AR at B = 1 and 32, codec at 1 x 256 and 32 x 256 frames
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
mkdir -p gpurun_out
rm -rf gpurun_out/p_*
for cfg in "ar1 tools/prof_ar.py bf16 1" "ar32 tools/prof_ar.py bf16 32" "c1 tools/prof_codec.py bf16 256 1" "c32 tools/prof_codec.py bf16 256 32"; do
  set -- $cfg
  tag=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/p_$tag -o run --output-format csv -- python3 "$@" > gpurun_out/p_$tag.log 2>&1 || { echo "FAIL $tag"; exit 1; }
done
echo OK
