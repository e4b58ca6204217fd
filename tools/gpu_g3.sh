#!/bin/bash
# codec large-M GEMM A/B: bf16 codec tests, decode timings with option values ($OPTS, space-separated
# "k=v,k=v" sets), kernel-trace stats of the 32 x 256 decode per set. Outputs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
OPTS=${OPTS:-"exp=0 exp=1"}
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec_bf16.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g3_tests.log 2>&1; rc=$?
tail -3 gpurun_out/g3_tests.log
[ $rc = 0 ] || exit $rc
: > gpurun_out/g3_probe.txt
for o in $OPTS; do
  timeout -k 10 120 python tools/codec_probe.py 20 bf16 $o 32x256,16x256,8x256,2x1280 >> gpurun_out/g3_probe.txt 2>&1 || exit 1
done
grep frames gpurun_out/g3_probe.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for o in $OPTS; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/g3kt -o run --output-format csv -- python3 tools/codec_probe.py 10 bf16 $o 32x256 > gpurun_out/g3kt.log 2>&1 || exit 1
  f=$(find gpurun_out/g3kt -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/g3_kstats_$o.csv; rm -rf gpurun_out/g3kt
  echo "== $o"; grep -E "gemm|dwconv|gn_apply|istft" gpurun_out/g3_kstats_$o.csv | cut -d, -f1-4 | cut -c1-150
done
