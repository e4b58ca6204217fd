#!/bin/bash
# codec A/B on one GPU: the codec GPU tests, the codec probe (HIP events) and a kernel trace of it.
# Outputs under gpurun_out/. usage: bash tools/gpu_codec_ab.sh [probe opts]
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 400 python -u -m pytest tests/test_gpu_codec_bf16.py tests/test_gpu_large_dumps.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/codec_tests.log 2>&1
rc=$?; tail -3 gpurun_out/codec_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python tools/codec_probe.py 20 bf16 "${1:-}" > gpurun_out/codec_probe.txt 2>&1 || { cat gpurun_out/codec_probe.txt; exit 1; }
cat gpurun_out/codec_probe.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/ctrace -o run --output-format csv -- python3 tools/codec_probe.py 10 bf16 "${1:-}" 32x256 > gpurun_out/ctrace.log 2>&1 || { tail -5 gpurun_out/ctrace.log; exit 1; }
f=$(find gpurun_out/ctrace -name '*kernel_stats.csv' | head -1)
python3 tools/kstats.py "$f"
