#!/bin/bash
# Full GPU check of the tree: the -m gpu suite, the driver's default bench line, codec timings and
# the vendor-GEMM ceiling on the codec shapes. Outputs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 700 python -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -3 gpurun_out/tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.jsonl 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
tail -c 1500 gpurun_out/bench.jsonl
timeout -k 10 120 python tools/codec_probe.py 20 > gpurun_out/codec_probe.txt 2>&1 || exit 1
cat gpurun_out/codec_probe.txt
timeout -k 10 120 python tools/gemm_ceiling.py > gpurun_out/gemm_ceiling.txt 2>&1 || exit 1
cat gpurun_out/gemm_ceiling.txt
