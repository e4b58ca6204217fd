#!/bin/bash
# codec: vendor-GEMM ceiling on the codec shapes + a kernel trace of tools/codec_probe.py
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
mkdir -p gpurun_out
[ "${CEIL:-1}" = 0 ] || timeout -k 10 120 python tools/gemm_ceiling.py > gpurun_out/gemm_ceiling.txt 2>&1 || { [ "${CEIL:-1}" = 0 ] || cat gpurun_out/gemm_ceiling.txt; exit 1; }
[ "${CEIL:-1}" = 0 ] || cat gpurun_out/gemm_ceiling.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ctrace -o run --output-format csv -- python3 tools/codec_probe.py 10 bf16 > gpurun_out/ctrace.log 2>&1 || { tail -20 gpurun_out/ctrace.log; exit 1; }
grep TFLOP gpurun_out/ctrace.log
find gpurun_out/ctrace -name "*kernel_trace.csv" | head -1 | xargs -I{} cp {} gpurun_out/codec_kernel_trace.csv
find gpurun_out/ctrace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/codec_kernel_stats.csv
rm -rf gpurun_out/ctrace
