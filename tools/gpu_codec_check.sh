#!/bin/bash
# codec parity tests (fp32 golden + bf16 tolerance + large dumps + streams) and codec timing
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_codec_bf16.py tests/test_gpu_large_dumps.py tests/test_gpu_streaming.py tests/test_gpu_fp8.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/codec_tests.log 2>&1 || { tail -40 gpurun_out/codec_tests.log; exit 1; }
tail -1 gpurun_out/codec_tests.log
timeout -k 10 120 python tools/codec_probe.py 20 bf16 2>/dev/null
