#!/bin/bash
# codec A/B of a dev option (default: the skinny small-M GEMM variants) + the codec parity tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
OPT=${OPT:-codec_skinny}
VALS=${VALS:-"0 1"}
[ "${TESTS:-1}" = 0 ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_codec_bf16.py tests/test_gpu_parity.py tests/test_gpu_fp8.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/codec_ab_tests.log 2>&1 || { tail -30 gpurun_out/codec_ab_tests.log; exit 1; }
[ "${TESTS:-1}" = 0 ] || tail -1 gpurun_out/codec_ab_tests.log
for v in $VALS; do timeout -k 10 120 python tools/codec_probe.py 20 bf16 $OPT=$v $CASES | grep -v "32 x 256" || exit 1; done
