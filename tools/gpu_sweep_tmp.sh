set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_codec_bf16.py tests/test_gpu_fp8.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1 \
 && timeout -k 10 200 python -u tools/codec_sweep.py 1:256,8:256,32:256 "" "" > gpurun_out/sweep.log 2>&1 \
 && LVX_LIB_PATH=$PWD/llmvox_amd/libllmvox_hip_ab.so timeout -k 10 200 python -u tools/codec_sweep.py 1:256,8:256,32:256 "" "" >> gpurun_out/sweep.log 2>&1
rc=$?
grep -E "passed|failed|Error" gpurun_out/tests.log | tail -5
cat gpurun_out/sweep.log | grep -v amdgpu.ids
exit $rc
