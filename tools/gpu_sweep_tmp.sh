set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 400 python -u -m pytest tests/test_gpu_batched.py tests/test_gpu_select.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1 \
 && timeout -k 10 200 python -u tools/step_sweep.py 32 256 mfma_btile=0 mfma_btile=1 mfma_btile=0 mfma_btile=1 > gpurun_out/sweep.log 2>&1 \
 && timeout -k 10 200 python -u tools/step_sweep.py 24 256 mfma_btile=0 mfma_btile=1 >> gpurun_out/sweep.log 2>&1 \
 && timeout -k 10 200 python -u tools/step_sweep.py 32 512 mfma_btile=0 mfma_btile=1 >> gpurun_out/sweep.log 2>&1
rc=$?
grep -E "passed|failed|Error" gpurun_out/tests.log | tail -5
cat gpurun_out/sweep.log | grep -v amdgpu.ids
exit $rc
