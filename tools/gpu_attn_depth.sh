set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 300 python -u -m pytest tests/test_gpu_batched.py tests/test_gpu_parity.py tests/test_gpu_fp8.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1 \
 && timeout -k 10 200 python -u tools/step_sweep.py 32 256 attn_depth=2 attn_depth=4 attn_depth=8 > gpurun_out/sweep.log 2>&1 \
 && timeout -k 10 200 python -u tools/step_sweep.py 64 256 attn_depth=2 attn_depth=4 attn_depth=8 >> gpurun_out/sweep.log 2>&1 \
 && timeout -k 10 200 python -u tools/step_sweep.py 1 1024 attn_depth=2 attn_depth=4 >> gpurun_out/sweep.log 2>&1 \
 && timeout -k 10 200 python -u tools/step_sweep.py 16 2048 attn_depth=2 attn_depth=4 attn_depth=8 >> gpurun_out/sweep.log 2>&1
rc=$?
grep -E "passed|failed|Error" gpurun_out/tests.log | tail -5
cat gpurun_out/sweep.log | grep -v amdgpu.ids
echo "EXIT $rc"
exit $rc
