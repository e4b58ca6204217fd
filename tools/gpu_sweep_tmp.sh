set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 300 python -u -m pytest tests/test_gpu_select.py tests/test_gpu_bf16.py tests/test_gpu_streaming.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1 \
 && timeout -k 10 200 python -u tools/step_sweep.py 1 1024 fuse_mlp=1 fuse_mlp=3 fuse_mlp=1 fuse_mlp=3 > gpurun_out/sweep.log 2>&1 \
 && timeout -k 10 200 python -u tools/step_sweep.py 2 1024 fuse_mlp=1 fuse_mlp=3 >> gpurun_out/sweep.log 2>&1
rc=$?
grep -E "passed|failed|Error" gpurun_out/tests.log | tail -5
cat gpurun_out/sweep.log | grep -v amdgpu.ids
exit $rc
