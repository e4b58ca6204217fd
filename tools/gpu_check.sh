set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1 \
 && timeout -k 10 200 python -u tools/step_sweep.py 32 256 defer_select=0 defer_select=1 > gpurun_out/sweep.log 2>&1 \
 && timeout -k 10 200 python -u tools/step_sweep.py 64 256 defer_select=0 defer_select=1 >> gpurun_out/sweep.log 2>&1 \
 && timeout -k 10 200 python -u tools/step_sweep.py 12 256 defer_select=0 defer_select=1 >> gpurun_out/sweep.log 2>&1 \
 && timeout -k 10 200 python -u tools/step_sweep.py 16 256 defer_select=0 defer_select=1 >> gpurun_out/sweep.log 2>&1
rc=$?
grep -E "passed|failed|Error" gpurun_out/tests.log | tail -5
cat gpurun_out/sweep.log | grep -v amdgpu.ids
echo "EXIT $rc"
exit $rc
