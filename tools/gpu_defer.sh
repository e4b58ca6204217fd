set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 400 python -u -m pytest tests/test_gpu_select.py tests/test_gpu_parity.py tests/test_gpu_bf16.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1 \
 && timeout -k 10 200 python -u tools/step_sweep.py 1 1024 defer_select=0 defer_select=1 defer_select=0 defer_select=1 > gpurun_out/sweep.log 2>&1 \
 && timeout -k 10 200 python -u tools/step_sweep.py 2 1024 defer_select=0 defer_select=1 >> gpurun_out/sweep.log 2>&1 \
 && timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_c1.jsonl 2> gpurun_out/bench_c1.err
rc=$?
grep -E "passed|failed|Error" gpurun_out/tests.log | tail -5
cat gpurun_out/sweep.log; tail -c 600 gpurun_out/bench_c1.jsonl
echo "EXIT $rc"
exit $rc
