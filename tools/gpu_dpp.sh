set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1 \
 && timeout -k 10 200 python -u tools/step_sweep.py 1 1024 "" > gpurun_out/sweep.log 2>&1 \
 && timeout -k 10 200 python -u tools/step_sweep.py 2 1024 "" >> gpurun_out/sweep.log 2>&1 \
 && timeout -k 10 200 python -u tools/step_sweep.py 32 256 attn_depth=2 attn_depth=4 >> gpurun_out/sweep.log 2>&1 \
 && timeout -k 10 200 python -u tools/step_sweep.py 64 256 attn_depth=2 attn_depth=4 >> gpurun_out/sweep.log 2>&1 \
 && timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_c1.jsonl 2> gpurun_out/bench_c1.err \
 && timeout -k 10 300 python bench.py --config 2 --steps 2 --no-cpu-baseline > gpurun_out/bench_c2.jsonl 2> gpurun_out/bench_c2.err
rc=$?
grep -E "passed|failed|Error" gpurun_out/tests.log | tail -5
cat gpurun_out/sweep.log | grep -v amdgpu.ids
for f in gpurun_out/bench_c1.jsonl gpurun_out/bench_c2.jsonl; do python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], {k:v['avg_us'] for k,v in d['kernels'].items()})" 2>/dev/null; done
echo "EXIT $rc"
exit $rc
