set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b1.jsonl 2> gpurun_out/b1.err \
 && timeout -k 10 200 python -u tools/step_sweep.py 1 1024 "" "" > gpurun_out/sweep.log 2>&1 \
 && timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b2.jsonl 2> gpurun_out/b2.err
rc=$?
for f in gpurun_out/b1.jsonl gpurun_out/b2.jsonl; do python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], {k:v['avg_us'] for k,v in d['kernels'].items()})"; done
cat gpurun_out/sweep.log | grep -v amdgpu.ids
exit $rc
