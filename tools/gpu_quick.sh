#!/bin/bash
# quick GPU iteration: the given pytest selection, then bench configs[1] and configs[2] (no CPU baseline)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/} -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1 \
 && timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_c1.jsonl 2> gpurun_out/bench_c1.err \
 && timeout -k 10 300 python bench.py --streams 32 --steps 2 --no-cpu-baseline > gpurun_out/bench_c2.jsonl 2> gpurun_out/bench_c2.err \
 && timeout -k 10 300 python bench.py --streams 64 --steps 2 --no-cpu-baseline > gpurun_out/bench_c64.jsonl 2> gpurun_out/bench_c64.err
rc=$?
grep -E "passed|failed|Error" gpurun_out/tests.log | tail -5
for f in gpurun_out/bench_c*.jsonl; do python -c "
import json,sys
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], {k:v['avg_us'] for k,v in d['kernels'].items()})" 2>/dev/null; done
echo "EXIT $rc"
exit $rc
