#!/bin/bash
# quick GPU check: the given pytest selection (default: the whole -m gpu suite), then the default
# bench line without the CPU baseline. Outputs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
SEL=${SEL:-tests/}
timeout -k 10 ${TTO:-700} python -u -m pytest $SEL -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -5 gpurun_out/tests.log; [ $rc = 0 ] || exit $rc
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 400 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench.jsonl 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('gpurun_out/bench.jsonl').read().strip().splitlines()[-1])
print('value', d['value'], 'ms/step', d['ms_per_step'], 'p50', d['p50_first_chunk_latency_ms'])
print('roof', d['roofline']['kernel'], d['roofline']['frac'], 'step_rl', d.get('step_roofline'))
print('codec', d['codec_roofline']['avg_ms'], d['codec_roofline']['frac'], 'parity', (d.get('parity_mode_fp32') or {}).get('value'))
print({k: v['avg_us'] for k, v in d['kernels'].items()})
print(d['roofline'].get('traffic_ratio'))"
