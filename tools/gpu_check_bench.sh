#!/bin/bash
# the -m gpu suite, then the driver's default bench line (no CPU baseline) and the codec probe
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 700 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -3 gpurun_out/tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench.jsonl 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('gpurun_out/bench.jsonl').read().strip().splitlines()[-1])
print('value', d['value'], 'ms/step', d['ms_per_step'], 'p50', d['p50_first_chunk_latency_ms'], 'roof', d['roofline']['kernel'], d['roofline']['frac'], 'codec', d['codec_roofline']['avg_ms'], d['codec_roofline']['frac'])
print({k: v['avg_us'] for k, v in d['kernels'].items()})"
timeout -k 10 120 python tools/codec_probe.py 20 > gpurun_out/codec_probe.txt 2>&1 || exit 1
cat gpurun_out/codec_probe.txt
