#!/bin/bash
# bench lines of every BASELINE config on one GPU (no CPU baseline unless CPU=1)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
CB="--no-cpu-baseline"; [ "$CPU" == "1" ] && CB=""
for c in ${CONFIGS:-1 2 3 4}; do
  extra=""; [ "$c" == "3" ] && extra="--steps 2 --warmup 1"; [ "$c" == "2" ] && extra="--steps 2"; [ "$c" == "4" ] && extra="--steps 8"
  timeout -k 10 400 python bench.py --config $c $extra $CB > gpurun_out/bench_cfg$c.jsonl 2> gpurun_out/bench_cfg$c.err || { echo "config $c FAILED"; tail -5 gpurun_out/bench_cfg$c.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/bench_cfg$c.jsonl').read().strip().splitlines()[-1])
print('config $c', d['value'], 'tok/s', d['ms_per_step'], 'ms/step p50', d['p50_first_chunk_latency_ms'], 'rl', (d['roofline'] or {}).get('kernel'), (d['roofline'] or {}).get('frac'), 'codec', d.get('codec_roofline'))"
done
