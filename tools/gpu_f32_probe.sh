#!/bin/bash
# fp32 parity mode breakdown on one GPU: the bench line in fp32 (per-kernel probes, step_roofline) and
# the fp32 codec (HIP events + kernel trace). Outputs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 300 python bench.py --dtype fp32 --steps 2 --warmup 1 --no-cpu-baseline --no-parity-line > gpurun_out/b32.jsonl 2> gpurun_out/b32.err || { tail -20 gpurun_out/b32.err; exit 1; }
python3 -c "
import json
d=json.loads(open('gpurun_out/b32.jsonl').read().strip().splitlines()[-1])
print('value', d['value'], 'ms/step', d['ms_per_step'])
print('step_rl', d.get('step_roofline'))
print('codec', d['codec_roofline']['avg_ms'])
print({k: v for k, v in d['kernels'].items()})"
timeout -k 10 120 python tools/codec_probe.py 3 fp32 "" 32x256 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/f32c -o run --output-format csv -- python3 tools/codec_probe.py 3 fp32 "" 32x256 > gpurun_out/f32c.log 2>&1 || { tail -5 gpurun_out/f32c.log; exit 1; }
python3 tools/kstats.py $(find gpurun_out/f32c -name '*kernel_stats.csv' | head -1) | head -25
