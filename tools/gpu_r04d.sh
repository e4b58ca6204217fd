#!/bin/bash
# round 4: fused c_attn + attention (option fuse_attn): the -m gpu suite, step A/B at B = 16 / 24 / 32,
# the default bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
O=gpurun_out/r04d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc = 0 ] || exit $rc
for B in 32 24 16; do
  LVX_SWEEP_STREAM=1 timeout -k 10 200 python tools/step_sweep.py $B 384 'fuse_attn=1' 'fuse_attn=0' 'fuse_attn=1' 'fuse_attn=0' > $O/sweep_B$B.txt 2>&1 || { tail $O/sweep_B$B.txt; exit 1; }
  cat $O/sweep_B$B.txt
done
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.jsonl 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench.jsonl').read().strip().splitlines()[-1])
print('value', d['value'], 'ms/step', d['ms_per_step'], 'p50', d['p50_first_chunk_latency_ms'], 'loaded', d['p50_first_chunk_latency_loaded_ms'])
print('roof', d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['avg_us'], 'step', d['step_roofline']['us_per_step'], d['step_roofline']['frac'])
print('codec', d['codec_roofline']['avg_ms'], 'parity', d['parity_mode_fp32']['value'], d['parity_mode_fp32']['ratio_to_headline'])
print({k: v['avg_us'] for k, v in d['kernels'].items()})"
