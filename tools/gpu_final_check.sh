#!/bin/bash
# smoke() and the default bench line (no CPU baseline) on the current library; outputs under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_final.jsonl 2> gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 1; }
python3 -c "
import json
d = json.loads(open('gpurun_out/bench_final.jsonl').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['step_roofline']['us_per_step'], d['codec_roofline']['avg_ms'], d['parity_mode_fp32']['value'])"
