#!/bin/bash
# A/B: decode steps per captured HIP graph (16 default vs 64 / 256 variant builds), alternating
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
O=gpurun_out/abgs; mkdir -p $O
B="timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity-line --no-loaded-latency --no-probe --steps 8 --warmup 2"
val() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], (d.get('step_roofline') or {}).get('us_per_step'))" $1 "$2"; }
for cfg in 2 4 1; do
  for v in base g64 g256 base g64 g256; do
    if [ $v = base ]; then unset LVX_LIB_PATH; else export LVX_LIB_PATH=llmvox_amd/libllmvox_hip_$v.so; fi
    $B --config $cfg > $O/c${cfg}_$v.jsonl 2> $O/c${cfg}_$v.err || { echo "bench c$cfg $v failed"; tail -5 $O/c${cfg}_$v.err; exit 1; }
    val $O/c${cfg}_$v.jsonl "c$cfg $v"
  done
done
