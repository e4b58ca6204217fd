#!/bin/bash
# A/B: DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 vs the runtime default, configs[1] / [4] / [2], alternating
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
O=gpurun_out/abenv2; mkdir -p $O
B="timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity-line --no-loaded-latency --no-probe --steps 8 --warmup 2"
val() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], (d.get('step_roofline') or {}).get('us_per_step'), d.get('p50_first_chunk_latency_ms'))" $1 "$2"; }
for cfg in 1 4 2; do
  for v in base pc0 base pc0 base pc0; do
    unset DEBUG_CLR_GRAPH_PACKET_CAPTURE
    [ $v = pc0 ] && export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
    $B --config $cfg > $O/c${cfg}_$v.jsonl 2> $O/c${cfg}_$v.err || { echo "bench c$cfg $v failed"; tail -5 $O/c${cfg}_$v.err; exit 1; }
    val $O/c${cfg}_$v.jsonl "c$cfg $v"
  done
done
