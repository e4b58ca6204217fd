#!/bin/bash
# A/B: HIP runtime graph knobs (DEBUG_CLR_GRAPH_PACKET_CAPTURE, DEBUG_HIP_GRAPH_BATCH_SIZE), alternating
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
O=gpurun_out/abenv; mkdir -p $O
B="timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity-line --no-loaded-latency --no-probe --steps 8 --warmup 2"
val() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], (d.get('step_roofline') or {}).get('us_per_step'))" $1 "$2"; }
for cfg in 2 1; do
  for v in base pc0 pc1 bs8 bs1024 base pc0 pc1 bs8 bs1024; do
    unset DEBUG_CLR_GRAPH_PACKET_CAPTURE DEBUG_HIP_GRAPH_BATCH_SIZE
    case $v in pc0) export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0;; pc1) export DEBUG_CLR_GRAPH_PACKET_CAPTURE=1;;
      bs8) export DEBUG_HIP_GRAPH_BATCH_SIZE=8;; bs1024) export DEBUG_HIP_GRAPH_BATCH_SIZE=1024;; esac
    $B --config $cfg > $O/c${cfg}_$v.jsonl 2> $O/c${cfg}_$v.err || { echo "bench c$cfg $v failed"; tail -5 $O/c${cfg}_$v.err; exit 1; }
    val $O/c${cfg}_$v.jsonl "c$cfg $v"
  done
done
