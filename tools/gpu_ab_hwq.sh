#!/bin/bash
# A/B: GPU_MAX_HW_QUEUES 1 / 2 vs the default 4 (configs[2], configs[1]), alternating on one box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
O=gpurun_out/abhwq; mkdir -p $O
B="timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity-line --no-loaded-latency --no-probe --steps 8 --warmup 2"
val() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['step_roofline']['us_per_step'], d['codec_roofline']['avg_ms'], d.get('p50_first_chunk_latency_ms'))" $1 "$2"; }
for q in 4 1 2 4 1; do
  GPU_MAX_HW_QUEUES=$q $B > $O/b_q$q.jsonl 2> $O/b_q$q.err || { echo "bench q$q failed"; tail -5 $O/b_q$q.err; exit 1; }
  val $O/b_q$q.jsonl "c2 q$q"
done
for q in 4 1 4 1; do
  GPU_MAX_HW_QUEUES=$q $B --config 1 > $O/c1_q$q.jsonl 2> $O/c1_q$q.err || { echo "bench c1 q$q failed"; tail -5 $O/c1_q$q.err; exit 1; }
  val $O/c1_q$q.jsonl "c1 q$q"
done
