#!/bin/bash
# codec on a second stream (--codec-overlap) under HIP runtime settings: does any avoid the
# per-dispatch cost a second stream puts on the AR chain?
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
O=gpurun_out/abovl; mkdir -p $O
B="timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity-line --no-loaded-latency --no-probe --steps 8 --warmup 2"
val() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], (d.get('step_roofline') or {}).get('us_per_step'))" $1 "$2"; }
run() { local tag=$1; shift; env "$@" $B $OVL > $O/$tag.jsonl 2> $O/$tag.err || { echo "bench $tag failed"; tail -5 $O/$tag.err; exit 1; }; val $O/$tag.jsonl $tag; }
OVL=""; run serial X=1
OVL="--codec-overlap"; run ovl X=1
run ovl_pc0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run ovl_q8 GPU_MAX_HW_QUEUES=8
run ovl_q2 GPU_MAX_HW_QUEUES=2
run ovl_q1 GPU_MAX_HW_QUEUES=1
run ovl_async DEBUG_HIP_FORCE_ASYNC_QUEUE=1
OVL=""; run serial2 X=1
