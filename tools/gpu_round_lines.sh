#!/bin/bash
# round-end bench lines on one GPU (outputs under gpurun_out/lines): configs[1], configs[3],
# configs[4] (8 x 256-token steps and the 60-s steady state), the 2-rank gloo rehearsal of the
# multi-rank path (configs[2] and configs[3] with their RCCL-shaped exchanges), and last a
# FETCH_SIZE PMC pass over the full default bench command, fp32 parity line included (VERDICT r02
# item 8: the segfault seen in round 2 under --pmc with the parity line)
set -o pipefail
export PYTHONPATH=.
O=gpurun_out/lines; mkdir -p $O
line() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d['value'], 'tok/s', d['ms_per_step'], 'ms/step; p50', d.get('p50_first_chunk_latency_ms'), '; step_rl', (d.get('step_roofline') or {}).get('us_per_step'), (d.get('step_roofline') or {}).get('frac'), '; roof', (d.get('roofline') or {}).get('kernel'), (d.get('roofline') or {}).get('frac'), '; steady', (d.get('steady_state') or {}).get('spread'))" $1; }
timeout -k 10 300 python bench.py --config 1 --no-cpu-baseline --no-parity-line > $O/cfg1.jsonl 2> $O/cfg1.err || { tail -5 $O/cfg1.err; exit 1; }
line $O/cfg1.jsonl
timeout -k 10 300 python bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline > $O/cfg3.jsonl 2> $O/cfg3.err || { tail -5 $O/cfg3.err; exit 1; }
line $O/cfg3.jsonl
timeout -k 10 300 python bench.py --config 4 --steps 8 --no-cpu-baseline > $O/cfg4.jsonl 2> $O/cfg4.err || { tail -5 $O/cfg4.err; exit 1; }
line $O/cfg4.jsonl
timeout -k 10 300 python bench.py --config 4 --seconds 60 --no-cpu-baseline --no-probe > $O/cfg4_60s.jsonl 2> $O/cfg4_60s.err || { tail -5 $O/cfg4_60s.err; exit 1; }
line $O/cfg4_60s.jsonl
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --no-probe --dist-backend gloo > $O/dist2.jsonl 2> $O/dist2.err || { tail -5 $O/dist2.err; exit 1; }
line $O/dist2.jsonl
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --config 3 --steps 1 --warmup 1 --no-cpu-baseline --no-probe --dist-backend gloo --sched cs=0 > $O/dist2_c3.jsonl 2> $O/dist2_c3.err || { tail -5 $O/dist2_c3.err; exit 1; }
line $O/dist2_c3.jsonl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d $O/pmcpar -o run --output-format csv -- python3 bench.py --steps 4 --no-cpu-baseline --null-stream > $O/pmc_parity.log 2>&1
rc=$?; echo "pmc FETCH_SIZE pass with the parity line: rc $rc"; tail -3 $O/pmc_parity.log | cut -c1-400
rm -rf $O/pmcpar
exit $rc
