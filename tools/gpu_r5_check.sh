#!/bin/bash
# round-5 check: the -m gpu suite (or SEL), configs[2] (LINE2_ARGS), configs[3] overlapped and serial,
# the 2-rank gloo rehearsal of the overlapped N > 1 schedule. Outputs under gpurun_out/${OUT:-r5}.
set -o pipefail
export PYTHONPATH=.
O=gpurun_out/${OUT:-r5}; mkdir -p $O
timeout -k 10 600 python -u -m pytest ${SEL:-tests/} -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline ${LINE2_ARGS:-} > $O/c2.jsonl 2> $O/c2.err || { tail -20 $O/c2.err; exit 1; }
timeout -k 10 300 python bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline > $O/c3.jsonl 2> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
timeout -k 10 300 python bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline --serial-codec --no-probe > $O/c3s.jsonl 2> $O/c3s.err || { tail -20 $O/c3s.err; exit 1; }
[ -n "$NODIST" ] && exit 0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-probe --dist-backend gloo > $O/dist2.jsonl 2> $O/dist2.err || { tail -20 $O/dist2.err; exit 1; }
echo done
