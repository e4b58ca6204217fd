#!/bin/bash
# Round-2 measurement call: the default bench line (configs[2], the driver's arguments), then one
# FETCH_SIZE PMC pass of the full bench (faulthandler on: bench.py enables it) to root-cause the
# round-1 profiler segfault, then the codec MFMA-busy pass.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
O=gpurun_out/r02; mkdir -p $O
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.jsonl 2> $O/bench_default.err || { echo BENCH_FAIL; tail -20 $O/bench_default.err; exit 1; }
tail -c 1500 $O/bench_default.jsonl
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/f_full -o run --output-format csv -- python3 bench.py --steps 20 --warmup 0 --no-cpu-baseline --no-parity-line > $O/f_full.log 2>&1
echo "pmc full rc=$?"; tail -40 $O/f_full.log
