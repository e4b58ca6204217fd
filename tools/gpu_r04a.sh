#!/bin/bash
# round 4, first GPU call: the -m gpu suite, the default bench line, the persistent step A/B and its
# timeline, and the library-free --pmc graph-replay check (tools/pmc_graph_repro.hip)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.jsonl 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 2500 $O/bench.jsonl
LVX_SWEEP_STREAM=1 timeout -k 10 200 python tools/step_sweep.py 32 384 'persist=0' 'persist=1' 'persist=0' 'persist=1' > $O/sweep.txt 2>&1 || { tail $O/sweep.txt; exit 1; }
cat $O/sweep.txt
timeout -k 10 120 python tools/persist_timeline.py 32 512 > $O/persist_timeline.txt 2>&1 || { tail $O/persist_timeline.txt; exit 1; }
cat $O/persist_timeline.txt
for m in 1 0 2; do
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d /tmp/pmcrep$m -o run --output-format csv -- ./tools/pmc_graph_repro $m > $O/repro_pmc_mode$m.log 2>&1
  rc=$?
  echo "repro mode $m under --pmc FETCH_SIZE: rc=$rc"; tail -3 $O/repro_pmc_mode$m.log
  [ $rc = 0 ] || exit 0   # a fault ends the call here (the log is the result)
done
