#!/bin/bash
# step-time A/B of library options: SWEEP="B P0 'opt=v' ..." lines, then optional pytest selection
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
O=gpurun_out/sweep; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
echo "$SWEEP" | while read -r line; do
  [ -z "$line" ] && continue
  eval "timeout -k 10 300 python tools/step_sweep.py $line" >> $O/sweep.txt 2>&1 || { echo "SWEEP FAIL $line"; tail -5 $O/sweep.txt; exit 1; }
done
cat $O/sweep.txt
