#!/bin/bash
# the -m gpu suite and smoke() on the current tree (outputs under gpurun_out/suite)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
O=gpurun_out/suite; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -3 $O/smoke.log; exit $rc
