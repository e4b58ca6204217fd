#!/bin/bash
# round-end call 1 of 2: the -m gpu suite, then tools/prof_round.sh (PMC traffic, MFMA busy, kernel
# trace, the driver's bench line). Outputs under gpurun_out/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -2 gpurun_out/tests.log; [ $rc = 0 ] || exit $rc
TAG=${TAG:-r04} bash tools/prof_round.sh || exit 1
echo FINAL_A_OK
