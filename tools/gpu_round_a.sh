#!/bin/bash
# round end, part 1 of 2 (one gpurun call): the -m gpu suite, smoke(), then tools/prof_round.sh for configs[2]
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -2 gpurun_out/tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; [ $rc = 0 ] || exit $rc
TAG=${TAG:-r06} bash tools/prof_round.sh || exit 1
echo PART1_OK
