#!/bin/bash
# Round-end measurement in one gpurun call: the -m gpu suite, then tools/prof_round.sh (PMC traffic,
# MFMA busy, kernel trace and the driver's bench line) and tools/gpu_round_lines.sh (configs 1/3/4,
# the 60-s steady state, the 2-rank rehearsals, the PMC pass with the parity line). Stops at the
# first failure. Outputs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -2 gpurun_out/tests.log; [ $rc = 0 ] || exit $rc
TAG=${TAG:-r06} bash tools/prof_round.sh || exit 1
bash tools/gpu_round_lines.sh || exit 1
echo FINAL_OK
