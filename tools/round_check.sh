#!/bin/bash
# One GPU call: parity tests, smoke, bench configs[1] and configs[2]. Each step time-limited,
# chained so the first failure ends the call.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
 && timeout -k 10 300 python bench.py > gpurun_out/bench_c1.jsonl 2> gpurun_out/bench_c1.err \
 && timeout -k 10 300 python bench.py --streams 32 --steps 2 --no-cpu-baseline > gpurun_out/bench_c2.jsonl 2> gpurun_out/bench_c2.err
rc=$?
tail -3 gpurun_out/tests.log
echo "EXIT $rc"
exit $rc
