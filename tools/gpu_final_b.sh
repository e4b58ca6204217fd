#!/bin/bash
# round-end call 2 of 2: kernel trace of the default bench command and the driver's bench line
# (profiles/r04), then tools/gpu_round_lines.sh (configs 1/3/4, the 60-s steady state, the 2-rank
# gloo rehearsals, the FETCH_SIZE pass with the parity line). Outputs under gpurun_out/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
O=gpurun_out/r04b; mkdir -p $O
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --steps 20 --warmup 0 --no-cpu-baseline --no-parity-line > $O/kt.log 2>&1 || { echo "FAIL kt"; tail -30 $O/kt.log; exit 1; }
find $O/kt -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
python3 tools/probe_trace.py $(find $O/kt -name "*kernel_trace.csv" | head -1) > $O/probe_trace.txt || exit 1
cat $O/probe_trace.txt
rm -rf $O/kt
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.jsonl 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
tail -c 300 $O/bench.jsonl
bash tools/gpu_round_lines.sh || exit 1
echo FINAL_B_OK
