#!/bin/bash
# Round measurement refresh (round 2+; TAG defaults to the current round): PMC passes over the driver's default bench command
# (configs[2], --steps 20: the roofline probe at KV position 2,560), kernel-trace stats of it, and
# the bench line itself (BENCH_ARGS; configs[4]: ARGS="--config 4 ..." KEY=bf16/kvfp8/B8/P512
# CKEY=fp8/F2048/L256 BENCH_ARGS="--config 4 --steps 20 --warmup 5"). Outputs under gpurun_out/$TAG;
# copy the summaries to profiles/.
#   FETCH_SIZE and WRITE_SIZE passes  -> tools/pmc_traffic.py  -> pmc_traffic.json
#   SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE pass -> tools/pmc_codec.py -> pmc_codec.json
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
TAG=${TAG:-r06}
O=gpurun_out/$TAG; mkdir -p $O
# PMC passes launch the steps one by one on the null stream (--null-stream): with the default
# side-stream HIP-graph replay, rocprofv3 --pmc segfaults in its own thread (profiles/r03/pmc_segv_graph_replay.log);
# per-dispatch counters do not depend on how the dispatch was submitted
ARGS=${ARGS:-"--steps 20 --warmup 0 --no-cpu-baseline --no-parity-line"}
PARGS=${PARGS:-"$ARGS --null-stream --no-dist-world1"}
KEY=${KEY:-bf16/kvbf16/B32/P512}
CKEY=${CKEY:-bf16/F8192/L256}
run() { # tag, timeout, rocprof args..., -- cmd
  local tag=$1 t=$2; shift 2
  timeout -s KILL $t rocprofv3 "$@" > $O/$tag.log 2>&1 || { echo "FAIL $tag"; tail -30 $O/$tag.log; exit 1; }
}
csv() { find $O/$1 -name "*counter_collection.csv" | head -1; }
run f 300 --pmc FETCH_SIZE -d $O/f -o run --output-format csv -- python3 bench.py $PARGS
run w 300 --pmc WRITE_SIZE -d $O/w -o run --output-format csv -- python3 bench.py $PARGS
python3 tools/pmc_traffic.py $(csv f) $(csv w) $KEY $O/pmc_traffic.json > $O/pmc_traffic.txt || exit 1
cat $O/pmc_traffic.txt
rm -rf $O/f $O/w  # raw per-dispatch CSVs: too large to merge back (gpurun_out <= 64 MiB)
run m 300 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/m -o run --output-format csv -- python3 bench.py $PARGS
python3 tools/pmc_codec.py $(csv m) $CKEY $O/pmc_codec.json || exit 1
rm -rf $O/m
run kt 300 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py $ARGS
find $O/kt -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
python3 tools/probe_trace.py $(find $O/kt -name "*kernel_trace.csv" | head -1) > $O/probe_trace.txt || exit 1
cat $O/probe_trace.txt
rm -rf $O/kt
timeout -k 10 400 python bench.py ${BENCH_ARGS:---gpus 1 --steps 20 --warmup 5} > $O/bench.jsonl 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
tail -c 600 $O/bench.jsonl
echo PROF_OK
