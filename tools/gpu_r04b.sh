#!/bin/bash
# round 4, second GPU call: persistent-step prefetch-timing A/B (option pexp), the PMC traffic
# passes of the default bench (c_proj XCD order), and the --pmc reproducer characterised by stream
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_persist.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc = 0 ] || exit $rc
LVX_SWEEP_STREAM=1 timeout -k 10 300 python tools/step_sweep.py 32 384 'persist=0' 'persist=1' 'persist=1,pexp=2' 'persist=1,pexp=4' 'persist=1,pexp=6' 'persist=0' > $O/sweep.txt 2>&1 || { tail $O/sweep.txt; exit 1; }
cat $O/sweep.txt
for px in 2 6; do
  LVX_PEXP=$px timeout -k 10 120 python tools/persist_timeline.py 32 512 > $O/persist_timeline_pexp$px.txt 2>&1 || { tail $O/persist_timeline_pexp$px.txt; exit 1; }
  tail -30 $O/persist_timeline_pexp$px.txt
done
run() { local tag=$1 t=$2; shift 2
  timeout -s KILL $t rocprofv3 "$@" > $O/$tag.log 2>&1 || { echo "FAIL $tag rc=$?"; tail -30 $O/$tag.log; exit 1; }; }
csv() { find $O/$1 -name "*counter_collection.csv" | head -1; }
PARGS="--steps 20 --warmup 0 --no-cpu-baseline --no-parity-line --no-loaded-latency --null-stream"
run f 300 --pmc FETCH_SIZE -d $O/f -o run --output-format csv -- python3 bench.py $PARGS
run w 300 --pmc WRITE_SIZE -d $O/w -o run --output-format csv -- python3 bench.py $PARGS
python3 tools/pmc_traffic.py $(csv f) $(csv w) bf16/kvbf16/B32/P512 $O/pmc_traffic.json > $O/pmc_traffic.txt || exit 1
cat $O/pmc_traffic.txt
rm -rf $O/f $O/w
for spec in "3 416 320 0" "2 416 320 0" "1 16 1 0" "1 416 320 1"; do
  set -- $spec
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d /tmp/pmcrep -o run --output-format csv -- ./tools/pmc_graph_repro $1 $2 $3 $4 > $O/repro_pmc_m$1_k$2_r$3_s$4.log 2>&1
  rc=$?
  echo "repro mode $1 kernels $2 reps $3 small $4 under --pmc FETCH_SIZE: rc=$rc"; tail -2 $O/repro_pmc_m$1_k$2_r$3_s$4.log
  [ $rc = 0 ] || exit 0
done
