#!/bin/bash
# End-of-round refresh: GPU tests + smoke, PMC FETCH/WRITE passes of the roofline probes (B = 1 at
# 1024 and 2048 positions, B = 32, fp8 KV at B = 8), then bench lines of every config (configs[1]
# with the CPU baseline; their roofline.traffic read from this call's PMC passes) and kernel-trace
# stats of configs[1]/[2].
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
mkdir -p gpurun_out
# STAGE=1: tests, smoke, PMC passes; STAGE=2: bench lines + kernel traces (copy stage 1's
# gpurun_out/pmc_traffic.json to profiles/ first); unset: both in one call
run() { # tag, timeout, rocprof args..., -- cmd
  local tag=$1 t=$2; shift 2
  timeout -s KILL $t rocprofv3 "$@" > $O/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 $O/$tag.log; exit 1; }
}
csv() { find $O/$1 -name "*counter_collection.csv" | head -1; }
# tag, pmc key prefix, target...
pmc() {
  local tag=$1 key=$2; shift 2
  run f_$tag 120 --pmc FETCH_SIZE -d $O/f_$tag -o run --output-format csv -- "$@"
  run w_$tag 120 --pmc WRITE_SIZE -d $O/w_$tag -o run --output-format csv -- "$@"
  python3 tools/pmc_traffic.py $(csv f_$tag) $(csv w_$tag) $key gpurun_out/pmc_traffic.json > gpurun_out/pmc_$tag.txt || exit 1
}
if [ "$STAGE" != "2" ]; then
O=gpurun_out/prof_round; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -20 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
pmc b1 bf16 python3 bench.py --no-cpu-baseline --steps 1 --probe-pos 1024
pmc b32 bf16/B32 python3 tools/probe_pmc.py 32 512
pmc c3 bf16/P2048 python3 tools/probe_pmc.py 1 2048
pmc c4 bf16/kvfp8/B8 python3 tools/probe_pmc.py 8 1024 fp8
cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
cat gpurun_out/pmc_b1.txt gpurun_out/pmc_b32.txt gpurun_out/pmc_c3.txt gpurun_out/pmc_c4.txt
fi
[ "$STAGE" == "1" ] && { echo STAGE1_OK; exit 0; }
O=gpurun_out/prof_round2; mkdir -p $O
CPU=1 bash tools/gpu_configs.sh || exit 1
run kt_c1 300 --kernel-trace --stats -d $O/kt_c1 -o run --output-format csv -- python3 bench.py --no-cpu-baseline
run kt_c2 300 --kernel-trace --stats -d $O/kt_c2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --config 2 --steps 2
echo FINAL_OK
