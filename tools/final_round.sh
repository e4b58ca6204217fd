#!/bin/bash
# End-of-round refresh: GPU tests + smoke, bench lines of every config (configs[1] with the CPU
# baseline), kernel-trace stats of configs[1]/[2], PMC FETCH/WRITE passes of the roofline probes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -20 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
CPU=1 bash tools/gpu_configs.sh || exit 1
O=gpurun_out/prof_round; rm -rf $O; mkdir -p $O
run() { # tag, timeout, rocprof args..., -- cmd
  local tag=$1 t=$2; shift 2
  timeout -s KILL $t rocprofv3 "$@" > $O/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 $O/$tag.log; exit 1; }
}
run kt_c1 300 --kernel-trace --stats -d $O/kt_c1 -o run --output-format csv -- python3 bench.py --no-cpu-baseline
run kt_c2 300 --kernel-trace --stats -d $O/kt_c2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --config 2 --steps 2
run f_b1 120 --pmc FETCH_SIZE -d $O/f_b1 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --probe-pos 1024
run w_b1 120 --pmc WRITE_SIZE -d $O/w_b1 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --probe-pos 1024
run f_b32 120 --pmc FETCH_SIZE -d $O/f_b32 -o run --output-format csv -- python3 tools/probe_pmc.py 32 512
run w_b32 120 --pmc WRITE_SIZE -d $O/w_b32 -o run --output-format csv -- python3 tools/probe_pmc.py 32 512
python3 tools/pmc_traffic.py $(find gpurun_out/prof_round/f_b1 -name "*counter_collection.csv" | head -1) $(find gpurun_out/prof_round/w_b1 -name "*counter_collection.csv" | head -1) bf16 gpurun_out/pmc_traffic.json > gpurun_out/pmc_b1.txt || exit 1
python3 tools/pmc_traffic.py $(find gpurun_out/prof_round/f_b32 -name "*counter_collection.csv" | head -1) $(find gpurun_out/prof_round/w_b32 -name "*counter_collection.csv" | head -1) bf16/B32 gpurun_out/pmc_traffic.json > gpurun_out/pmc_b32.txt || exit 1
cat gpurun_out/pmc_b1.txt gpurun_out/pmc_b32.txt
echo FINAL_OK
