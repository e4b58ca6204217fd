#!/bin/bash
# Round profiles: kernel-trace stats of bench configs[1] and configs[2], PMC FETCH/WRITE passes of
# the roofline probes (B = 1 at KV position 1024, B = 32 at 512), each step time-limited.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
O=gpurun_out/prof_round
rm -rf $O; mkdir -p $O
run() { # tag, timeout, rocprof args..., -- cmd
  local tag=$1 t=$2; shift 2
  timeout -s KILL $t rocprofv3 "$@" > $O/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 $O/$tag.log; exit 1; }
}
run kt_c1 300 --kernel-trace --stats -d $O/kt_c1 -o run --output-format csv -- python3 bench.py --no-cpu-baseline
run kt_c2 300 --kernel-trace --stats -d $O/kt_c2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --config 2 --steps 2
run f_b1 120 --pmc FETCH_SIZE -d $O/f_b1 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --probe-pos 1024
run w_b1 120 --pmc WRITE_SIZE -d $O/w_b1 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --probe-pos 1024
run f_b32 160 --pmc FETCH_SIZE -d $O/f_b32 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --streams 32 --steps 1 --probe-pos 512
run w_b32 160 --pmc WRITE_SIZE -d $O/w_b32 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --streams 32 --steps 1 --probe-pos 512
echo OK
