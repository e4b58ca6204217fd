#!/bin/bash
# Which launches fault inside rocprofv3's --pmc dispatch hook? (round-1 VERDICT item 8)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
O=gpurun_out/r02/segv; mkdir -p $O
i=0
for S in 9 16; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d /tmp/segv$i -o run --output-format csv -- python3 bench.py --config 2 --streams $S --dtype fp32 --steps 1 --warmup 0 --no-cpu-baseline --no-probe > $O/b$i.log 2>&1
  echo "fp32 B=$S pmc rc=$?"
done
timeout -s KILL 200 rocprofv3 --kernel-trace -d /tmp/segvk -o run --output-format csv -- python3 bench.py --config 2 --dtype fp32 --steps 1 --warmup 0 --no-cpu-baseline --no-probe > $O/kt.log 2>&1
echo "fp32 B=32 kernel-trace rc=$?"
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE -d /tmp/segvg -o run --output-format csv -- python3 bench.py --config 2 --dtype fp32 --steps 1 --warmup 0 --no-cpu-baseline --no-probe > $O/g.log 2>&1
echo "fp32 B=32 pmc GRBM rc=$?"
