#!/bin/bash
# PMC FETCH_SIZE / WRITE_SIZE passes of the roofline probes at B = 32, KV position 512
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
O=gpurun_out/prof_b32; rm -rf $O; mkdir -p $O
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $O/$c -o run --output-format csv -- python3 tools/probe_pmc.py ${S:-32} ${P:-512} ${KV:-bf16} > $O/$c.log 2>&1 || { echo "FAIL $c"; exit 1; }
done
