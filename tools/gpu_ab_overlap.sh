#!/bin/bash
# host-paced codec overlap (--codec-overlap) vs serial, alternating
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
O=gpurun_out/abovl2; mkdir -p $O
B="timeout -k 10 300 python bench.py --no-cpu-baseline --no-loaded-latency --no-probe --steps 8 --warmup 2"
val() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d.get('parity_mode_fp32') or {}; print(sys.argv[2], d['value'], d['ms_per_step'], (d.get('step_roofline') or {}).get('us_per_step'), 'parity', p.get('value'), p.get('ms_per_step'), p.get('ar_ms_per_chunk'))" $1 "$2"; }
for v in serial ovl serial ovl; do
  a=""; [ $v = ovl ] && a="--codec-overlap"
  $B $a > $O/c2_$v.jsonl 2> $O/c2_$v.err || { echo "bench c2 $v failed"; tail -5 $O/c2_$v.err; exit 1; }
  val $O/c2_$v.jsonl "c2 $v"
done
for cfg in 1 4; do
  for v in serial ovl serial ovl; do
    a=""; [ $v = ovl ] && a="--codec-overlap"
    $B --no-parity-line --config $cfg $a > $O/c${cfg}_$v.jsonl 2> $O/c${cfg}_$v.err || { echo "bench c$cfg $v failed"; tail -5 $O/c${cfg}_$v.err; exit 1; }
    val $O/c${cfg}_$v.jsonl "c$cfg $v"
  done
done
