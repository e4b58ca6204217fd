#!/bin/bash
# round 4, third GPU call: the -m gpu suite (fp32 per-slot attention now default), fp32 step A/B,
# configs[4] 16-wave attention A/B, CU-partitioned codec overlap A/B, then the --pmc reproducer
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc = 0 ] || exit $rc
LVX_SWEEP_STREAM=1 LVX_SWEEP_W=fp32 timeout -k 10 200 python tools/step_sweep.py 32 384 'exp=0' 'exp=16384' 'exp=0' > $O/sweep_fp32.txt 2>&1 || { tail $O/sweep_fp32.txt; exit 1; }
cat $O/sweep_fp32.txt
LVX_SWEEP_STREAM=1 LVX_SWEEP_KV=fp8 timeout -k 10 200 python tools/step_sweep.py 8 384 'exp=0' 'exp=8192' 'exp=0' 'exp=8192' > $O/sweep_b8.txt 2>&1 || { tail $O/sweep_b8.txt; exit 1; }
cat $O/sweep_b8.txt
LVX_SWEEP_STREAM=1 timeout -k 10 200 python tools/step_sweep.py 8 384 'exp=0' 'exp=8192' > $O/sweep_b8_bf16.txt 2>&1 || { tail $O/sweep_b8_bf16.txt; exit 1; }
cat $O/sweep_b8_bf16.txt
B="timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity-line --no-loaded-latency --no-probe --steps 8 --warmup 2"
val() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['step_roofline']['us_per_step'], d['codec_roofline']['avg_ms'])" $1 "$2"; }
for v in "base:" "cus32s:--codec-cus 32" "cus48s:--codec-cus 48" "cus32c:--codec-cus 32 --cu-layout contig" "base2:"; do
  tag=${v%%:*}; a=${v#*:}
  $B $a > $O/b_$tag.jsonl 2> $O/b_$tag.err || { echo "bench $tag failed"; tail -5 $O/b_$tag.err; exit 1; }
  val $O/b_$tag.jsonl $tag
done
for v in "c4:" "c4nw16:--opt exp=8192"; do
  tag=${v%%:*}; a=${v#*:}
  $B --config 4 $a > $O/b_$tag.jsonl 2> $O/b_$tag.err || { echo "bench $tag failed"; tail -5 $O/b_$tag.err; exit 1; }
  val $O/b_$tag.jsonl $tag
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-loaded-latency --no-probe --steps 4 --warmup 1 > $O/b_parity.jsonl 2> $O/b_parity.err || { tail -5 $O/b_parity.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/b_parity.jsonl').read().strip().splitlines()[-1]); print('headline', d['value'], 'parity', d['parity_mode_fp32'])"
for spec in "3 16 1 0" "3 416 1 0" "3 416 20 0" "3 416 320 1"; do
  set -- $spec
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d /tmp/pmcrep -o run --output-format csv -- ./tools/pmc_graph_repro $1 $2 $3 $4 > $O/repro_pmc_m$1_k$2_r$3_s$4.log 2>&1
  rc=$?
  echo "repro mode $1 kernels $2 reps $3 small $4 under --pmc FETCH_SIZE: rc=$rc"; tail -2 $O/repro_pmc_m$1_k$2_r$3_s$4.log
  [ $rc = 0 ] || exit 0
done
