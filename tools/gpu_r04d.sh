#!/bin/bash
# round 4: bf16x3 split fp32 codec GEMMs: PCM against exact fp32 and the reference fixtures, codec
# timing A/B, fp32 parity line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_codec_variants.py tests/test_gpu_large_dumps.py tests/test_gpu_parity.py -x -v -s --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "split|LDS-DMA|passed|failed|Error" $O/tests.log | tail -12; [ $rc = 0 ] || exit $rc


timeout -k 10 200 python tools/codec_probe.py 10 fp32 codec_g3f=2 32x256,2x1280 > $O/probe_g3f2.txt 2>&1 && cat $O/probe_g3f2.txt || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python tools/codec_probe.py 5 fp32 codec_g3f=2 32x256 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_codec_fp32_split.csv \;
head -12 $O/kernel_stats_codec_fp32_split.csv | cut -c1-200
timeout -k 10 300 python bench.py --no-cpu-baseline --no-loaded-latency --no-probe --steps 4 --warmup 1 > $O/b_parity.jsonl 2> $O/b_parity.err || { tail -5 $O/b_parity.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/b_parity.jsonl').read().strip().splitlines()[-1]); print('headline', d['value'], 'parity', d['parity_mode_fp32'])"
