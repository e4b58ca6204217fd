#!/bin/bash
# codec timing + SQ counters of the large-M GEMM (one PMC pass, <= 8 SQ counters) + codec parity tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
O=gpurun_out/codec; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_codec_bf16.py tests/test_gpu_large_dumps.py -m gpu -x -q --timeout 200 --timeout-method thread -k "codec or Codec" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python tools/codec_probe.py 10 bf16 || exit 1
timeout -k 10 120 python tools/codec_probe.py 3 fp32 || exit 1
if [ -n "$PMC" ]; then
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES -d $O/sq -o run --output-format csv -- python3 tools/codec_probe.py 3 bf16 > $O/sq.log 2>&1 || { echo PMC_FAIL; tail -5 $O/sq.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/codec/sq/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0][:70]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k] += 1
for k, v in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:8]:
    w = v.get("SQ_WAVE_CYCLES", 1)
    print(k, {c: round(x / w, 3) for c, x in v.items() if c != "SQ_WAVE_CYCLES"}, "lds_conf/insts", round(v.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, v.get("SQ_INSTS_LDS", 1)), 3))
PY
rm -rf $O/sq
fi
