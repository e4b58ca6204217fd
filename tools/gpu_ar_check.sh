#!/bin/bash
# AR iteration: bf16 / batched / teacher-forced GPU tests, the B = 32 step timeline at t = 512,
# step sweeps at three positions and the default bench line (no CPU baseline / parity line)
set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=.
O=gpurun_out/archeck.txt; : > $O
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_bf16.py tests/test_gpu_batched.py tests/test_gpu_teacher_forced.py} -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/artests.log 2>&1
rc=$?; grep -E "teacher-forced|passed|failed|Error" gpurun_out/artests.log | tail -12; [ $rc = 0 ] || { tail -40 gpurun_out/artests.log; exit $rc; }
timeout -k 10 120 python tools/step_timeline.py 32 512 1 2>&1 | grep -v amdgpu.ids >> $O || exit 1
for P in 0 512 896; do timeout -k 10 120 python tools/step_sweep.py 32 $P "" 2>&1 | grep -v amdgpu.ids >> $O || exit 1; done
timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-line 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['roofline']['avg_us'], d['codec_roofline']['avg_ms'], d['p50_first_chunk_latency_ms'])" >> $O || exit 1
cat $O
