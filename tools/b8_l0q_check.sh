# round 6: layer 0's c_attn from the q0 tables at 4 <= B <= 8 (now the default): GPU tests of the select
# and table paths, the step sweep against l0q 0, configs[4] and configs[1] lines
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
O=gpurun_out/b8l0q_check.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_batched.py tests/test_gpu_select.py tests/test_gpu_teacher_forced.py tests/test_gpu_fp8.py > $O 2>&1 || { tail -30 $O; exit 1; }
tail -2 $O
export LVX_SWEEP_STREAM=1
LVX_SWEEP_KV=fp8 timeout -k 10 200 python tools/step_sweep.py 8 384 'l0q=0' '' 'l0q=0' '' >> $O 2>&1 || exit 1
timeout -k 10 300 python bench.py --config 4 --steps 8 --no-cpu-baseline > gpurun_out/cfg4_l0q.jsonl 2> gpurun_out/cfg4_l0q.err || { tail -5 gpurun_out/cfg4_l0q.err; exit 1; }
grep -v amdgpu.ids $O | tail -4
python3 -c "
import json; d=json.loads(open('gpurun_out/cfg4_l0q.jsonl').read().strip().splitlines()[-1]); print('cfg4', d['value'], d['ms_per_step'], d.get('p50_first_chunk_latency_ms'), d['step_roofline']['us_per_step'])"
