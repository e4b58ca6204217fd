# round 6: the mlp c_proj at B <= ln_max as 2 K slices of 1,536 (2 pending copies for the LayerNorm
# prologues to fold; build LVX_YCS=2) against 4 slices of 768 (production); alternating on one box
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
O=gpurun_out/ycs.txt
: > $O
V=${V:-llmvox_amd/libllmvox_hip_ycs2.so}
for i in 1 2; do
for lib in llmvox_amd/libllmvox_hip.so $V; do
echo "## $lib" >> $O
LVX_LIB_PATH=$lib LVX_SWEEP_STREAM=1 LVX_SWEEP_KV=fp8 timeout -k 10 200 python tools/step_sweep.py 8 384 '' >> $O 2>&1 || exit 1
LVX_LIB_PATH=$lib LVX_SWEEP_STREAM=1 timeout -k 10 200 python tools/step_sweep.py 8 384 '' >> $O 2>&1 || exit 1
LVX_LIB_PATH=$lib LVX_SWEEP_STREAM=1 timeout -k 10 200 python tools/step_sweep.py 4 384 '' >> $O 2>&1 || exit 1
done
done
for lib in llmvox_amd/libllmvox_hip.so $V; do
LVX_LIB_PATH=$lib timeout -k 10 300 python tools/l0q_accuracy.py fp8 8 'l0q=1' >> $O 2>&1 || exit 1
LVX_LIB_PATH=$lib timeout -k 10 300 python bench.py --config 4 --steps 20 --warmup 5 --no-cpu-baseline --no-probe --no-loaded-latency > gpurun_out/ycs_c4.jsonl 2> gpurun_out/ycs_c4.err || { tail -5 gpurun_out/ycs_c4.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('configs[4] $lib', d['value'], d['ms_per_step'], d['step_roofline']['us_per_step'])" gpurun_out/ycs_c4.jsonl >> $O
done
LVX_LIB_PATH=$V timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_batched.py tests/test_gpu_select.py tests/test_gpu_fp8.py tests/test_gpu_teacher_forced.py >> $O 2>&1 || { tail -20 $O; exit 1; }
grep -v amdgpu.ids $O | grep -v "^\.\|^$"
