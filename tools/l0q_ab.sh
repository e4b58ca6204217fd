# round 6: layer 0's c_attn from the q0 tables (option l0q) -- step time and accuracy against the reference
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
export LVX_SWEEP_STREAM=1
timeout -k 10 200 python tools/step_sweep.py 32 384 'l0q=0' 'l0q=1' 'l0q=0' 'l0q=1' || exit 1
timeout -k 10 200 python tools/step_sweep.py 16 384 'l0q=0' 'l0q=1' || exit 1
timeout -k 10 200 python tools/step_sweep.py 32 896 'l0q=0' 'l0q=1' || exit 1
timeout -k 10 300 python tools/l0q_accuracy.py bf16 || exit 1
timeout -k 10 300 python tools/l0q_accuracy.py fp8 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_batched.py tests/test_gpu_select.py tests/test_gpu_teacher_forced.py
