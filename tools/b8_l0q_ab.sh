# round 6: layer 0's c_attn from the q0 tables at 4 <= B <= 8 (the default since) against the GEMM with the
# select in its prologue (l0q 0): step time (tools/step_sweep.py, graph replay on a side stream) and the
# teacher-forced accuracy against the reference (tools/l0q_accuracy.py)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
export LVX_SWEEP_STREAM=1
O=gpurun_out/b8l0q.txt
LVX_SWEEP_KV=fp8 timeout -k 10 200 python tools/step_sweep.py 8 384 'l0q=0' '' 'l0q=0' '' > $O 2>&1 || exit 1
timeout -k 10 200 python tools/step_sweep.py 8 384 'l0q=0' '' 'l0q=0' '' >> $O 2>&1 || exit 1
LVX_SWEEP_KV=fp8 timeout -k 10 200 python tools/step_sweep.py 8 896 'l0q=0' '' >> $O 2>&1 || exit 1
timeout -k 10 200 python tools/step_sweep.py 4 384 'l0q=0' '' >> $O 2>&1 || exit 1
timeout -k 10 200 python tools/step_sweep.py 6 384 'l0q=0' '' >> $O 2>&1 || exit 1
timeout -k 10 300 python tools/l0q_accuracy.py fp8 8 'l0q=0' 'l0q=1' >> $O 2>&1 || exit 1
timeout -k 10 300 python tools/l0q_accuracy.py bf16 8 'l0q=0' 'l0q=1' >> $O 2>&1 || exit 1
timeout -k 10 300 python tools/l0q_accuracy.py bf16 4 'l0q=0' 'l0q=1' >> $O 2>&1 || exit 1
