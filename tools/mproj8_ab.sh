# round 6: mlp c_proj as 8 K slices x 32-column tiles at 9 <= B <= 32 (ar_mproj8_kernel, option exp bit 2)
# against 4 slices x 16 columns: step time, accuracy against the reference, a bounded comparison
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
O=gpurun_out/mproj8.txt
export LVX_SWEEP_STREAM=1
timeout -k 10 200 python tools/step_sweep.py 32 384 '' 'exp=2' '' 'exp=2' > $O 2>&1 || exit 1
timeout -k 10 200 python tools/step_sweep.py 16 384 '' 'exp=2' >> $O 2>&1 || exit 1
timeout -k 10 200 python tools/step_sweep.py 32 896 '' 'exp=2' >> $O 2>&1 || exit 1
timeout -k 10 300 python tools/l0q_accuracy.py bf16 32 'exp=0' 'exp=2' >> $O 2>&1 || exit 1
timeout -k 10 300 python tools/l0q_accuracy.py bf16 16 'exp=0' 'exp=2' >> $O 2>&1 || exit 1
grep -v amdgpu.ids $O
