# round 6: small batches on the rows-kernel structure (option ln_max below B) against the LayerNorm-prologue
# GEMMs, re-measured with the layer-0 tables (B = 8 fp8 / bf16 KV, B = 6, t = 384-639)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=. LVX_SWEEP_STREAM=1
O=gpurun_out/lnmax.txt
LVX_SWEEP_KV=fp8 timeout -k 10 200 python tools/step_sweep.py 8 384 '' 'ln_max=4' '' 'ln_max=4' > $O 2>&1 || exit 1
timeout -k 10 200 python tools/step_sweep.py 8 384 '' 'ln_max=4' >> $O 2>&1 || exit 1
timeout -k 10 200 python tools/step_sweep.py 6 384 '' 'ln_max=4' >> $O 2>&1 || exit 1
grep -v amdgpu.ids $O
