# round 6: what the GELU in pwconv1's epilogue costs the bf16 codec decode (a timing build with the GELU
# left out, LVX_GELU_PROBE, against the production library; tools/codec_probe.py, HIP events)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
O=gpurun_out/gelu_probe.txt
: > $O
for i in 1 2; do
timeout -k 10 200 python tools/codec_probe.py 10 bf16 "" 32x256,8x256 >> $O 2>&1 || exit 1
LVX_LIB_PATH=llmvox_amd/libllmvox_hip_geluprobe.so timeout -k 10 200 python tools/codec_probe.py 10 bf16 "" 32x256,8x256 | sed 's/^/no-gelu /' >> $O 2>&1 || exit 1
done
grep -v amdgpu $O
