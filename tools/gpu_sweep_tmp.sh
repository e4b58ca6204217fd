set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
rm -f gpurun_out/sweep.log
for BP in "32 256" "32 512" "64 512" "16 1024"; do
  timeout -k 10 200 python -u tools/probe_ops.py $BP attn_depth=2 attn_depth=4 attn_depth=2 attn_depth=4 >> gpurun_out/sweep.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/sweep.log
