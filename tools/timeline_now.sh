# in-kernel step timelines (timing build) at B = 32 / 16 / 8 (fp8 KV), t = 384
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
O=gpurun_out/timeline_now.txt
timeout -k 10 200 python tools/step_timeline.py 32 384 1 > $O 2>&1 || exit 1
timeout -k 10 200 python tools/step_timeline.py 8 384 1 >> $O 2>&1 || exit 1
grep -v amdgpu.ids $O
