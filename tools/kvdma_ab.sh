# round 6: the fp8 8-wave attention with its K / V tiles staged by LDS-DMA (option exp bit 2) against the
# register form: bit-identity, step time at B = 8 / 12 / 16 (fp8 KV), configs[4] line
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
O=gpurun_out/kvdma.txt
LVX_AB_KV=fp8 timeout -k 10 200 python tools/ab_bitcheck.py exp 2 5 8 12 16 > $O 2>&1 || { cat $O; exit 1; }
export LVX_SWEEP_STREAM=1 LVX_SWEEP_KV=fp8
timeout -k 10 200 python tools/step_sweep.py 8 384 '' 'exp=2' '' 'exp=2' >> $O 2>&1 || exit 1
timeout -k 10 200 python tools/step_sweep.py 8 896 '' 'exp=2' >> $O 2>&1 || exit 1
timeout -k 10 200 python tools/step_sweep.py 16 384 '' 'exp=2' >> $O 2>&1 || exit 1
for o in "exp=0" "exp=2"; do
timeout -k 10 300 python bench.py --config 4 --steps 20 --warmup 5 --no-cpu-baseline --no-probe --no-loaded-latency --opt $o > gpurun_out/kvdma_c4.jsonl 2> gpurun_out/kvdma_c4.err || { tail -5 gpurun_out/kvdma_c4.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('configs[4] $o', d['value'], d['ms_per_step'], d['step_roofline']['us_per_step'], d['tokens_head'])" gpurun_out/kvdma_c4.jsonl >> $O
done
grep -v amdgpu.ids $O
