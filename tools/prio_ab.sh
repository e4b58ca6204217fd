# round 6: the decode kernels' waves at raised issue priority (s_setprio 3 at entry; a timing build,
# LVX_AR_SETPRIO) against the production library: the codec's interference with the decode steps
# (tools/interference_probe.py) and the configs[2] line, alternating
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
O=gpurun_out/prio_ab.txt
: > $O
for i in 1 2; do
for lib in llmvox_amd/libllmvox_hip.so llmvox_amd/libllmvox_hip_prio3.so; do
echo "## $lib" >> $O
LVX_LIB_PATH=$lib timeout -k 10 200 python tools/interference_probe.py 384 all >> $O 2>&1 || exit 1
LVX_LIB_PATH=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity-line --no-probe --no-loaded-latency > gpurun_out/prio_c2.jsonl 2> gpurun_out/prio_c2.err || { tail -5 gpurun_out/prio_c2.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c2', d['value'], d['ms_per_step'], d['step_roofline']['us_per_step'], d['tokens_head'])" gpurun_out/prio_c2.jsonl >> $O
done
done
grep -v amdgpu.ids $O
