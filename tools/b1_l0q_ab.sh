# round 6: layer 0's c_attn from the q0 tables at B <= 2 (the embedding + select kernel) against the GEMV
# with the granule select (l0q 0): the -m gpu suite, step time, teacher-forced accuracy, configs[1] line
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
O=gpurun_out/b1l0q.txt
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/b1_tests.log 2>&1 || { tail -30 gpurun_out/b1_tests.log; exit 1; }
tail -1 gpurun_out/b1_tests.log > $O
export LVX_SWEEP_STREAM=1
timeout -k 10 200 python tools/step_sweep.py 1 384 'l0q=0' '' 'l0q=0' '' >> $O 2>&1 || exit 1
timeout -k 10 200 python tools/step_sweep.py 2 384 'l0q=0' '' >> $O 2>&1 || exit 1
timeout -k 10 300 python tools/l0q_accuracy.py bf16 1 'l0q=0' 'l0q=1' >> $O 2>&1 || exit 1
timeout -k 10 300 python tools/l0q_accuracy.py bf16 2 'l0q=0' 'l0q=1' >> $O 2>&1 || exit 1
for o in "l0q=0" "l0q=1"; do
timeout -k 10 300 python bench.py --config 1 --steps 8 --no-cpu-baseline --no-parity-line --opt $o > gpurun_out/b1_cfg1_$o.jsonl 2> gpurun_out/b1_cfg1.err || { tail -5 gpurun_out/b1_cfg1.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('configs[1] $o', d['value'], d['ms_per_step'], d['p50_first_chunk_latency_ms'], d['step_roofline']['us_per_step'])" gpurun_out/b1_cfg1_$o.jsonl >> $O
done
grep -v amdgpu.ids $O
