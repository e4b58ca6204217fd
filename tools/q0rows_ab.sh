# round 6: the select + layer-0 q0-table launch over 9 column slices per row (ar_q0_rows_kernel, default)
# against one ar_embed_select_kernel<false, true> block per row (option exp bit 2; that form and the bit
# were removed after this A/B, profiles/r06/q0rows_ab.txt): -m gpu suite, step
# sweeps at B = 32 / 16 / 8 (fp8) / 4, accuracy against the reference, configs[2] and configs[4] lines
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
O=gpurun_out/q0rows.txt
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/q0rows_tests.log 2>&1 || { tail -30 gpurun_out/q0rows_tests.log; exit 1; }
tail -1 gpurun_out/q0rows_tests.log > $O
export LVX_SWEEP_STREAM=1
timeout -k 10 200 python tools/step_sweep.py 32 384 'exp=2' '' 'exp=2' '' >> $O 2>&1 || exit 1
timeout -k 10 200 python tools/step_sweep.py 16 384 'exp=2' '' >> $O 2>&1 || exit 1
LVX_SWEEP_KV=fp8 timeout -k 10 200 python tools/step_sweep.py 8 384 'exp=2' '' 'exp=2' '' >> $O 2>&1 || exit 1
timeout -k 10 200 python tools/step_sweep.py 4 384 'exp=2' '' >> $O 2>&1 || exit 1
timeout -k 10 300 python tools/l0q_accuracy.py bf16 32 'l0q=0' 'l0q=1' >> $O 2>&1 || exit 1
timeout -k 10 300 python tools/l0q_accuracy.py fp8 8 'l0q=0' 'l0q=1' >> $O 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity-line > gpurun_out/q0rows_c2.jsonl 2> gpurun_out/q0rows_c2.err || { tail -5 gpurun_out/q0rows_c2.err; exit 1; }
timeout -k 10 300 python bench.py --config 4 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/q0rows_c4.jsonl 2> gpurun_out/q0rows_c4.err || { tail -5 gpurun_out/q0rows_c4.err; exit 1; }
for f in c2 c4; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d['p50_first_chunk_latency_ms'], d['step_roofline']['us_per_step'], d['tokens_head'])" gpurun_out/q0rows_$f.jsonl >> $O; done
grep -v amdgpu.ids $O
