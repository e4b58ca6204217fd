# the -m gpu suite and smoke() after a library change, then the configs[2] and configs[4] lines
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/after_tests.log 2>&1 || { tail -30 gpurun_out/after_tests.log; exit 1; }
tail -1 gpurun_out/after_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/after_smoke.log 2>&1 || { tail -5 gpurun_out/after_smoke.log; exit 1; }
tail -1 gpurun_out/after_smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity-line > gpurun_out/after_c2.jsonl 2> gpurun_out/after_c2.err || { tail -5 gpurun_out/after_c2.err; exit 1; }
timeout -k 10 300 python bench.py --config 4 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/after_c4.jsonl 2> gpurun_out/after_c4.err || { tail -5 gpurun_out/after_c4.err; exit 1; }
for f in c2 c4; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d['p50_first_chunk_latency_ms'], d['step_roofline']['us_per_step'], d['tokens_head'])" gpurun_out/after_$f.jsonl; done
