set -o pipefail
mkdir -p gpurun_out/det
export PYTHONPATH=.
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity-line > gpurun_out/det/b$i.jsonl 2> gpurun_out/det/b$i.err || { tail -5 gpurun_out/det/b$i.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/det/b$i.jsonl').read().strip().splitlines()[-1]); print($i, d['value'], d['tokens_head'])"
done
