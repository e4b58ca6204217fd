# Development check: the 2-rank gloo configs[3] rehearsal (two processes on one GPU, the FusedScheduler
# service path) alone, as tools/gpu_round_lines.sh runs it. Round 6 used it to find the cost of a
# capture stream created by the library (profiles/r06/capture_stream_ab.txt).
set -o pipefail
mkdir -p gpurun_out/c3ab
export PYTHONPATH=.
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --config 3 --steps 1 --warmup 1 --no-cpu-baseline --no-probe --dist-backend gloo --sched cs=0 > gpurun_out/c3ab/d.jsonl 2> gpurun_out/c3ab/d.err || { tail -5 gpurun_out/c3ab/d.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open('gpurun_out/c3ab/d.jsonl').read().strip().splitlines()[-1]); print('dist2_c3', d['value'], d['ms_per_step'], d['p50_first_chunk_latency_ms'])"
