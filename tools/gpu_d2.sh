set -o pipefail
export PYTHONPATH=.
O=gpurun_out/d2; mkdir -p $O
for m in "" "--serial-codec"; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --config 3 --steps 1 --warmup 1 --no-cpu-baseline --no-probe --dist-backend gloo $m > $O/c3$m.jsonl 2> $O/c3$m.err || { tail -5 $O/c3$m.err; exit 1; }
python3 tools/summ.py $O/c3$m.jsonl
done
OUT=ab A_ARGS="" B_ARGS="--ar-priority" PAIRS=3 bash tools/gpu_ab.sh
