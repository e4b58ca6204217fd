set -o pipefail
export PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 120 python -c "import torch; print('default cuda_stream', torch.cuda.current_stream(0).cuda_stream); s=torch.cuda.Stream(); print('side', s.cuda_stream)" > gpurun_out/chk_stream.txt 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-probe > gpurun_out/chk_g.jsonl 2>gpurun_out/chk_g.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-probe --no-graphs > gpurun_out/chk_ng.jsonl 2>gpurun_out/chk_ng.err
rc=$?
cat gpurun_out/chk_stream.txt; cut -c1-200 gpurun_out/chk_g.jsonl gpurun_out/chk_ng.jsonl; exit $rc
