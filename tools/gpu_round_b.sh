#!/bin/bash
# round end, part 2 of 2 (one gpurun call): tools/prof_round.sh for configs[4] (PMC traffic at
# bf16/kvfp8/B8/P512, MFMA busy at fp8/F2048/L256, kernel trace, the configs[4] line), then
# tools/gpu_round_lines.sh (configs 1/3/4, the 60-s steady state, 2-rank rehearsals, the parity-line PMC pass)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
TAG=r06c4 ARGS="--config 4 --steps 20 --warmup 0 --no-cpu-baseline --no-parity-line" KEY=bf16/kvfp8/B8/P512 \
  CKEY=fp8/F2048/L256 BENCH_ARGS="--config 4 --steps 20 --warmup 5 --no-cpu-baseline" bash tools/prof_round.sh || exit 1
bash tools/gpu_round_lines.sh || exit 1
echo PART2_OK
