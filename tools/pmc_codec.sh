#!/bin/bash
# L2 hit/miss of the codec GEMMs with and without the XCD-aware tile order
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
rm -rf gpurun_out/pmc_c*
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_c1 -o run --output-format csv -- python3 tools/prof_codec.py bf16 256 32 codec_xcd=1 > gpurun_out/pmc_c1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_c0 -o run --output-format csv -- python3 tools/prof_codec.py bf16 256 32 codec_xcd=0 > gpurun_out/pmc_c0.log 2>&1
