set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
mkdir -p gpurun_out/q
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec_variants.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/q/tests.log 2>&1
rc=$?; grep -E "split|LDS-DMA|passed|failed|Error" gpurun_out/q/tests.log | tail -12; exit $rc
