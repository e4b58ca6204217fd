set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
export LVX_SWEEP_STREAM=1
for v in 0 1 0 1; do
  echo "HIP_FORCE_DEV_KERNARG=$v"
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 120 python tools/step_sweep.py 32 384 || exit 1
done
for v in 0 1; do
  echo "DEBUG_CLR_GRAPH_PACKET_CAPTURE=$v"
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=$v timeout -k 10 120 python tools/step_sweep.py 32 384 || exit 1
done
