# round 6: kernel trace of the B = 1 step (tools/step_sweep.py 1 384, graph replay on a side stream): per-kernel durations
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=. LVX_SWEEP_STREAM=1
mkdir -p gpurun_out/b1t
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/b1t/kt -o run --output-format csv -- python3 tools/step_sweep.py 1 384 '' > gpurun_out/b1t/kt.log 2>&1 || { tail -20 gpurun_out/b1t/kt.log; exit 1; }
find gpurun_out/b1t/kt -name "*kernel_stats.csv" -exec cp {} gpurun_out/b1t/kernel_stats.csv \;
rm -rf gpurun_out/b1t/kt
head -12 gpurun_out/b1t/kernel_stats.csv | cut -d, -f1-4
