cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
mkdir -p gpurun_out/r02
timeout -k 10 300 python tools/overlap_probe.py 2560 64 > gpurun_out/r02/overlap_2560.txt 2>&1; echo rc=$?; cat gpurun_out/r02/overlap_2560.txt
timeout -k 10 300 python tools/overlap_probe.py 512 64 > gpurun_out/r02/overlap_512.txt 2>&1; echo rc=$?; cat gpurun_out/r02/overlap_512.txt
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d /tmp/r1cmd -o run --output-format csv -- python3 bench.py --no-cpu-baseline --config 2 --steps 2 > gpurun_out/r02/r1cmd_pmc.log 2>&1; echo "r1 pmc cmd rc=$?"; tail -30 gpurun_out/r02/r1cmd_pmc.log
