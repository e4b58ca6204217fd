export PYTHONPATH=.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6h; mkdir -p $O
timeout -k 10 120 python tools/codec_probe.py 20 fp32 "" 32x256 > $O/fp32_ev.txt 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 tools/codec_probe.py 10 fp32 "" 32x256 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
f=$(find $O/kt -name '*kernel_stats.csv' | head -1)
python3 tools/kstats.py "$f" lvx > $O/fp32_kstats.txt
cat $O/fp32_ev.txt $O/fp32_kstats.txt
rm -rf $O/kt
