# Device timeline of the odometry chain (kernel + memory copy trace, 120 frames): busy vs idle per frame and the
# average kernel sequence (tools/odom_timeline.py)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6r
mkdir -p $O
rm -rf $O/tr
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr -o run -- python3 tools/odom_probe.py --frames 120 --modes 0 > $O/probe.log 2>&1 || { echo PROF_FAIL; tail $O/probe.log; exit 1; }
grep "ms/frame" $O/probe.log
head -1 $O/tr/run_kernel_trace.csv
python3 tools/odom_timeline.py $O/tr run --skip 30 > $O/odom_timeline.txt || exit 1
rm -rf $O/tr
cat $O/odom_timeline.txt
