# odometry pass order vs. upload time (used via gpurun)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/odomorder
timeout -k 10 300 python -u tools/odom_order.py > gpurun_out/odomorder/o.txt 2> gpurun_out/odomorder/o.err || { tail -20 gpurun_out/odomorder/o.err; exit 1; }
cat gpurun_out/odomorder/o.txt; grep -E "odom timing|^---" gpurun_out/odomorder/o.err
