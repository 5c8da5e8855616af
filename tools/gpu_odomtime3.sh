# odometry per-phase wall times with the pre-frame device drain split out (used via gpurun)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/odomtime3
DDLO_ODOM_TIMING=1 timeout -k 10 300 python -u bench.py --no-cpu --no-sharded --no-gn --no-seg --no-batch --steps 10 > gpurun_out/odomtime3/b.json 2> gpurun_out/odomtime3/b.err || { tail -20 gpurun_out/odomtime3/b.err; exit 1; }
grep "odom timing" gpurun_out/odomtime3/b.err
