# odometry driver per-phase wall times, nanoflann and Morton order (used via gpurun)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/odomtime
DDLO_ODOM_TIMING=1 timeout -k 10 300 python -u bench.py --no-cpu --no-sharded --no-gn --no-seg --no-batch --steps 10 > gpurun_out/odomtime/b.json 2> gpurun_out/odomtime/b.err || { tail -20 gpurun_out/odomtime/b.err; exit 1; }
grep "odom timing" gpurun_out/odomtime/b.err
python -c "import json; d = json.load(open('gpurun_out/odomtime/b.json')); print('odom', d['odometry']['ms_per_frame'], d['odometry']['ms_per_frame_morton_tie_order'])"
