# odometry driver: partial tree beside the covariance kernel vs gated on its own stream (used via gpurun)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/odomown
for os in 0 1; do
  DDLO_NF_OWN_STREAM=$os timeout -k 10 300 python -u bench.py --no-cpu --no-sharded --no-gn --no-seg --no-batch --steps 10 > gpurun_out/odomown/b$os.json 2> gpurun_out/odomown/b$os.err || { tail -20 gpurun_out/odomown/b$os.err; exit 1; }
  python3 -c "import json; d = json.load(open('gpurun_out/odomown/b$os.json')); print('own stream $os', d['odometry']['ms_per_frame'], d['odometry']['ms_per_frame_morton_tie_order'])"
done
for os in 0 1; do
  DDLO_NF_OWN_STREAM=$os DDLO_ODOM_TIMING=1 timeout -k 10 300 python -u bench.py --no-cpu --no-sharded --no-gn --no-seg --no-batch --steps 10 > gpurun_out/odomown/t$os.json 2> gpurun_out/odomown/t$os.err || { tail -20 gpurun_out/odomown/t$os.err; exit 1; }
  echo "own stream $os"; grep "odom timing" gpurun_out/odomown/t$os.err | tail -2
done
