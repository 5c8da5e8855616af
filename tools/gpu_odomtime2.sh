# odometry per-phase wall times: lazy search vs whole tree (used via gpurun)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/odomtime
for lz in 1 0; do
  DDLO_TIE_LAZY=$lz DDLO_ODOM_TIMING=1 timeout -k 10 300 python -u bench.py --no-cpu --no-sharded --no-gn --no-seg --no-batch --steps 10 > gpurun_out/odomtime/b$lz.json 2> gpurun_out/odomtime/b$lz.err || { tail -20 gpurun_out/odomtime/b$lz.err; exit 1; }
  echo "lazy=$lz"; grep "odom timing" gpurun_out/odomtime/b$lz.err | tail -2
done
