# odometry per-phase wall times (dev build, DDLO_ODOM_TIMING=1: a stream wait per phase) after the hull cache
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/odomtime
L=$PWD/dynamic_direct_lidar_odometry_amd/_lib
DDLO_GICP_LIB=$L/dev/libddlo_gicp.so DDLO_ODOM_TIMING=1 timeout -k 10 300 python -u bench.py --no-cpu --no-sharded --no-gn --no-seg --no-batch --no-walk --steps 10 > gpurun_out/odomtime/r6.json 2> gpurun_out/odomtime/r6.err || { tail -20 gpurun_out/odomtime/r6.err; exit 1; }
grep "odom timing" gpurun_out/odomtime/r6.err | tail -2
