# The odometry chain (tools/odom_churn.py bare: a fresh process, 300 frames) with the product library
# against an alternative in-tree build (DDLO_GICP_LIB), interleaved three times.  Usage: bash tools/gpu_odom_ab.sh prev
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=$PWD/dynamic_direct_lidar_odometry_amd/_lib
for rep in 1 2 3; do
  for v in base "$@"; do
    lib=$L/libddlo_gicp.so; [ $v != base ] && lib=$L/$v/libddlo_gicp.so
    r=$(DDLO_GICP_LIB=$lib timeout -k 10 300 python -u tools/odom_churn.py bare 2> gpurun_out/odom_ab_$v.err) || { echo "FAIL $v"; tail gpurun_out/odom_ab_$v.err; exit 1; }
    echo "$v $r"
  done
done
