# k_covariances2's per-group cycle split (covprof build: s_memtime around a leaf's point wait, its scan and a leaf
# block's box tests), raw and voxel-filtered cfg 5 scans
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
L=$PWD/dynamic_direct_lidar_odometry_amd/_lib
DDLO_GICP_LIB=$L/covprof/libddlo_gicp.so timeout -k 10 120 python -u tools/cov_timeline.py 2 > gpurun_out/r6_cov_cycles.log 2>&1; echo "rc $?"; grep -v "^   group" gpurun_out/r6_cov_cycles.log
DDLO_GICP_LIB=$L/covprof/libddlo_gicp.so timeout -k 10 120 python -u tools/cov_timeline.py 2 --voxel > gpurun_out/r6_cov_cycles_voxel.log 2>&1; echo "rc $?"; grep -v "^   group" gpurun_out/r6_cov_cycles_voxel.log
