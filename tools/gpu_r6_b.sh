# round 6: chain divergence probe + the GPU suite on the current library
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/chain_diff.py 120 > gpurun_out/r6_chain_diff.log 2>&1; echo "chain_diff rc $?"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not identical_input and not loop_revisit" > gpurun_out/r6_gputests.log 2>&1; echo "gpu tests rc $?"
DDLO_GICP_LIB=$PWD/dynamic_direct_lidar_odometry_amd/_lib/covprof/libddlo_gicp.so timeout -k 10 120 python -u tools/cov_timeline.py 4 > gpurun_out/r6_cov_timeline.log 2>&1; echo "cov timeline rc $?"
DDLO_GICP_LIB=$PWD/dynamic_direct_lidar_odometry_amd/_lib/covprof/libddlo_gicp.so timeout -k 10 120 python -u tools/cov_timeline.py 4 --voxel > gpurun_out/r6_cov_timeline_voxel.log 2>&1; echo "cov timeline voxel rc $?"
