# one-compare insertion network: exactness (GPU suite), k_covariances2's per-group timeline, the cfg 5
# batch leg against round 5's library (_lib/head), and the covariance timing of one scan
mkdir -p gpurun_out
L=$PWD/dynamic_direct_lidar_odometry_amd/_lib
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "not loop_revisit and not identical_input" > gpurun_out/r6_gputests_i.log 2>&1; echo "gpu tests rc $?"
DDLO_GICP_LIB=$L/covprof/libddlo_gicp.so timeout -k 10 120 python -u tools/cov_timeline.py 3 > gpurun_out/r6_cov_timeline_cx.log 2>&1; echo "cov timeline rc $?"
DDLO_GICP_LIB=$L/covprof/libddlo_gicp.so timeout -k 10 120 python -u tools/cov_timeline.py 3 --voxel > gpurun_out/r6_cov_timeline_cx_voxel.log 2>&1; echo "cov timeline voxel rc $?"
timeout -k 10 120 python -u tools/time_cov.py > gpurun_out/r6_time_cov_cx.log 2>&1; echo "time_cov rc $?"
DDLO_GICP_LIB=$L/head/libddlo_gicp.so timeout -k 10 120 python -u tools/time_cov.py > gpurun_out/r6_time_cov_head.log 2>&1; echo "time_cov head rc $?"
for rep in 1 2; do
  timeout -k 10 300 python3 tools/batch_leg_alone.py bare > gpurun_out/r6_batch_new.log 2>&1 && echo "new:  $(grep '^bare' gpurun_out/r6_batch_new.log)"
  DDLO_GICP_LIB=$L/head/libddlo_gicp.so timeout -k 10 300 python3 tools/batch_leg_alone.py bare > gpurun_out/r6_batch_head.log 2>&1 && echo "head: $(grep '^bare' gpurun_out/r6_batch_head.log)"
done
