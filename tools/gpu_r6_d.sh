mkdir -p gpurun_out
DDLO_GICP_LIB=$PWD/dynamic_direct_lidar_odometry_amd/_lib/covprof/libddlo_gicp.so timeout -k 10 120 python -u tools/cov_timeline.py 3 > gpurun_out/r6_cov_timeline_uns.log 2>&1; echo "cov timeline rc $?"
timeout -k 10 120 python -u tools/time_cov.py > gpurun_out/r6_time_cov_uns.log 2>&1; echo "time_cov rc $?"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not identical_input and not loop_revisit" > gpurun_out/r6_gputests_d.log 2>&1; echo "gpu tests rc $?"
