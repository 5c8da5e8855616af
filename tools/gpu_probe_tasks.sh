# task-search probe + kernel trace of a short bench (used via gpurun)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
DDLO_GICP_LIB=$PWD/dynamic_direct_lidar_odometry_amd/_lib/statsprof/libddlo_gicp.so timeout -k 10 120 python -u tools/probe_tasks.py > gpurun_out/probe_tasks.log 2>&1 || { echo PROBE_FAIL; tail -20 gpurun_out/probe_tasks.log; exit 1; }
cat gpurun_out/probe_tasks.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt -o run -- python3 bench.py --no-cpu --no-sharded --no-batch --steps 10 --warmup 2 > gpurun_out/kt.log 2>&1 || { tail -20 gpurun_out/kt.log; exit 1; }
python3 tools/profile_summary.py gpurun_out/kt run
