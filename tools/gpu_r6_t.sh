# k_covariances2 with the seed leaves with the next leaf's points in flight:
# exactness (GPU suite), the per-group timeline, covariance timing and batch + odometry legs against HEAD's kernels (_lib/head)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
L=$PWD/dynamic_direct_lidar_odometry_amd/_lib
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "cov or knn or batch or nftree or tie" > gpurun_out/r6_gputests_t.log 2>&1; echo "gpu tests rc $?"; tail -1 gpurun_out/r6_gputests_t.log
DDLO_GICP_LIB=$L/covprof/libddlo_gicp.so timeout -k 10 120 python -u tools/cov_timeline.py 3 --voxel > gpurun_out/r6_cov_timeline_seedpipe_voxel.log 2>&1; echo "timeline voxel rc $?"; grep "^frame\|finished\|per scanned" gpurun_out/r6_cov_timeline_seedpipe_voxel.log
for v in head new head new; do
  lib=$L/libddlo_gicp.so; [ $v = head ] && lib=$L/head/libddlo_gicp.so
  DDLO_GICP_LIB=$lib timeout -k 10 120 python -u tools/time_cov.py > gpurun_out/r6_time_cov_$v.log 2>&1; echo "$v: $(tail -2 gpurun_out/r6_time_cov_$v.log | tr '\n' ' ')"
done
run() {
  local n=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --no-cpu --no-sharded --no-gn --no-seg --no-walk --steps 20 > gpurun_out/ab/$n.json 2> gpurun_out/ab/$n.err || { echo "FAIL $n"; tail gpurun_out/ab/$n.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab/$n.json')); o=d['odometry']; b=d['batched_s2s']; print('$n odom', o['ms_per_frame'], o['ms_per_frame_morton_tie_order'], 'batch', b['ms_per_pair'], b['ms_per_pair_morton_tie_order'], 'cov', b['cfg5_stages_rank0']['covariances']['avg_launch_us'])"
}
for rep in 1 2; do
  run new DDLO_GICP_LIB=$L/libddlo_gicp.so || exit 1
  run head DDLO_GICP_LIB=$L/head/libddlo_gicp.so || exit 1
done
