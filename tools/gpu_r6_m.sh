# four lanes per covariance query for small clouds: the odometry leg (voxel-filtered ~82k-point scans) and the
# cfg 5 batch leg (raw 131k) with the threshold on (200k) and off (0), dev build; per-group timelines
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
L=$PWD/dynamic_direct_lidar_odometry_amd/_lib
for m in 0 200000; do
  DDLO_GICP_LIB=$L/covprof/libddlo_gicp.so DDLO_COV_4LANE_MAX=$m timeout -k 10 120 python -u tools/cov_timeline.py 3 --voxel $([ $m = 0 ] || echo --g16) > gpurun_out/r6_cov_vox_$m.log 2>&1; echo "timeline $m rc $?"; grep "^frame" gpurun_out/r6_cov_vox_$m.log
done
run() {
  local n=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --no-cpu --no-sharded --no-gn --no-seg --no-walk --steps 20 > gpurun_out/ab/$n.json 2> gpurun_out/ab/$n.err || { echo "FAIL $n"; tail gpurun_out/ab/$n.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab/$n.json')); o=d['odometry']; b=d['batched_s2s']; print('$n odom', o['ms_per_frame'], o['ms_per_frame_morton_tie_order'], 'batch', b['ms_per_pair'], b['ms_per_pair_morton_tie_order'])"
}
for rep in 1 2; do
  run four DDLO_GICP_LIB=$L/dev/libddlo_gicp.so DDLO_COV_4LANE_MAX=200000 || exit 1
  run two DDLO_GICP_LIB=$L/dev/libddlo_gicp.so DDLO_COV_4LANE_MAX=0 || exit 1
done
