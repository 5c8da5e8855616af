# Segmentation host labelling: the angle test without atan2 away from the threshold (ratio against
# tan(theta (1 -+ 1e-6))), persistent BFS queues, the pinned read-back used in place: exactness
# (segmentation tests) and the segmentation leg against _lib/head, three interleaved repeats.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
L=$PWD/dynamic_direct_lidar_odometry_amd/_lib
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "segment" > gpurun_out/r6_gputests_z.log 2>&1; rc=$?; echo "gpu tests rc $rc"; tail -1 gpurun_out/r6_gputests_z.log; [ $rc = 0 ] || exit 1
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu --no-sharded --no-gn --no-walk --no-batch --no-odom --steps 20 > gpurun_out/ab/$n.json 2> gpurun_out/ab/$n.err || { echo "FAIL $n"; tail gpurun_out/ab/$n.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab/$n.json')); s=d['segmentation']; print('$n seg', s['ms_per_frame'], s['segments'], s['ground_pixels'])"
}
for rep in 1 2 3; do
  run new DDLO_GICP_LIB=$L/libddlo_gicp.so || exit 1
  run head DDLO_GICP_LIB=$L/head/libddlo_gicp.so || exit 1
done
