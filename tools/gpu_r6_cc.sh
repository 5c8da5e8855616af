# Cloud index build: the leaves' SoA copy and boxes in one kernel (k_leaf_soa_boxes): the whole GPU suite, then the
# odometry leg against HEAD (_lib/head), two interleaved repeats.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
L=$PWD/dynamic_direct_lidar_odometry_amd/_lib
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > gpurun_out/r6_gputests_cc.log 2>&1; rc=$?; echo "gpu tests rc $rc"; tail -1 gpurun_out/r6_gputests_cc.log; [ $rc = 0 ] || exit 1
run() {
  local n=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --no-cpu --no-sharded --no-gn --no-seg --no-walk --no-batch --steps 20 > gpurun_out/ab/$n.json 2> gpurun_out/ab/$n.err || { echo "FAIL $n"; tail gpurun_out/ab/$n.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab/$n.json')); o=d['odometry']; print('$n cfg3', d['ms_per_step'], 'odom', o['ms_per_frame'], o['ms_per_frame_morton_tie_order'])"
}
for rep in 1 2; do
  run new DDLO_GICP_LIB=$L/libddlo_gicp.so || exit 1
  run head DDLO_GICP_LIB=$L/head/libddlo_gicp.so || exit 1
done
