# cached keyframe hulls: the odometry leg (cfg 5 chain, 1000 frames) against the library before it (_lib/prev),
# interleaved twice; then the odometry GPU tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
L=$PWD/dynamic_direct_lidar_odometry_amd/_lib
run() {
  local n=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --no-cpu --no-sharded --no-batch --no-gn --no-seg --no-walk --steps 20 > gpurun_out/ab/$n.json 2> gpurun_out/ab/$n.err || { echo "FAIL $n"; tail gpurun_out/ab/$n.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab/$n.json')); o=d['odometry']; print('$n', o['ms_per_frame'], o['ms_per_frame_morton_tie_order'])"
}
for rep in 1 2; do
  run hulls DDLO_X=1 || exit 1
  run prev DDLO_GICP_LIB=$L/prev/libddlo_gicp.so || exit 1
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_odom.py tests/test_gpu_odom_long.py -x -q --timeout 600 --timeout-method thread -k "not loop_revisit and not identical_input" > gpurun_out/r6_gputests_k.log 2>&1; echo "odom tests rc $?"
