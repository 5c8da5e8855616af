# leaf_block: two leaves' boxes read from LDS per step (tested in leaf order as before):
# exactness (covariance / kNN / batch / tie tests), covariance timing, batch + odometry legs against HEAD (_lib/head)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
L=$PWD/dynamic_direct_lidar_odometry_amd/_lib
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "cov or knn or batch or nftree or tie" > gpurun_out/r6_gputests_bb.log 2>&1; echo "gpu tests rc $?"; tail -1 gpurun_out/r6_gputests_bb.log
tc() {
  local n=$1; shift
  env "$@" timeout -k 10 120 python -u tools/time_cov.py > gpurun_out/r6_time_cov_$n.log 2>&1; echo "$n: $(tail -2 gpurun_out/r6_time_cov_$n.log | tr '\n' ' ')"
}
run() {
  local n=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --no-cpu --no-sharded --no-gn --no-seg --no-walk --steps 20 > gpurun_out/ab/$n.json 2> gpurun_out/ab/$n.err || { echo "FAIL $n"; tail gpurun_out/ab/$n.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab/$n.json')); o=d['odometry']; b=d['batched_s2s']; print('$n odom', o['ms_per_frame'], o['ms_per_frame_morton_tie_order'], 'batch', b['ms_per_pair'], b['ms_per_pair_morton_tie_order'], 'cov', b['cfg5_stages_rank0']['covariances']['avg_launch_us'])"
}
for rep in 1 2; do
  tc head DDLO_GICP_LIB=$L/head/libddlo_gicp.so
  tc pair DDLO_GICP_LIB=$L/libddlo_gicp.so
done
for rep in 1 2; do
  run head DDLO_GICP_LIB=$L/head/libddlo_gicp.so || exit 1
  run pair DDLO_GICP_LIB=$L/libddlo_gicp.so || exit 1
done
