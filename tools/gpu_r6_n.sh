# wide covariance groups searched as two halves in parallel (k_covariances2 presplit): exactness (GPU suite),
# the per-item timeline, covariance timing at thresholds off / 1 / 2 / 4 m (dev build), batch + odometry legs
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
L=$PWD/dynamic_direct_lidar_odometry_amd/_lib
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "not loop_revisit and not identical_input" > gpurun_out/r6_gputests_n.log 2>&1; echo "gpu tests rc $?"; tail -1 gpurun_out/r6_gputests_n.log
DDLO_GICP_LIB=$L/covprof/libddlo_gicp.so timeout -k 10 120 python -u tools/cov_timeline.py 3 --items > gpurun_out/r6_cov_timeline_presplit.log 2>&1; echo "timeline rc $?"; grep "^frame\|finished" gpurun_out/r6_cov_timeline_presplit.log
for dm in 0 10 20 40; do
  DDLO_GICP_LIB=$L/dev/libddlo_gicp.so DDLO_COV_PRESPLIT_DM=$dm timeout -k 10 120 python -u tools/time_cov.py > gpurun_out/r6_time_cov_ps$dm.log 2>&1; echo "presplit $dm dm: $(tail -2 gpurun_out/r6_time_cov_ps$dm.log | tr '\n' ' ')"
done
run() {
  local n=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --no-cpu --no-sharded --no-gn --no-seg --no-walk --steps 20 > gpurun_out/ab/$n.json 2> gpurun_out/ab/$n.err || { echo "FAIL $n"; tail gpurun_out/ab/$n.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab/$n.json')); o=d['odometry']; b=d['batched_s2s']; print('$n odom', o['ms_per_frame'], o['ms_per_frame_morton_tie_order'], 'batch', b['ms_per_pair'], b['ms_per_pair_morton_tie_order'], 'cov', b['cfg5_stages_rank0']['covariances']['avg_launch_us'])"
}
for rep in 1 2; do
  run ps20 DDLO_GICP_LIB=$L/dev/libddlo_gicp.so DDLO_COV_PRESPLIT_DM=20 || exit 1
  run ps0 DDLO_GICP_LIB=$L/dev/libddlo_gicp.so DDLO_COV_PRESPLIT_DM=0 || exit 1
done
