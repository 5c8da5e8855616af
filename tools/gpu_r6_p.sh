# The reuse check as its own one-lane-per-query kernel (k_nn_reuse) ahead of the fused seed, which then walks only
# the listed sub-groups: exactness (GPU suite), cfg 2 / cfg 3 walk / odometry legs against HEAD's library (_lib/head)
# and the dev build with the list off, and a kernel trace of the cfg 2 leg.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6p
mkdir -p $O
L=$PWD/dynamic_direct_lidar_odometry_amd/_lib
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "not loop_revisit" > $O/gputests.log 2>&1; rc=$?; echo "gpu tests rc $rc"; tail -3 $O/gputests.log; [ $rc = 0 ] || exit 1
run() {
  local n=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --no-cpu --no-sharded --no-seg --no-batch --steps 50 > $O/$n.json 2> $O/$n.err || { echo "FAIL $n"; tail $O/$n.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); o=d['odometry']; print('$n cfg3', d['ms_per_step'], 'cfg2', d['s2s_gn']['ms_per_align'], 'walk', d['cfg3_walk']['ms_per_scan'], 'odom', o['ms_per_frame'], o['ms_per_frame_morton_tie_order'])"
}
for rep in 1 2; do
  run new DDLO_GICP_LIB=$L/libddlo_gicp.so || exit 1
  run head DDLO_GICP_LIB=$L/head/libddlo_gicp.so || exit 1
  run listoff DDLO_GICP_LIB=$L/dev/libddlo_gicp.so DDLO_REUSE_LIST=0 || exit 1
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cfg2 -o run -- python3 tools/legs.py cfg2 5 > $O/prof_cfg2.log 2>&1 || { echo "PROF cfg2 FAIL"; tail -20 $O/prof_cfg2.log; exit 1; }
python3 tools/profile_summary.py $O/prof_cfg2 run > $O/cfg2_summary.md
rm -rf $O/prof_cfg2
grep -A 24 "Active outer" $O/cfg2_summary.md
