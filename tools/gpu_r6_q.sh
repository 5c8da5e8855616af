# Launch-grid A/B of the walk's seed (DDLO_SEED_BLOCKS) and scan (DDLO_SCAN_WAVES) kernels with the reuse list
# on: per-iteration kernel times of the cfg 2 leg (dev build), then cfg 2 / cfg 3 walk / odometry legs.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6q
mkdir -p $O
L=$PWD/dynamic_direct_lidar_odometry_amd/_lib
prof() {
  local n=$1; shift
  env DDLO_GICP_LIB=$L/dev/libddlo_gicp.so "$@" timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$n -o run -- python3 tools/legs.py cfg2 5 > $O/prof_$n.log 2>&1 || { echo "PROF $n FAIL"; tail -20 $O/prof_$n.log; return 1; }
  python3 tools/profile_summary.py $O/prof_$n run > $O/cfg2_$n.md
  rm -rf $O/prof_$n
  echo "== $n"; grep -E "^\| (0|2|5|9|15) \||linearize \(search" $O/cfg2_$n.md
}
prof base || exit 1
prof listoff DDLO_REUSE_LIST=0 || exit 1
prof seed1024 DDLO_SEED_BLOCKS=1024 || exit 1
prof seed512 DDLO_SEED_BLOCKS=512 || exit 1
prof scan4096 DDLO_SCAN_WAVES=4096 || exit 1
prof s512_sc2048 DDLO_SEED_BLOCKS=512 DDLO_SCAN_WAVES=2048 || exit 1
