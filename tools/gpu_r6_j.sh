# two-level fan-in of the fused LM step (default) against the single-counter fan-in (_lib/prev) and round 5 (_lib/head)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
L=$PWD/dynamic_direct_lidar_odometry_amd/_lib
run() {   # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --no-cpu --no-sharded --no-batch --no-odom --no-seg --no-walk --no-gn --steps 200 > gpurun_out/ab/$n.json 2> gpurun_out/ab/$n.err || { echo "FAIL $n"; tail gpurun_out/ab/$n.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab/$n.json')); print('$n', d['ms_per_step'], d.get('cfg3_varied_guesses', {}).get('ms_per_scan'))"
}
for rep in 1 2 3; do
  run fan2 DDLO_X=1 || exit 1
  run fan1 DDLO_GICP_LIB=$L/prev/libddlo_gicp.so || exit 1
  run head DDLO_GICP_LIB=$L/head/libddlo_gicp.so || exit 1
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "not loop_revisit and not identical_input" > gpurun_out/r6_gputests_j.log 2>&1; echo "gpu tests rc $?"
