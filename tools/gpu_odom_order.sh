# Which earlier bench leg slows the odometry leg inside bench.py: the odometry leg after the headline only,
# after the headline + batch leg, after the headline + sharded leg, and the default order.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/odom_order
mkdir -p $O
run() {
  timeout -k 10 600 python -u bench.py --no-cpu --no-seg --no-walk --steps 20 --warmup 5 "$@" > $O/b.json 2> $O/b.err || { echo "BENCH FAIL $*"; tail $O/b.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/b.json')); o=d['odometry']; print(sys.argv[1:], o['ms_per_frame'], o['ms_per_frame_morton_tie_order'])" "$@"
}
run --no-sharded --no-gn --no-batch
run --no-sharded --no-gn
run --no-gn --no-batch
run
