cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for o in 0 1; do
DDLO_SEED_ORDER=$o DDLO_GICP_LIB=ab/libC.so timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ord$o -o run -- python3 bench.py --no-cpu --no-sharded --no-batch --no-odom --no-gn --no-seg --steps 40 > gpurun_out/ord$o.log 2>&1 || exit 1
echo ORDER=$o; python3 tools/profile_summary.py gpurun_out/ord$o run | grep -E "^\| [0-3] \|"
done
