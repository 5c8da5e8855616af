# Tree-build A/B (used via gpurun): GPU tests on the in-tree library, then
# covariance wall times and the cfg 5 legs for ab/libB.so vs ab/libC.so.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_tree.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_tree.log; exit 1; }
tail -1 gpurun_out/pytest_tree.log
for L in B C; do
  echo "== $L"; DDLO_GICP_LIB=ab/lib$L.so timeout -k 10 120 python -u tools/time_cov.py || exit 1
done
for L in B C; do
  DDLO_GICP_LIB=ab/lib$L.so timeout -k 10 300 python -u bench.py --no-cpu --no-sharded --no-gn --no-seg --steps 20 --batch-frames 300 > gpurun_out/tree_$L.json 2> gpurun_out/tree_$L.err || { echo "BENCH_FAIL $L"; tail -5 gpurun_out/tree_$L.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/tree_$L.json')); b=d['batched_s2s']; o=d['odometry']; print('$L', 'cfg3', d['ms_per_step'], 'batch ms/pair', b['ms_per_pair'], 'odom ms/frame', o.get('ms_per_frame'))"
done
for S in; do
  DDLO_GICP_LIB=ab/libC.so timeout -k 10 300 python -u bench.py --no-cpu --no-sharded --no-gn --no-seg --no-odom --steps 20 --batch-frames 300 --batch-streams $S > gpurun_out/tree_s.json 2> gpurun_out/tree_s.err || { echo "BENCH_FAIL streams $S"; tail -5 gpurun_out/tree_s.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/tree_s.json')); b=d['batched_s2s']; print('C streams $S batch ms/pair', b['ms_per_pair'])"
done
if [ -n "$NFTRACE" ]; then
  DDLO_GICP_LIB=ab/libC.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/nft -o run -- python3 tools/time_cov.py > gpurun_out/nft.log 2>&1 || { tail -5 gpurun_out/nft.log; exit 1; }
  python3 tools/nf_trace.py gpurun_out/nft/run_kernel_trace.csv | tail -14
fi
