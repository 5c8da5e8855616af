# order-free inner ties dropped from the re-run list (used via gpurun): covariance exactness, tests, timing
cd $GRAFT_REPO_ROOT
O=gpurun_out/orderfree
mkdir -p $O
timeout -k 10 300 python -u tools/probe_cov_exact.py > $O/exact.log 2>&1 || { tail -20 $O/exact.log; exit 1; }
cat $O/exact.log
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_nftree.py tests/test_gpu_gicp.py tests/test_gpu_knn.py tests/test_gpu_odom.py > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python -u tools/tie_classify.py 4 > $O/classify.log 2>&1 || exit 1
grep -v "^\[ties\]" $O/classify.log
timeout -k 10 120 python -u tools/time_cov.py > $O/time_cov.log 2>&1 || exit 1
cat $O/time_cov.log
timeout -k 10 300 python -u bench.py --no-cpu --no-sharded --no-gn --no-seg --steps 20 > $O/b.json 2>/dev/null || exit 1
python -c "import json; d = json.load(open('$O/b.json')); print('batched', d['batched_s2s']['ms_per_pair'], d['batched_s2s']['ms_per_pair_morton_tie_order'], 'odom', d['odometry']['ms_per_frame'], d['odometry']['ms_per_frame_morton_tie_order'])"
