# lazy search with DPP reductions / readlane: tests, profile, timing (used via gpurun)
cd $GRAFT_REPO_ROOT
O=gpurun_out/lazy6
mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_nftree.py > $O/nftree.log 2>&1 || { echo NFTREE_FAIL; tail -30 $O/nftree.log; exit 1; }
tail -1 $O/nftree.log
DDLO_TIE_PARTIAL_LEVELS=3 DDLO_LAZY_PROF=1 timeout -k 10 120 python -u tools/time_cov.py > $O/prof3.log 2>&1 || { tail -20 $O/prof3.log; exit 1; }
grep "\[lazy\]" $O/prof3.log | head -6 | cut -c1-330
for L in 3; do
  DDLO_TIE_PARTIAL_LEVELS=$L timeout -k 10 120 python -u tools/time_cov.py > $O/t_L$L.log 2>&1 || exit 1
  cat $O/t_L$L.log
  DDLO_TIE_PARTIAL_LEVELS=$L timeout -k 10 300 python -u bench.py --no-cpu --no-sharded --no-gn --no-seg --steps 20 > $O/b_L$L.json 2>/dev/null || exit 1
  python -c "import json; d = json.load(open('$O/b_L$L.json')); print('L$L', 'batched', d['batched_s2s']['ms_per_pair'], d['batched_s2s']['ms_per_pair_morton_tie_order'], 'odom', d['odometry']['ms_per_frame'], d['odometry']['ms_per_frame_morton_tie_order'])"
done
