# lazy search with 16-byte loads in the global passes (used via gpurun): tests, profile, timing, cfg5 legs
cd $GRAFT_REPO_ROOT
O=gpurun_out/lazy7
mkdir -p $O
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_nftree.py > $O/nftree.log 2>&1 || { echo NFTREE_FAIL; tail -30 $O/nftree.log; exit 1; }
tail -1 $O/nftree.log
DDLO_LAZY_PROF=1 timeout -k 10 120 python -u tools/time_cov.py > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
grep "\[lazy\]" $O/prof.log | head -6 | cut -c1-330
timeout -k 10 120 python -u tools/time_cov.py > $O/t.log 2>&1 || exit 1
cat $O/t.log
timeout -k 10 300 python -u bench.py --no-cpu --no-sharded --no-gn --no-seg --steps 20 > $O/b.json 2>/dev/null || exit 1
python -c "import json; d = json.load(open('$O/b.json')); print('batched', d['batched_s2s']['ms_per_pair'], d['batched_s2s']['ms_per_pair_morton_tie_order'], 'odom', d['odometry']['ms_per_frame'], d['odometry']['ms_per_frame_morton_tie_order'])"
