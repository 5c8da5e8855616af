# lazy tie search per-phase cycles at 3 prebuilt levels (used via gpurun)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lazy
DDLO_TIE_PARTIAL_LEVELS=3 DDLO_LAZY_PROF=1 timeout -k 10 120 python -u tools/time_cov.py > gpurun_out/lazy/prof3.log 2>&1 || { tail -20 gpurun_out/lazy/prof3.log; exit 1; }
grep "\[lazy\]" gpurun_out/lazy/prof3.log | head -12
for L in 2 3; do
  DDLO_TIE_PARTIAL_LEVELS=$L timeout -k 10 300 python -u bench.py --no-cpu --no-sharded --no-gn --no-seg --steps 20 > gpurun_out/lazy/b_L$L.json 2>/dev/null || exit 1
  python -c "import json; d = json.load(open('gpurun_out/lazy/b_L$L.json')); print('L$L', 'batched', d['batched_s2s']['ms_per_pair'], d['batched_s2s']['ms_per_pair_morton_tie_order'], 'odom', d['odometry']['ms_per_frame'], d['odometry']['ms_per_frame_morton_tie_order'])"
done
