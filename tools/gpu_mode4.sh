# tie_scan 4 (key atomic return instead of the mirrored key) and the faster lazy tie search (used via gpurun):
# tie tests under mode 4, cfg3/cfg2 A/B of modes 3 / 4, then the lazy A/B script.
cd $GRAFT_REPO_ROOT
O=gpurun_out/mode4
mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
DDLO_TIE_SCAN=4 timeout -k 10 600 $T tests/test_gpu_ties.py tests/test_gpu_shard.py tests/test_gpu_gicp.py > $O/tests4.log 2>&1 || { echo TESTS4_FAIL; tail -30 $O/tests4.log; exit 1; }
tail -1 $O/tests4.log
for m in 3 4 3 4; do
  DDLO_TIE_SCAN=$m timeout -k 10 200 python3 tools/ab_ties.py > $O/ab_mode$m.log 2>&1 || { echo AB_FAIL; tail $O/ab_mode$m.log; exit 1; }
  echo "mode $m"; tail -4 $O/ab_mode$m.log
done
bash tools/gpu_lazy.sh
for s in 3 5 8; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-sharded --no-gn --no-seg --no-odom --steps 20 --batch-streams $s > $O/batch_s$s.json 2> $O/batch_s$s.err || { echo BATCH_FAIL; tail $O/batch_s$s.err; exit 1; }
  python -c "import json; d = json.load(open('$O/batch_s$s.json')); print('streams $s', {k: v for k, v in d['batched_s2s'].items() if 'ms' in k})"
done
