# Round-4 closing evidence (used via gpurun): GPU tests, the batched leg's stream-history check, the default bench, smoke
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { echo GPUTEST_FAIL; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
for m in bare churn; do
  timeout -k 10 300 python3 -u tools/batch_leg_alone.py $m > $O/leg_$m.txt 2> $O/leg_$m.err || { cat $O/leg_$m.txt; tail -20 $O/leg_$m.err; exit 1; }
  tail -1 $O/leg_$m.txt
done
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d = json.load(open('$O/bench.json')); b = d['batched_s2s']; o = d['odometry']; print('cfg3', d['ms_per_step'], 'batch', b['ms_per_pair'], b['ms_per_pair_morton_tie_order'], 'odom', o['ms_per_frame'], o['ms_per_frame_morton_tie_order'])"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $O/smoke.log; exit 1; }
echo ALL_OK
