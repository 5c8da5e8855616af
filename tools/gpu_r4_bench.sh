# the default bench on HEAD + smoke (used via gpurun)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d = json.load(open('$O/bench.json')); b = d['batched_s2s']; o = d['odometry']; print('cfg3', d['ms_per_step'], 'cpu', d['cpu_baseline']['value'], 'batch', b['ms_per_pair'], b['ms_per_pair_morton_tie_order'], b['streams_per_gpu'], 'odom', o['ms_per_frame'], o['ms_per_frame_morton_tie_order'])"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $O/smoke.log; exit 1; }
echo ALL_OK
