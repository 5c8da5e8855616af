cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for n in 2 3 4 2 3 4; do
  timeout -k 10 200 python -u bench.py --no-cpu --no-sharded --no-gn --no-seg --no-odom --steps 3 --batch-streams $n > gpurun_out/bs.json 2> gpurun_out/bs.err || { echo FAIL $n; tail -3 gpurun_out/bs.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/bs.json')); print('streams', sys.argv[1], 'ms/pair', d['batched_s2s']['ms_per_pair'])" $n
done
