# bench.py's batched leg (after the headline) at 3 / 4 / 6 workers (used via gpurun)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/benchstreams
for ns in 3 4 6; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-sharded --no-gn --no-odom --no-seg --steps 10 --batch-streams $ns > gpurun_out/benchstreams/b$ns.json 2> gpurun_out/benchstreams/b$ns.err || { tail -20 gpurun_out/benchstreams/b$ns.err; exit 1; }
  python3 -c "import json; b = json.load(open('gpurun_out/benchstreams/b$ns.json'))['batched_s2s']; print('streams $ns', b['ms_per_pair'], b['ms_per_pair_morton_tie_order'])"
done
