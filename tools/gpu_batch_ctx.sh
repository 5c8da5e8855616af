# the batched leg alone vs after the other legs (used via gpurun)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/batchctx
timeout -k 10 300 python -u bench.py --no-cpu --no-sharded --no-gn --no-odom --no-seg --steps 10 > gpurun_out/batchctx/alone.json 2> gpurun_out/batchctx/alone.err || { tail -20 gpurun_out/batchctx/alone.err; exit 1; }
python3 -c "import json; b = json.load(open('gpurun_out/batchctx/alone.json'))['batched_s2s']; print('alone', b['ms_per_pair'], b['ms_per_pair_morton_tie_order'])"
timeout -k 10 300 python -u bench.py --no-cpu --no-odom --no-seg --steps 10 > gpurun_out/batchctx/after.json 2> gpurun_out/batchctx/after.err || { tail -20 gpurun_out/batchctx/after.err; exit 1; }
python3 -c "import json; b = json.load(open('gpurun_out/batchctx/after.json'))['batched_s2s']; print('after legs', b['ms_per_pair'], b['ms_per_pair_morton_tie_order'])"
