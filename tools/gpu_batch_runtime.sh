# frame-parallel S2S: one stream per worker, with and without an extra live ctx (used via gpurun)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/runtime
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_batch.py > gpurun_out/runtime/t.txt 2>&1 || { tail -30 gpurun_out/runtime/t.txt; exit 1; }
tail -1 gpurun_out/runtime/t.txt
for m in "lib" "lib ctx"; do
  timeout -k 10 300 python3 -u tools/batch_runtime.py $m > gpurun_out/runtime/o.txt 2> gpurun_out/runtime/o.err || { cat gpurun_out/runtime/o.txt; tail -20 gpurun_out/runtime/o.err; exit 1; }
  grep ms/pair gpurun_out/runtime/o.txt
done
timeout -k 10 300 python -u bench.py --no-cpu --no-sharded --no-gn --no-odom --no-seg --steps 10 > gpurun_out/runtime/alone.json 2> gpurun_out/runtime/alone.err || { tail -20 gpurun_out/runtime/alone.err; exit 1; }
python3 -c "import json; b = json.load(open('gpurun_out/runtime/alone.json'))['batched_s2s']; print('bench alone', b['ms_per_pair'], b['ms_per_pair_morton_tie_order'])"
