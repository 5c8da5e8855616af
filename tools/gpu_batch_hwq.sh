# frame-parallel S2S with more hardware queues per process (used via gpurun)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/hwq
export GPU_MAX_HW_QUEUES=16
for m in "lib" "lib ctx"; do
  timeout -k 10 300 python3 -u tools/batch_runtime.py $m > gpurun_out/hwq/o.txt 2> gpurun_out/hwq/o.err || { cat gpurun_out/hwq/o.txt; tail -20 gpurun_out/hwq/o.err; exit 1; }
  grep ms/pair gpurun_out/hwq/o.txt
done
timeout -k 10 300 python -u bench.py --no-cpu --no-sharded --no-gn --no-seg --steps 10 > gpurun_out/hwq/alone.json 2> gpurun_out/hwq/alone.err || { tail -20 gpurun_out/hwq/alone.err; exit 1; }
python3 -c "import json; d = json.load(open('gpurun_out/hwq/alone.json')); b = d['batched_s2s']; o = d['odometry']; print('bench', d['ms_per_step'], 'batch', b['ms_per_pair'], b['ms_per_pair_morton_tie_order'], 'odom', o['ms_per_frame'], o['ms_per_frame_morton_tie_order'])"
