# Full GPU pass (used via gpurun): GPU tests, PMC traffic of the linearize, bench, rocprof kernel stats.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_t_$c -o run -- python3 bench.py --no-cpu --no-sharded --no-batch --no-odom --no-gn --no-seg --steps 5 --warmup 1 > gpurun_out/pmc_t_$c.log 2>&1 || { echo "PMC pass $c failed"; tail -5 gpurun_out/pmc_t_$c.log; exit 1; }
done
python3 tools/pmc_traffic.py gpurun_out/pmc_t_FETCH_SIZE/run_counter_collection.csv gpurun_out/pmc_t_WRITE_SIZE/run_counter_collection.csv gpurun_out/traffic.json
DDLO_TRAFFIC_JSON=gpurun_out/traffic.json timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- python3 bench.py --no-cpu --no-sharded --no-batch --no-odom --no-gn --no-seg --steps 20 > gpurun_out/prof_bench.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof_bench.log; exit 1; }
python3 tools/profile_summary.py gpurun_out/prof_bench run > gpurun_out/prof_bench.md
echo ALL_OK
