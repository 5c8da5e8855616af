# HBM-side traffic of the linearize kernels on the bench workload (used via gpurun):
# one rocprofv3 --pmc pass per TCC counter group (FETCH_SIZE and WRITE_SIZE do not fit one pass),
# no tracing domains combined with --pmc.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_t_$c -o run -- python3 bench.py --no-cpu --no-sharded --steps 5 --warmup 1 > gpurun_out/pmc_t_$c.log 2>&1 || { echo "pass $c failed"; tail -5 gpurun_out/pmc_t_$c.log; exit 1; }
done
python3 tools/pmc_traffic.py gpurun_out/pmc_t_FETCH_SIZE/run_counter_collection.csv gpurun_out/pmc_t_WRITE_SIZE/run_counter_collection.csv
