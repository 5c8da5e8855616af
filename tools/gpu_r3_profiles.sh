# Round-3 evidence (used via gpurun): PMC passes (FETCH_SIZE, WRITE_SIZE) of the cfg3 linearize,
# the rocprofv3 kernel trace + stats of the cfg3 bench, the summary.  Outputs under gpurun_out/r03/.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/r03/pmc_$c -o run -- python3 bench.py --no-cpu --no-sharded --no-batch --no-odom --no-gn --no-seg --steps 5 --warmup 1 > gpurun_out/r03/pmc_$c.log 2>&1 || { echo "PMC pass $c failed"; tail -5 gpurun_out/r03/pmc_$c.log; exit 1; }
done
python3 tools/pmc_traffic.py gpurun_out/r03/pmc_FETCH_SIZE/run_counter_collection.csv gpurun_out/r03/pmc_WRITE_SIZE/run_counter_collection.csv gpurun_out/r03/traffic.json || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03/prof_bench -o run -- python3 bench.py --no-cpu --no-sharded --no-batch --no-odom --no-gn --no-seg --steps 20 > gpurun_out/r03/prof_bench.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/r03/prof_bench.log; exit 1; }
python3 tools/profile_summary.py gpurun_out/r03/prof_bench run > gpurun_out/r03/bench_summary.md
echo ALL_OK
