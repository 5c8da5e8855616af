# Round-4 evidence on HEAD (used via gpurun): cfg3 PMC traffic + kernel trace, the default bench (all legs,
# CPU thread sweep), per-leg kernel traces and PMC passes (cfg2, cfg4, cfg5 stages), smoke.
# Outputs under gpurun_out/r04/.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04
mkdir -p $O
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$c -o run -- python3 bench.py --no-cpu --no-sharded --no-batch --no-odom --no-gn --no-seg --steps 5 --warmup 1 > $O/pmc_$c.log 2>&1 || { echo "PMC pass $c failed"; tail -5 $O/pmc_$c.log; exit 1; }
done
python3 tools/pmc_traffic.py $O/pmc_FETCH_SIZE/run_counter_collection.csv $O/pmc_WRITE_SIZE/run_counter_collection.csv $O/traffic.json > /dev/null || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python3 bench.py --no-cpu --no-sharded --no-batch --no-odom --no-gn --no-seg --steps 100 > $O/prof_bench.log 2>&1 || { echo PROF_FAIL; tail -20 $O/prof_bench.log; exit 1; }
python3 tools/profile_summary.py $O/prof_bench run > $O/bench_summary.md
for leg in cfg2 cfg4 cfg5; do
  n=5; [ $leg = cfg5 ] && n=24
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$leg -o run -- python3 tools/legs.py $leg $n > $O/prof_$leg.log 2>&1 || { echo "PROF $leg FAIL"; tail -20 $O/prof_$leg.log; exit 1; }
  python3 tools/profile_summary.py $O/prof_$leg run > $O/${leg}_summary.md
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${leg}_$c -o run -- python3 tools/legs.py $leg 3 > $O/pmc_${leg}_$c.log 2>&1 || { echo "PMC $leg $c failed"; tail -5 $O/pmc_${leg}_$c.log; exit 1; }
  done
  python3 tools/pmc_kernels.py $O/pmc_${leg}_FETCH_SIZE $O/pmc_${leg}_WRITE_SIZE > $O/${leg}_pmc_kernels.txt || exit 1
done
DDLO_TRAFFIC_JSON=$O/traffic.json timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python -u -m pytest -s -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py -k slab > $O/slab_table.log 2>&1 || { echo SLAB_FAIL; tail -20 $O/slab_table.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
echo ALL_OK
