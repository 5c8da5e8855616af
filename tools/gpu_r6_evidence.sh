# Round-6 evidence (used via gpurun): cfg3 PMC traffic + kernel trace of the headline (candidate cells),
# per-leg kernel traces and PMC passes (cfg2, cfg4, cfg5 stages), the default bench with the round's
# traffic figure, the slab table, smoke.  Outputs under gpurun_out/r06/ (raw traces deleted after their
# summaries: the copy-back limit is 64 MiB).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06
mkdir -p $O
HEAD="--no-cpu --no-sharded --no-batch --no-odom --no-gn --no-seg --no-walk"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$c -o run -- python3 bench.py $HEAD --steps 5 --warmup 1 > $O/pmc_$c.log 2>&1 || { echo "PMC pass $c failed"; tail -5 $O/pmc_$c.log; exit 1; }
done
python3 tools/pmc_traffic.py $O/pmc_FETCH_SIZE/run_counter_collection.csv $O/pmc_WRITE_SIZE/run_counter_collection.csv $O/traffic.json || exit 1
rm -rf $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python3 bench.py $HEAD --steps 100 > $O/prof_bench.log 2>&1 || { echo PROF_FAIL; tail -20 $O/prof_bench.log; exit 1; }
python3 tools/profile_summary.py $O/prof_bench run > $O/bench_summary.md
cp $O/prof_bench/run_kernel_stats.csv $O/bench_kernel_stats.csv
rm -rf $O/prof_bench
echo "headline traced"
for leg in cfg2 cfg4 cfg5; do
  n=5; [ $leg = cfg5 ] && n=24; [ $leg = cfg4 ] && n=12
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$leg -o run -- python3 tools/legs.py $leg $n > $O/prof_$leg.log 2>&1 || { echo "PROF $leg FAIL"; tail -20 $O/prof_$leg.log; exit 1; }
  python3 tools/profile_summary.py $O/prof_$leg run > $O/${leg}_summary.md
  rm -rf $O/prof_$leg
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${leg}_$c -o run -- python3 tools/legs.py $leg 3 > $O/pmc_${leg}_$c.log 2>&1 || { echo "PMC $leg $c failed"; tail -5 $O/pmc_${leg}_$c.log; exit 1; }
  done
  python3 tools/pmc_kernels.py $O/pmc_${leg}_FETCH_SIZE $O/pmc_${leg}_WRITE_SIZE > $O/${leg}_pmc_kernels.txt || exit 1
  rm -rf $O/pmc_${leg}_FETCH_SIZE $O/pmc_${leg}_WRITE_SIZE
  echo "$leg done"
done
DDLO_TRAFFIC_JSON=$O/traffic.json timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json | cut -c1-600
timeout -k 10 600 python -u tools/slab_cells_table.py 2 4 8 > $O/slab_cells_table.log 2>&1 || { echo SLAB_FAIL; tail -20 $O/slab_cells_table.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
echo ALL_OK
bash tools/gpu_odom_prof.sh > $O/odom_prof.txt 2>&1 || { echo ODOM_PROF_FAIL; tail $O/odom_prof.txt; exit 1; }
echo ODOM_PROF_OK
