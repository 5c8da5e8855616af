# Round-4 final evidence on HEAD (used via gpurun): the whole GPU test suite, the default bench, cfg3 and cfg5
# kernel traces, smoke.  Outputs under gpurun_out/r04f/.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { echo GPUTEST_FAIL; tail -30 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python3 bench.py --no-cpu --no-sharded --no-batch --no-odom --no-gn --no-seg --steps 100 > $O/prof_bench.log 2>&1 || { echo PROF_FAIL; tail -20 $O/prof_bench.log; exit 1; }
python3 tools/profile_summary.py $O/prof_bench run > $O/bench_summary.md
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cfg5 -o run -- python3 tools/legs.py cfg5 24 > $O/prof_cfg5.log 2>&1 || { echo PROF5_FAIL; tail -20 $O/prof_cfg5.log; exit 1; }
python3 tools/profile_summary.py $O/prof_cfg5 run > $O/cfg5_summary.md
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_batch -o run -- python3 tools/batch_prof.py 1 > $O/prof_batch.log 2>&1 || { echo PROFB_FAIL; tail -20 $O/prof_batch.log; exit 1; }
python3 tools/profile_summary.py $O/prof_batch run > $O/batch_summary.md
timeout -k 10 120 python -u tools/time_cov.py > $O/time_cov.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
cat $O/time_cov.log
echo ALL_OK
