# A/B/C of library builds in ab/ (used via gpurun): GPU tests on the in-tree
# library first, then alternating cfg 3 benches of each build given in LIBS
# (default "B C"), then knob cases (AB_CASES file) on the last build.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_abc.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_abc.log; exit 1; }
  tail -2 gpurun_out/pytest_abc.log
fi
LIBS=${LIBS:-"B C"}
for r in 1 2 3; do
  for L in $LIBS; do
    DDLO_GICP_LIB=ab/lib$L.so timeout -k 10 150 python -u bench.py --no-cpu --no-sharded --no-batch --no-odom --no-seg --steps 200 > gpurun_out/ab_$L.json 2> gpurun_out/ab_$L.err || { echo "AB_FAIL $L"; tail -5 gpurun_out/ab_$L.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_$L.json')); v=d.get('cfg3_varied_guesses',{}); print('$L', 'ms/scan', d['ms_per_step'], 'lin us', d['roofline']['avg_launch_us'], 'varied', v.get('ms_per_scan'), 'cfg2 ms', d.get('s2s_gn', {}).get('ms_per_align'))"
  done
done
LAST=${LIBS##* }
if [ -n "$AB_CASES" ]; then
  while read -r line; do
    [ -z "$line" ] && continue
    env DDLO_GICP_LIB=ab/lib$LAST.so $line timeout -k 10 150 python -u bench.py --no-cpu --no-sharded --no-batch --no-odom --no-seg --steps 200 > gpurun_out/abk.json 2> gpurun_out/abk.err || { echo "ABK_FAIL $line"; tail -5 gpurun_out/abk.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/abk.json')); v=d.get('cfg3_varied_guesses',{}); print(sys.argv[1], 'ms/scan', d['ms_per_step'], 'lin us', d['roofline']['avg_launch_us'], 'varied', v.get('ms_per_scan'), 'cfg2 ms', d.get('s2s_gn', {}).get('ms_per_align'))" "$line"
  done < "$AB_CASES"
fi
if [ -n "$TRACE" ]; then
  DDLO_GICP_LIB=ab/lib$LAST.so timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abc_trace -o run -- python3 bench.py --no-cpu --no-sharded --no-batch --no-odom --no-gn --no-seg --steps 40 > gpurun_out/abc_trace.log 2>&1 || { echo TRACE_FAIL; tail -5 gpurun_out/abc_trace.log; exit 1; }
  python3 tools/profile_summary.py gpurun_out/abc_trace run | tail -12
fi
