# A/B of two builds of the library (used via gpurun): ab/libA.so vs ab/libB.so,
# alternating, cfg 3 only (plus the varied-guess leg); then a kernel trace of B.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2 3; do
  for L in A B; do
    DDLO_GICP_LIB=ab/lib$L.so timeout -k 10 150 python -u bench.py --no-cpu --no-sharded --no-batch --no-odom --no-gn --no-seg --steps 200 "$@" > gpurun_out/ab_$L.json 2> gpurun_out/ab_$L.err || { echo "AB_FAIL $L"; tail -5 gpurun_out/ab_$L.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_$L.json')); v=d.get('cfg3_varied_guesses',{}); print('$L', 'ms/scan', d['ms_per_step'], 'lin us', d['roofline']['avg_launch_us'], 'varied', v.get('ms_per_scan'))"
  done
done
DDLO_GICP_LIB=ab/libB.so timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab_trace -o run -- python3 bench.py --no-cpu --no-sharded --no-batch --no-odom --no-gn --no-seg --steps 40 > gpurun_out/ab_trace.log 2>&1 || { echo TRACE_FAIL; tail -5 gpurun_out/ab_trace.log; exit 1; }
python3 tools/trace_gaps.py gpurun_out/ab_trace/run_kernel_trace.csv
# knob cases for lib B (tools/ab_cases.txt format), if a case file is given in AB_CASES
if [ -n "$AB_CASES" ]; then
  while read -r line; do
    [ -z "$line" ] && continue
    env DDLO_GICP_LIB=ab/libB.so $line timeout -k 10 150 python -u bench.py --no-cpu --no-sharded --no-batch --no-odom --no-seg --steps 200 > gpurun_out/abk.json 2> gpurun_out/abk.err || { echo "ABK_FAIL $line"; tail -5 gpurun_out/abk.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/abk.json')); v=d.get('cfg3_varied_guesses',{}); print(sys.argv[1], 'ms/scan', d['ms_per_step'], 'lin us', d['roofline']['avg_launch_us'], 'varied', v.get('ms_per_scan'), 'cfg2 ms', d.get('s2s_gn', {}).get('ms_per_align'))" "$line"
  done < "$AB_CASES"
fi
