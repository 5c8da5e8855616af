cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_grid.py tests/test_gpu_ties.py -x -q --timeout 300 --timeout-method thread > gpurun_out/quick_tests.log 2>&1; rc=$?
tail -2 gpurun_out/quick_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/quick_tests.log | head -20; exit 1; }
for v in 0 1 0 1; do
  DDLO_GRID_FUSED=$v timeout -k 10 120 python -u tools/grid_probe.py --aligns 300 2>&1 | grep "^grid" | python3 -c "import sys,json; l=sys.stdin.read(); d=json.loads(l[l.index('{'):]); print('GRID_FUSED=$v', round(d['ms_per_scan'],4), 'dev', round(d['device_ms_median'],4), 'lin', round(d['linearize_us_per_iter'],2))" || exit 1
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_multiproc.py -x -q --timeout 300 --timeout-method thread > gpurun_out/multiproc.log 2>&1; rc=$?
tail -3 gpurun_out/multiproc.log
exit $rc
