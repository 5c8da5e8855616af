cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_grid.py tests/test_gpu_shard.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/grid_tests.log 2>&1; echo "pytest rc $?" >> gpurun_out/grid_tests.log
tail -3 gpurun_out/grid_tests.log
timeout -k 10 300 python -u tools/grid_probe.py --aligns 100 > gpurun_out/grid_probe.log 2>&1 || { echo PROBE_FAIL; tail gpurun_out/grid_probe.log; exit 1; }
cat gpurun_out/grid_probe.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof_grid; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_grid -o run -- python3 tools/grid_probe.py --aligns 30 > gpurun_out/prof_grid.log 2>&1; echo prof rc $?
