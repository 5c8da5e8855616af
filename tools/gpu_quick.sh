# correctness (GICP core, ties, cells, cfg3 size) + cfg3 probe + LM phases
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gicp.py tests/test_gpu_ties.py tests/test_gpu_grid.py tests/test_gpu_large.py -x -q --timeout 300 --timeout-method thread > gpurun_out/quick_tests.log 2>&1; rc=$?
tail -3 gpurun_out/quick_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/quick_tests.log | head -20; exit 1; }
bash tools/gpu_grid_lm.sh
