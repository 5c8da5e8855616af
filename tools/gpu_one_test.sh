cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_gicp.py -k "${TEST_K:-reused}" -x -q --timeout 200 --timeout-method thread 2>&1 | tail -15
