# Round 3: device nanoflann tree tests only (used via gpurun), all results.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_nftree.py tests/test_gpu_knn.py -v --timeout 150 --timeout-method thread "$@" > gpurun_out/r3_nf.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error|assert '" gpurun_out/r3_nf.log | tail -60
exit $rc
