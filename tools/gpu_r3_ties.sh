# Round 3: device nanoflann tree + tie resolution tests, then the whole GPU suite (used via gpurun).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_nftree.py tests/test_gpu_knn.py -x -v --timeout 150 --timeout-method thread > gpurun_out/r3_ties.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error" gpurun_out/r3_ties.log | tail -40
[ $rc -eq 0 ] || { tail -60 gpurun_out/r3_ties.log; exit $rc; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread "$@" > gpurun_out/r3_all.log 2>&1
rc=$?
tail -25 gpurun_out/r3_all.log
exit $rc
