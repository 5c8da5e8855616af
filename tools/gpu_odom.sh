# odometry driver tests (used via gpurun)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_odom.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_odom.log 2>&1; rc=$?
tail -40 gpurun_out/pytest_odom.log
exit $rc
