# Round 3: the whole GPU suite, every failure listed (used via gpurun).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 150 --timeout-method thread "$@" > gpurun_out/r3_all.log 2>&1
rc=$?
tail -40 gpurun_out/r3_all.log
exit $rc
