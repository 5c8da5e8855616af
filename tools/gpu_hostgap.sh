cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for L in A B; do DDLO_GICP_LIB=ab/lib$L.so timeout -k 10 120 python -u tools/host_gap.py || exit 1; done
DDLO_SPIN_WAIT=1 DDLO_GICP_LIB=ab/libB.so timeout -k 10 120 python -u tools/host_gap.py || exit 1
DDLO_GICP_LIB=ab/libA.so timeout -k 10 120 python -u tools/host_gap.py || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_b.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_b.log; exit $rc
