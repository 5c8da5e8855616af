cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
DDLO_GICP_LIB=ab/libS.so timeout -k 10 200 python -u tools/tail_sim.py
