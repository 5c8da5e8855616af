cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && DDLO_TIE_DEBUG=1 timeout -k 10 200 python -u tools/probe_ties.py 2>&1 | grep ties
