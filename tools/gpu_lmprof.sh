cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/time_cfg3.py || exit 1
DDLO_GICP_LIB=$PWD/ab/libL.so timeout -k 10 120 python3 tools/time_cfg3.py > gpurun_out/lmprof.log 2>&1 || { tail gpurun_out/lmprof.log; exit 1; }
python3 - <<'PY'
import numpy as np
rows=[list(map(int,l.split()[1:])) for l in open('gpurun_out/lmprof.log') if l.startswith('lm_prof')]
a=np.array(rows)
print(len(a), 'steps; median cycles per phase (reduce, normal-eq+W12, lambda0+trial LDLT/so3, rows+rho, tid0 decisions):')
print(np.median(a[:,1:],axis=0))
print(open('gpurun_out/lmprof.log').read().splitlines()[-1])
PY
