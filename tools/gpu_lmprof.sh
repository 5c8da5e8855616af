# Per-phase cycle counts of the LM step (s_memtime; `make lmprof` build) over the headline's aligns
# (tools/legs.py cfg3), then the cfg3 and cfg2 legs' timing with the product library.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
DDLO_GICP_LIB=$PWD/dynamic_direct_lidar_odometry_amd/_lib/lmprof/libddlo_gicp.so timeout -k 10 180 python3 tools/legs.py cfg3 20 > gpurun_out/lmprof.log 2>&1 || { tail gpurun_out/lmprof.log; exit 1; }
python3 - <<'PY'
import numpy as np
rows=[list(map(int,l.split()[1:])) for l in open('gpurun_out/lmprof.log') if l.startswith('lm_prof')]
a=np.array(rows)
print(len(a), 'steps; median cycles per phase (reduce, H/b/W12 table, trials, cost rows, wave-0 decisions + state):')
print(np.median(a[:,1:6],axis=0), 'total', np.median(a[:,1:6].sum(1)))
print('trial 0 (lambda, LDLT solve, so3 exp, measures + stores):', np.median(a[:,6:10],axis=0))
PY
