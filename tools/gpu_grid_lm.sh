# cfg3 probe (cells on/off) + per-phase LM-step cycles (make lmprof build)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/grid_probe.py --aligns 200 > gpurun_out/grid_probe.log 2>&1 || { echo PROBE_FAIL; tail gpurun_out/grid_probe.log; exit 1; }
cut -c1-300 gpurun_out/grid_probe.log
DDLO_GICP_LIB=$PWD/dynamic_direct_lidar_odometry_amd/_lib/lmprof/libddlo_gicp.so timeout -k 10 200 python3 tools/grid_probe.py --aligns 20 > gpurun_out/lmprof.log 2>&1 || { tail gpurun_out/lmprof.log; exit 1; }
python3 - <<'PY'
import numpy as np
rows=[list(map(int,l.split()[1:])) for l in open('gpurun_out/lmprof.log') if l.startswith('lm_prof')]
a=np.array(rows)
print(len(a), "steps; median cycles per phase (reduce, normal-eq+W12, lambda0+trial LDLT/so3, rows+rho, tid0 decisions):")
print(np.median(a[:,1:],axis=0))
PY
