# lazy tie search per-phase cycles (used via gpurun)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lazy
DDLO_TIE_LAZY=1 DDLO_LAZY_PROF=1 timeout -k 10 120 python -u tools/time_cov.py > gpurun_out/lazy/prof.log 2>&1 || { tail -20 gpurun_out/lazy/prof.log; exit 1; }
grep "\[lazy\]" gpurun_out/lazy/prof.log | head -12
tail -2 gpurun_out/lazy/prof.log
