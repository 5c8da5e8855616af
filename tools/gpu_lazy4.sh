# lazy tie search with LDS instructions in the window (used via gpurun)
cd $GRAFT_REPO_ROOT
O=gpurun_out/lazy4
mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_nftree.py -k "lazy or ties_lattice" > $O/nftree.log 2>&1 || { echo NFTREE_FAIL; tail -30 $O/nftree.log; exit 1; }
tail -1 $O/nftree.log
for L in 3 4 5; do
  DDLO_TIE_LAZY=1 DDLO_TIE_PARTIAL_LEVELS=$L timeout -k 10 120 python -u tools/time_cov.py > $O/t_L$L.log 2>&1 || { echo FAIL; tail -20 $O/t_L$L.log; exit 1; }
  echo "levels $L"; cat $O/t_L$L.log
done
DDLO_TIE_LAZY=1 DDLO_TIE_PARTIAL_LEVELS=4 DDLO_LAZY_PROF=1 timeout -k 10 120 python -u tools/time_cov.py > $O/prof_L4.log 2>&1 || exit 1
grep "\[lazy\]" $O/prof_L4.log | head -5 | cut -c1-330
