# partial tree + lazy tie search (used via gpurun): parity tests, per-phase profile, timing A/B
cd $GRAFT_REPO_ROOT
O=gpurun_out/lazy2
mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_nftree.py -k "lazy or ties_lattice" > $O/nftree.log 2>&1 || { echo NFTREE_FAIL; tail -30 $O/nftree.log; exit 1; }
tail -1 $O/nftree.log
for L in 4 6 8; do
  DDLO_TIE_LAZY=1 DDLO_TIE_PARTIAL_LEVELS=$L DDLO_LAZY_PROF=1 timeout -k 10 120 python -u tools/time_cov.py > $O/prof_L$L.log 2>&1 || { echo PROF_FAIL; tail -20 $O/prof_L$L.log; exit 1; }
  echo "levels $L"; grep "\[lazy\]" $O/prof_L$L.log | head -4 | cut -c1-330; tail -2 $O/prof_L$L.log
done
timeout -k 10 120 python -u tools/time_cov.py > $O/time_cov_tree.log 2>&1 || exit 1
echo tree; cat $O/time_cov_tree.log
