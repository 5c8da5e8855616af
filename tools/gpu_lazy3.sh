# partial tree + lazy tie search timing without the profile printf (used via gpurun)
cd $GRAFT_REPO_ROOT
O=gpurun_out/lazy3
mkdir -p $O
for L in 2 4 6; do
  DDLO_TIE_LAZY=1 DDLO_TIE_PARTIAL_LEVELS=$L timeout -k 10 120 python -u tools/time_cov.py > $O/t_L$L.log 2>&1 || { echo FAIL; tail -20 $O/t_L$L.log; exit 1; }
  echo "levels $L"; cat $O/t_L$L.log
done
DDLO_TIE_LAZY=1 DDLO_TIE_PARTIAL_LEVELS=4 DDLO_NF_SAME_STREAM=1 timeout -k 10 120 python -u tools/time_cov.py > $O/t_same.log 2>&1 || exit 1
echo "levels 4 same stream"; cat $O/t_same.log
