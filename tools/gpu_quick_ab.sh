# quick A/B: tie mode 3 cost parts on cfg3/cfg2 (DDLO_TIE_AB bits), used via gpurun
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for ab in 0 1 2 4 7; do
  DDLO_TIE_AB=$ab DDLO_TIE_SCAN=3 timeout -k 10 200 python3 tools/ab_ties.py > gpurun_out/ab_tie_ab$ab.log 2>&1 || exit 1
done
