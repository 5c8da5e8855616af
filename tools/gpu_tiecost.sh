# cfg3 / cfg2 cost of the correspondence tie detection by part (tie_scan 4; DDLO_TIE_AB bits: 2 no slice-merge
# records, 4 no winner-slice check; tie_scan 0: no scan records at all) (used via gpurun)
cd $GRAFT_REPO_ROOT
O=gpurun_out/tiecost
mkdir -p $O
for v in "4 0" "4 2" "4 4" "4 6" "0 0" "4 0"; do
  set -- $v
  DDLO_TIE_SCAN=$1 DDLO_TIE_AB=$2 timeout -k 10 200 python3 tools/ab_ties.py > $O/ab_$1_$2.log 2>&1 || { echo AB_FAIL; tail $O/ab_$1_$2.log; exit 1; }
  echo "scan $1 ab $2: $(grep 'cfg3 nanoflann' $O/ab_$1_$2.log | cut -c1-40) | $(grep 'cfg3 morton' $O/ab_$1_$2.log | cut -c1-40) | $(grep 'cfg2 nanoflann' $O/ab_$1_$2.log | cut -c1-40) | $(grep 'cfg2 morton' $O/ab_$1_$2.log | cut -c1-40)"
done
