# partial-tree depth sweep of the lazy tie search (used via gpurun): covariance timing and the cfg 5 legs
cd $GRAFT_REPO_ROOT
O=gpurun_out/levels
mkdir -p $O
for L in 3 4 5 6; do
  DDLO_TIE_PARTIAL_LEVELS=$L timeout -k 10 120 python -u tools/time_cov.py > $O/t_L$L.log 2>&1 || { echo FAIL; tail -20 $O/t_L$L.log; exit 1; }
  DDLO_TIE_PARTIAL_LEVELS=$L timeout -k 10 300 python -u bench.py --no-cpu --no-sharded --no-gn --no-seg --steps 20 > $O/b_L$L.json 2> $O/b_L$L.err || { echo BENCH_FAIL; tail -20 $O/b_L$L.err; exit 1; }
  python - <<PY
import json
d = json.load(open("$O/b_L$L.json"))
print("L$L", open("$O/t_L$L.log").read().strip().replace("\n", " "), "batched", d["batched_s2s"]["ms_per_pair"], d["batched_s2s"]["ms_per_pair_morton_tie_order"], "odom", d["odometry"]["ms_per_frame"], d["odometry"]["ms_per_frame_morton_tie_order"])
PY
done
