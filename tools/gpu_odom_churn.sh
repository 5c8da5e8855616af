# The odometry chain bare / after context churn, with 4 and 8 HIP hardware queues, in one call.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/odom_churn
mkdir -p $O
for q in 4 8; do
  for m in bare churn bare churn; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 tools/odom_churn.py $m > $O/q${q}_$m.log 2>&1 || { echo "Q$q $m FAIL"; tail $O/q${q}_$m.log; exit 1; }
    echo "hw queues $q: $(grep "^$m" $O/q${q}_$m.log)"
  done
done
