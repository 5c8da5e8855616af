# The odometry chain alone in fresh processes with different histories (tools/odom_churn.py modes).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for m in bare cfg3build cfg3 alloc bare cfg3; do
  timeout -k 10 300 python -u tools/odom_churn.py $m 2> gpurun_out/odom_churn_$m.err || { echo "FAIL $m"; tail gpurun_out/odom_churn_$m.err; exit 1; }
done
