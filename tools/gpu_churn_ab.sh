# A/B of the batch workers' own hardware queues (own_queue_pool) bare and after context churn, in one call:
# the default library (own queues) and the `make dev` library with DDLO_BATCH_OWN_QUEUE=0 (pooled streams).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/churn_ab
mkdir -p $O
DEV=$GRAFT_REPO_ROOT/dynamic_direct_lidar_odometry_amd/_lib/dev/libddlo_gicp.so
for rep in 1 2; do
  for m in bare churn; do
    timeout -k 10 300 python3 tools/batch_leg_alone.py $m > $O/own_$m.log 2>&1 || { echo "OWN $m FAIL"; tail $O/own_$m.log; exit 1; }
    echo "own queues: $(grep "^$m" $O/own_$m.log)"
    DDLO_GICP_LIB=$DEV DDLO_BATCH_OWN_QUEUE=0 timeout -k 10 300 python3 tools/batch_leg_alone.py $m > $O/pool_$m.log 2>&1 || { echo "POOL $m FAIL"; tail $O/pool_$m.log; exit 1; }
    echo "pooled:     $(grep "^$m" $O/pool_$m.log)"
  done
done
