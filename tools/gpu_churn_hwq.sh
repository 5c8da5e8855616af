# The batch leg bare / after context churn with HIP's default 4 hardware queues per process and with 8
# (GPU_MAX_HW_QUEUES, read at HIP initialisation), in one call.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/churn_hwq
mkdir -p $O
for q in 4 8; do
  for m in bare churn; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 tools/batch_leg_alone.py $m > $O/q${q}_$m.log 2>&1 || { echo "Q$q $m FAIL"; tail $O/q${q}_$m.log; exit 1; }
    echo "hw queues $q: $(grep "^$m" $O/q${q}_$m.log)"
  done
done
