# The batch leg bare and after 10 created-and-destroyed contexts: a kernel trace of each
# (no counters), for the queue / stream mapping and each worker's busy time.  The summary is printed; the
# traces are deleted (too large to copy back).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/churn
mkdir -p $O
for m in bare churn bare churn; do
  timeout -k 10 300 python3 tools/batch_leg_alone.py $m > $O/plain_$m.log 2>&1 || { echo "PLAIN $m FAIL"; tail $O/plain_$m.log; exit 1; }
  grep "^$m" $O/plain_$m.log
done
[ -n "$CHURN_NO_TRACE" ] && exit 0
for m in bare churn; do
  rm -rf $O/tr_$m
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$m -o run -- python3 tools/batch_leg_alone.py $m > $O/tr_$m.log 2>&1 || { echo "TRACE $m FAIL"; tail $O/tr_$m.log; exit 1; }
  grep "^$m" $O/tr_$m.log
done
python3 tools/churn_compare.py $O/tr_bare $O/tr_churn > $O/compare.md
rm -rf $O/tr_bare $O/tr_churn
cat $O/compare.md
