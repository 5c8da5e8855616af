# bench.py's batched leg: stream history (used via gpurun)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/batchleg
for m in bare churn prelude_closed; do
  timeout -k 10 300 python3 -u tools/batch_leg_alone.py $m > gpurun_out/batchleg/$m.txt 2> gpurun_out/batchleg/$m.err || { cat gpurun_out/batchleg/$m.txt; tail -20 gpurun_out/batchleg/$m.err; exit 1; }
  tail -1 gpurun_out/batchleg/$m.txt
done
