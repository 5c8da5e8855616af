# kernel traces of the frame-parallel S2S batch in both tie orders (used via gpurun)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/batchprof
for m in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/batchprof/p$m -o run --output-format csv -- python3 -u tools/batch_prof.py $m > gpurun_out/batchprof/o$m.txt 2>&1 || { tail -20 gpurun_out/batchprof/o$m.txt; exit 1; }
  grep "ms/pair" gpurun_out/batchprof/o$m.txt
done
