# frame-parallel S2S: worker streams sweep (used via gpurun)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/batchstreams
timeout -k 10 400 python3 -u tools/batch_streams.py 3 4 6 8 > gpurun_out/batchstreams/o.txt 2> gpurun_out/batchstreams/o.err || { cat gpurun_out/batchstreams/o.txt; tail -20 gpurun_out/batchstreams/o.err; exit 1; }
cat gpurun_out/batchstreams/o.txt
