# frame-parallel S2S: tree on the worker's own stream vs its second stream (used via gpurun)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/batchstreams2
timeout -k 10 300 python3 -u tools/batch_streams.py 3 4 6 8 > gpurun_out/batchstreams2/a.txt 2> gpurun_out/batchstreams2/a.err || { cat gpurun_out/batchstreams2/a.txt; tail -20 gpurun_out/batchstreams2/a.err; exit 1; }
echo "aux stream"; cat gpurun_out/batchstreams2/a.txt
DDLO_NF_SAME_STREAM=1 timeout -k 10 300 python3 -u tools/batch_streams.py 3 4 6 8 > gpurun_out/batchstreams2/s.txt 2> gpurun_out/batchstreams2/s.err || { cat gpurun_out/batchstreams2/s.txt; tail -20 gpurun_out/batchstreams2/s.err; exit 1; }
echo "same stream"; cat gpurun_out/batchstreams2/s.txt
