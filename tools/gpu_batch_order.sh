# host-page state vs. the frame-parallel S2S leg (used via gpurun)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/batchorder
timeout -k 10 300 python -u tools/batch_order.py > gpurun_out/batchorder/o.txt 2> gpurun_out/batchorder/o.err || { tail -20 gpurun_out/batchorder/o.err; exit 1; }
cat gpurun_out/batchorder/o.txt
