# frame-parallel S2S under the lazy tie search's knobs (used via gpurun)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/batchknobs
timeout -k 10 400 python3 -u tools/batch_knobs.py > gpurun_out/batchknobs/o.txt 2> gpurun_out/batchknobs/o.err || { cat gpurun_out/batchknobs/o.txt; tail -20 gpurun_out/batchknobs/o.err; exit 1; }
cat gpurun_out/batchknobs/o.txt
