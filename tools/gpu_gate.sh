# gated partial tree in the batch workers: tests + worker sweep (used via gpurun)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/gate
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_nftree.py > gpurun_out/gate/t.txt 2>&1 || { tail -30 gpurun_out/gate/t.txt; exit 1; }
tail -2 gpurun_out/gate/t.txt
timeout -k 10 300 python3 -u tools/batch_streams.py 3 4 6 > gpurun_out/gate/s.txt 2> gpurun_out/gate/s.err || { cat gpurun_out/gate/s.txt; tail -20 gpurun_out/gate/s.err; exit 1; }
cat gpurun_out/gate/s.txt
